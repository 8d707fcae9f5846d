# Round 6: per-kernel durations of the C3 resident estimate+stitch run (rocprofv3 --stats) for
# main / variants/r06pre.so / variants/orb32.so, then resident lines alternating three times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
for v in main r06pre orb32; do
  if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/orbt_$v" -o run -- python3 "$R/tools/estimate_bench.py" --stitch --pipelined --overlap --resident --depth 4 --steps 200 --warmup 10 --no-cpu-baseline > "$R/gpurun_out/orbt_$v.log" 2>&1) || { tail -20 "$R/gpurun_out/orbt_$v.log"; exit 1; }
  echo "== $v"; grep -h "mcs_orb_level\|mcs_direct\|mcs_orb_pyramid\|mcs_orb_describe" "$R"/gpurun_out/orbt_$v/run_kernel_stats.csv | cut -d, -f1-4
done
for i in 1 2 3; do
  for v in main r06pre orb32; do
    if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
    timeout -k 10 200 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth 4 --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/orb_res_$v.log 2>&1 || { tail -20 gpurun_out/orb_res_$v.log; exit 1; }
    echo "$v resident $(tail -1 gpurun_out/orb_res_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['max_abs_diff_vs_cpu_render'])")"
  done
done
