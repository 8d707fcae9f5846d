# Round 6: describe_geo's stage parameters by scalar loads (a wave-uniform loop over the wave's
# stages) -- the direct stitch and the prepare kernel.  GPU parity / blend / cylinder / estimate
# tests on main, then the direct kernel's standalone time (C3 serial run, rocprofv3 --stats) and
# C3 resident lines for main vs variants/pre_direct.so, alternating three times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blend.py tests/test_gpu_cylinder.py tests/test_gpu_estimate.py tests/test_gpu_remap.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_direct.log 2>&1 || { tail -30 gpurun_out/pytest_direct.log; exit 1; }
tail -1 gpurun_out/pytest_direct.log
for v in main pre_direct; do
  if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/dtr_$v" -o run -- python3 "$R/tools/estimate_bench.py" --stitch --steps 60 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/dtr_$v.log" 2>&1) || { tail -20 "$R/gpurun_out/dtr_$v.log"; exit 1; }
  echo "== $v"; grep -h "mcs_direct\|mcs_orb_level" "$R"/gpurun_out/dtr_$v/run_kernel_stats.csv | cut -d, -f1-4,6,7
done
for i in 1 2 3; do
  for v in main pre_direct; do
    if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
    timeout -k 10 200 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth 4 --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/dr_$v.log 2>&1 || { tail -20 gpurun_out/dr_$v.log; exit 1; }
    echo "$v resident $(tail -1 gpurun_out/dr_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['max_abs_diff_vs_cpu_render'])")"
  done
done
