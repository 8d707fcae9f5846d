# Round 6: C3 A/B of the main build against variants/$1.so: GPU ORB / estimate / RANSAC tests on main,
# per-kernel times of the C3 serial run (rocprofv3 --stats) for both, then C3 resident estimate +
# stitch lines alternating three times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"; V=$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_estimate.py tests/test_gpu_ransac.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_c3ab.log 2>&1 || { tail -30 gpurun_out/pytest_c3ab.log; exit 1; }
tail -1 gpurun_out/pytest_c3ab.log
for v in main $V; do
  if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/c3t_$v" -o run -- python3 "$R/tools/estimate_bench.py" --stitch --steps 60 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/c3t_$v.log" 2>&1) || { tail -20 "$R/gpurun_out/c3t_$v.log"; exit 1; }
  echo "== $v"; head -8 "$R"/gpurun_out/c3t_$v/run_kernel_stats.csv | tail -7 | cut -d, -f1-4
done
for i in 1 2 3; do
  for v in main $V; do
    if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
    timeout -k 10 200 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth 4 --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/c3ab_$v.log 2>&1 || { tail -20 gpurun_out/c3ab_$v.log; exit 1; }
    echo "$v resident $(tail -1 gpurun_out/c3ab_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['max_abs_diff_vs_cpu_render'])")"
  done
done
