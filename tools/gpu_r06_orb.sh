# Round 6: ORB level kernel -- dword staging of interior tiles (main) vs the byte staging
# (variants/r06pre.so) vs main with 64 x 32 tiles (variants/orb32.so).  ORB / rig GPU tests on
# main, then C3 estimation-only and resident estimate+stitch lines per library, alternating twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_estimate.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_orb6.log 2>&1 || { tail -30 gpurun_out/pytest_orb6.log; exit 1; }
tail -1 gpurun_out/pytest_orb6.log
for i in 1 2; do
  for v in main r06pre orb32; do
    if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
    timeout -k 10 200 python tools/estimate_bench.py --pinned --steps 200 --warmup 10 > gpurun_out/orb_est_$v.log 2>&1 || { tail -20 gpurun_out/orb_est_$v.log; exit 1; }
    timeout -k 10 200 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth 4 --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/orb_res_$v.log 2>&1 || { tail -20 gpurun_out/orb_res_$v.log; exit 1; }
    e=$(tail -1 gpurun_out/orb_est_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('stage_ms_per_capture'))")
    r=$(tail -1 gpurun_out/orb_res_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['max_abs_diff_vs_cpu_render'], d['max_reproj_err_px_vs_truth'])")
    echo "$v estimate $e | resident $r"
  done
done
