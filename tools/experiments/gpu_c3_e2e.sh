# C3 end to end: estimate tests + the estimate -> stitch bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_estimate.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_est.log 2>&1 || { tail -40 gpurun_out/pytest_est.log; exit 1; }
tail -2 gpurun_out/pytest_est.log
timeout -k 10 300 python tools/estimate_bench.py --stitch --steps 100 --warmup 10 > gpurun_out/c3_stitch.json 2> gpurun_out/c3_stitch.err || { tail -20 gpurun_out/c3_stitch.err; exit 1; }
cat gpurun_out/c3_stitch.json
