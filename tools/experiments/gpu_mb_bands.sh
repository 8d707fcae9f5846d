set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_mb.log 2>&1 || { tail -30 gpurun_out/pytest_mb.log; exit 1; }
tail -3 gpurun_out/pytest_mb.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_mb.log 2>&1 || { tail -20 gpurun_out/bench_mb.log; exit 1; }
tail -1 gpurun_out/bench_mb.log
MCS_MB_BANDS=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-paste-ref > gpurun_out/bench_mb0.log 2>&1 && tail -1 gpurun_out/bench_mb0.log
