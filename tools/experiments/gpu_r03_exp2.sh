# Round 3 experiment 2: the compact 4-byte pixel descriptors -- the full -m gpu suite on the new
# build, then same-box A/B bench lines against the 12-byte-table build (variants/tables.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
BLENDS="none multiband" bash tools/gpu_var_bench.sh main tables
