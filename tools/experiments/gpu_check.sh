set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
nproc > gpurun_out/nproc.txt; lscpu | grep -i "model name" >> gpurun_out/nproc.txt || true
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 && \
cd "$GRAFT_REPO_ROOT" && timeout -k 10 300 python tools/sweep.py > gpurun_out/sweep.log 2>&1
