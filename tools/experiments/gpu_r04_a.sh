# Round 4 session start: full -m gpu suite on the knob-stripped tree, then the mosaic store-form
# A/B (three dword nt stores = main, one dwordx3 nt = x3nt, one dwordx3 plain = x3).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r04a.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r04a.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r04a.log
bash tools/gpu_var_bench.sh main x3nt x3 > gpurun_out/ab_store.txt 2>&1 || { cat gpurun_out/ab_store.txt; exit 1; }
cat gpurun_out/ab_store.txt
