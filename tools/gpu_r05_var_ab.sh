# Round 5: full -m gpu suite on this build, then same-box bench A/B of this build (main) against
# the variants named as arguments (variants/<name>.so): C2 paste + multi-band, C4 seam +
# multi-band, alternating twice (tools/gpu_var_bench.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
RIG=chain BLENDS="none multiband" bash tools/gpu_var_bench.sh main "$@" || exit 1
RIG=cylinder BLENDS="seam multiband" bash tools/gpu_var_bench.sh main "$@" || exit 1
