# Round 5: streaming-block LDS budget A/B on the window-DMA kernel (paste + multi-band, C2 and
# C4), main against the variants given, alternating twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
RIG=chain BLENDS="none multiband" bash tools/gpu_var_bench.sh main "$@" || exit 1
RIG=cylinder BLENDS="multiband" bash tools/gpu_var_bench.sh main "$@" || exit 1
