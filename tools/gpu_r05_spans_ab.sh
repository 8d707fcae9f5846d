set -o pipefail
cd "$GRAFT_REPO_ROOT"
RIG=cylinder BLENDS="seam multiband" bash tools/gpu_var_bench.sh main boxspan || exit 1
RIG=chain BLENDS="none multiband" bash tools/gpu_var_bench.sh main boxspan || exit 1
