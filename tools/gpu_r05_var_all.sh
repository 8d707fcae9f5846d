# Round 5: same-box bench A/B (no tests) of main against the variants given as arguments:
# C2 paste + multi-band, C4 seam + multi-band, alternating twice (tools/gpu_var_bench.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
RIG=chain BLENDS="none multiband" bash tools/gpu_var_bench.sh main "$@" || exit 1
RIG=cylinder BLENDS="seam multiband" bash tools/gpu_var_bench.sh main "$@" || exit 1
