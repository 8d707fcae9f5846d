# Round 5: same-box multi-band A/B (C2 and C4 multi-band lines only) of main against the
# variants given as arguments, alternating twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
RIG=chain BLENDS="multiband" bash tools/gpu_var_bench.sh main "$@" || exit 1
RIG=cylinder BLENDS="multiband" bash tools/gpu_var_bench.sh main "$@" || exit 1
