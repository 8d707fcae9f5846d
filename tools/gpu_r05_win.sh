# Round 5: the window-DMA streaming loop (main) -- full GPU suite, then same-box A/B of the
# paste and multi-band lines (C2 and C4) against the variants given as arguments, alternating twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_win.log 2>&1 || { tail -40 gpurun_out/pytest_win.log; exit 1; }
tail -1 gpurun_out/pytest_win.log
RIG=chain BLENDS="none multiband" bash tools/gpu_var_bench.sh main "$@" || exit 1
RIG=cylinder BLENDS="multiband" bash tools/gpu_var_bench.sh main "$@" || exit 1
