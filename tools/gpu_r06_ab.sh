# Round 6: the multi-band sweep -- blend / cylinder / seam / stream GPU tests on this build, then a
# same-box bench A/B of this build (main) against variants/<name>.so (C2 paste + multi-band, C4
# seam + multi-band, alternating twice).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py tests/test_gpu_seam.py tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sweep.log 2>&1 || { tail -30 gpurun_out/pytest_sweep.log; exit 1; }
tail -1 gpurun_out/pytest_sweep.log
RIG=chain BLENDS="none multiband" bash tools/gpu_var_bench.sh main "$@" || exit 1
RIG=cylinder BLENDS="seam multiband" bash tools/gpu_var_bench.sh main "$@" || exit 1
