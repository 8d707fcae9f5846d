# Round 5: blend / band GPU tests on the main library, then the multi-band A/B of main against
# the variants given (tools/gpu_r05_var_mb.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py tests/test_gpu_seam.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_main.log 2>&1 || { tail -30 gpurun_out/pytest_main.log; exit 1; }
tail -1 gpurun_out/pytest_main.log
bash tools/gpu_r05_var_mb.sh "$@"
