# Multi-band check on the GPU box: blend/cylinder parity tests, the C2 launch probe, and the
# per-kernel times with the level pyramids run after (not beside) the streaming kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/profseq
timeout -k 10 400 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python tools/mb_probe.py > gpurun_out/mb_probe.log 2>&1 || exit $?
cd /tmp && MCS_MB_CONCURRENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/profseq" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit $?
