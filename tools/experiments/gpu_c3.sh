# C3 (pose re-estimation) on the GPU box: ORB parity tests, the C3 line with its CPU baseline,
# and the per-kernel times of the same chain.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/profc3
timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_orb.log 2>&1 || exit $?
timeout -k 10 400 python tools/estimate_bench.py > gpurun_out/c3.json 2> gpurun_out/c3.err && timeout -k 10 200 python tools/estimate_bench.py --pinned --no-cpu-baseline > gpurun_out/c3_pinned.json 2>> gpurun_out/c3.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/profc3" -o run -- python3 "$R/tools/estimate_bench.py" --no-cpu-baseline > /dev/null 2>&1
