# Round-2 first GPU pass: full -m gpu suite, smoke, the default bench line, the C5 stream bench
# with the link probe (zero-copy rows included).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 400 python tools/stream_bench.py --frames 120 > gpurun_out/stream.jsonl 2> gpurun_out/stream.err || exit $?
echo done
