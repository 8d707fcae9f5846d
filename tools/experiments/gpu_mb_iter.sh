# multi-band iteration: parity tests (blend, cylinder, parity), bench line, serial kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py tests/test_gpu_parity.py tests/test_gpu_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_mb.log 2>&1 || { tail -40 gpurun_out/pytest_mb.log; exit 1; }
tail -2 gpurun_out/pytest_mb.log
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_mb.log 2>&1 || { tail -20 gpurun_out/bench_mb.log; exit 1; }
tail -1 gpurun_out/bench_mb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'], 'paste', d['kernels'])"
cd /tmp
rm -rf "$R/gpurun_out/prof_ser"
MCS_MB_CONCURRENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_ser" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-paste-ref "$@" > "$R/gpurun_out/prof_ser.log" 2>&1 || exit $?
python3 "$R/tools/kstats.py" "$R/gpurun_out/prof_ser"
