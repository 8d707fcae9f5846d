# stream-kernel iteration: parity (paste/blend/cylinder/stream), paste-only + multi-band bench lines,
# paste-only kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blend.py tests/test_gpu_cylinder.py tests/test_gpu_stream.py tests/test_gpu_remap.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_st.log 2>&1 || { tail -40 gpurun_out/pytest_st.log; exit 1; }
tail -1 gpurun_out/pytest_st.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_st.log 2>&1 || { tail -20 gpurun_out/bench_st.log; exit 1; }
tail -1 gpurun_out/bench_st.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('multiband value', d['value'], 'ms', d['ms_per_step'], d['kernels'])"
timeout -k 10 300 python bench.py --blend none --no-cpu-baseline > gpurun_out/bench_paste.log 2>&1 || exit 1
tail -1 gpurun_out/bench_paste.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('paste value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'])"
rm -rf "$R/gpurun_out/prof_paste"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_paste" -o run -- python3 "$R/bench.py" --blend none --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_paste.log" 2>&1) || exit 1
python3 tools/kstats.py gpurun_out/prof_paste | grep stream
