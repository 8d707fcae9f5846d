# Round 3: C3 through libmcs's rig jobs -- parity (job vs Python-issued steps, ORB vs the
# restatement), serial and pipelined captures/s at depth 2 / 3 / 4, and a kernel trace of the
# pipelined loop.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_estimate.py tests/test_gpu_orb.py -x -v --timeout 120 --timeout-method thread > gpurun_out/c3_tests.log 2>&1 || { tail -30 gpurun_out/c3_tests.log; exit 1; }
tail -2 gpurun_out/c3_tests.log
timeout -k 10 300 python tools/estimate_bench.py --stitch --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/c3_serial.log 2>&1 || { tail -20 gpurun_out/c3_serial.log; exit 1; }
tail -1 gpurun_out/c3_serial.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 serial', d['value'], d.get('stage_ms_per_capture'), d['max_abs_diff_vs_cpu_render'], d['max_reproj_err_px_vs_truth'])"
for D in 2 3 4; do
timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --depth $D --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/c3_ov$D.log 2>&1 || { tail -20 gpurun_out/c3_ov$D.log; exit 1; }
tail -1 gpurun_out/c3_ov$D.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 overlap depth $D', d['value'], 'latency', d['latency_ms_upload_to_homographies'], d['max_abs_diff_vs_cpu_render'], d['max_reproj_err_px_vs_truth'])"
done
rm -rf "$R/gpurun_out/c3_trace"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/c3_trace" -o run -- python3 "$R/tools/estimate_bench.py" --stitch --pipelined --overlap --depth 3 --steps 100 --warmup 10 --no-cpu-baseline > "$R/gpurun_out/c3_trace.log" 2>&1) || exit $?
tail -1 gpurun_out/c3_trace.log | cut -c1-200
