# Round 3 experiment 1: HBM ceilings (copy probe), streaming-tile order (MCS_STREAM_ORDER 0/1),
# band pass with one capture per wave (variants/band1.so, 78 VGPRs: fits beside 6 streaming
# waves per SIMD), the blend tests, and a marker-bracketed kernel trace (tools/trace_stats.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 tools/probes/copy_probe > gpurun_out/copy_probe.txt 2>&1 || { cat gpurun_out/copy_probe.txt; exit 1; }
cat gpurun_out/copy_probe.txt
for i in 1 2; do
  for o in 0 1; do
    for b in none multiband; do
      MCS_STREAM_ORDER=$o timeout -k 10 200 python bench.py --blend $b --no-cpu-baseline --no-paste-ref > gpurun_out/ord.log 2>&1 || { tail -20 gpurun_out/ord.log; exit 1; }
      tail -1 gpurun_out/ord.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('order=$o $b', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
    done
  done
  MCS_LIBRARY=$R/variants/band1.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-paste-ref > gpurun_out/band1.log 2>&1 || { tail -20 gpurun_out/band1.log; exit 1; }
  tail -1 gpurun_out/band1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('band1 multiband', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_blend.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_blend.log 2>&1; tail -3 gpurun_out/pytest_blend.log
rm -rf "$R/gpurun_out/prof_mb"
(cd /tmp && MCS_BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_mb" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_mb.log" 2>&1) || { tail -20 gpurun_out/prof_mb.log; exit 1; }
tail -1 gpurun_out/prof_mb.log > gpurun_out/prof_mb_line.json
python tools/trace_stats.py gpurun_out/prof_mb --bench-line gpurun_out/prof_mb_line.json --out gpurun_out/trace_mb.json | head -60
