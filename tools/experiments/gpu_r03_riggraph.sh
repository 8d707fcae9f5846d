# Round 3: C3 rig jobs with / without the captured hipGraph -- parity, then pipelined captures/s
# (frames uploaded, and resident in HBM), alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_estimate.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c3_tests.log 2>&1 || { tail -30 gpurun_out/c3_tests.log; exit 1; }
tail -1 gpurun_out/c3_tests.log
for i in 1 2; do
  for g in 1 0; do
    for res in "" "--resident"; do
      MCS_RIG_GRAPH=$g timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap $res --depth 4 --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/c3g.log 2>&1 || { tail -20 gpurun_out/c3g.log; exit 1; }
      tail -1 gpurun_out/c3g.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('graph $g $res', d['value'], 'latency', d['latency_ms_upload_to_homographies'], d['max_abs_diff_vs_cpu_render'])"
    done
  done
done
