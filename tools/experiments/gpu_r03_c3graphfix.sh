# Round 3: rig-job graph replay fix -- estimate tests, serial latency (graph on / off), pipelined.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_estimate.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c3_tests.log 2>&1 || { tail -30 gpurun_out/c3_tests.log; exit 1; }
tail -1 gpurun_out/c3_tests.log
for cfg in "MCS_RIG_GRAPH=1" "MCS_RIG_GRAPH=0"; do
  env $cfg timeout -k 10 300 python tools/estimate_bench.py --stitch --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/c3s.log 2>&1 || { tail -20 gpurun_out/c3s.log; exit 1; }
  tail -1 gpurun_out/c3s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg serial', d['value'], d['stage_ms_per_capture'])"
  for res in "" "--resident"; do
    env $cfg timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap $res --depth 4 --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/c3p.log 2>&1 || { tail -20 gpurun_out/c3p.log; exit 1; }
    tail -1 gpurun_out/c3p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg pipelined $res', d['value'], 'latency', d['latency_ms_upload_to_homographies'], d['max_abs_diff_vs_cpu_render'])"
  done
done
