# Round 3: C3 rig jobs, blocking-sync waits (default) vs spinning waits (MCS_FEATURE_SYNC=spin),
# pipeline depth 2 / 3 / 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_estimate.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c3_tests.log 2>&1 || { tail -30 gpurun_out/c3_tests.log; exit 1; }
tail -1 gpurun_out/c3_tests.log
for S in block spin; do
  if [ $S = spin ]; then export MCS_FEATURE_SYNC=spin; else unset MCS_FEATURE_SYNC; fi
  timeout -k 10 300 python tools/estimate_bench.py --stitch --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/c3_serial_$S.log 2>&1 || { tail -20 gpurun_out/c3_serial_$S.log; exit 1; }
  tail -1 gpurun_out/c3_serial_$S.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$S serial', d['value'], d.get('stage_ms_per_capture'))"
  for D in 2 3 4; do
    timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --depth $D --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/c3_ov${D}_$S.log 2>&1 || { tail -20 gpurun_out/c3_ov${D}_$S.log; exit 1; }
    tail -1 gpurun_out/c3_ov${D}_$S.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$S depth $D', d['value'], 'latency', d['latency_ms_upload_to_homographies'], d['max_abs_diff_vs_cpu_render'])"
  done
done
