# Round 6: the persistent multi-band blend (mb_blend_q, per-XCD unit queues, next unit's loads
# issued during the current unit's compute) vs the one-unit-per-block blend (MCS_MB_BLQ=0).
# GPU blend / cylinder tests first (both multi-band paths), then C2 + C4 bench lines alternating
# twice, then C2 timelines of each form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py tests/test_gpu_seam.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_blq.log 2>&1 || { tail -30 gpurun_out/pytest_blq.log; exit 1; }
tail -1 gpurun_out/pytest_blq.log
for i in 1 2; do
  for rig in chain cylinder; do
    for v in 1 0; do
      MCS_MB_BLQ=$v timeout -k 10 200 python bench.py --rig $rig --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/blq_$v.log 2>&1 || { tail -20 gpurun_out/blq_$v.log; exit 1; }
      tail -1 gpurun_out/blq_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('blq=$v $rig', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
    done
  done
done
for v in 1 0; do
  (cd /tmp && MCS_MB_BLQ=$v MCS_BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/blqt_$v" -o run -- python3 "$R/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --no-also --no-paste-ref > "$R/gpurun_out/blqt_$v.log" 2>&1) || { tail -20 "$R/gpurun_out/blqt_$v.log"; exit 1; }
  echo "== blq=$v"; python3 tools/timeline.py "$R/gpurun_out/blqt_$v" 6
done
