# Round 3: multi-band list / band ordering A/B (MCS_MB_SORT), C2 and C4 lines alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for srt in 1 0; do
    for rig in chain cylinder; do
      MCS_MB_SORT=$srt timeout -k 10 300 python bench.py --rig $rig --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/srt.log 2>&1 || { tail -20 gpurun_out/srt.log; exit 1; }
      tail -1 gpurun_out/srt.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sort $srt $rig', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
    done
  done
done
