# Round 6: the multi-band launch with the blend after the whole streaming launch (MCS_MB_SPLIT=0:
# band pass beside the stream, blend alone at the end) vs the split default (blend beside the
# late streaming tiles).  C2 + C4 bench lines, alternating twice, then a C2 timeline of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
for i in 1 2; do
  for rig in chain cylinder; do
    for v in 1 0; do
      MCS_MB_SPLIT=$v timeout -k 10 200 python bench.py --rig $rig --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/sp_$v.log 2>&1 || { tail -20 gpurun_out/sp_$v.log; exit 1; }
      tail -1 gpurun_out/sp_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('split=$v $rig', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
    done
  done
done
for v in 0; do
  (cd /tmp && MCS_MB_SPLIT=$v MCS_BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/spt_$v" -o run -- python3 "$R/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --no-also --no-paste-ref > "$R/gpurun_out/spt_$v.log" 2>&1) || { tail -20 "$R/gpurun_out/spt_$v.log"; exit 1; }
  echo "== split=$v"; python3 tools/timeline.py "$R/gpurun_out/spt_$v" 8
done
