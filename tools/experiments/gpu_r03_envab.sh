# Round 3: multi-band launch-structure A/B by environment (each argument: NAME=VALUE or base),
# bench lines alternated twice, plus the C5 companion line once.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for v in "$@"; do
    tag=$(echo "$v" | tr '=' '_')
    env $( [ "$v" = base ] || echo "$v" ) timeout -k 10 300 python bench.py --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/bench_$tag.log 2>&1 || { tail -20 gpurun_out/bench_$tag.log; exit 1; }
    tail -1 gpurun_out/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
  done
done
timeout -k 10 300 python tools/stream_bench.py --sizes 3840x2160 --frames 200 --summary > gpurun_out/c5.log 2>&1 || { tail -20 gpurun_out/c5.log; exit 1; }
tail -1 gpurun_out/c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print([ (l.get('blend'), l.get('depth'), l.get('zero_copy'), l.get('fps')) for l in d['lines'] if 'fps' in l])"
