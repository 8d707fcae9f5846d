# Round 3: the default bench line with its companion lines (driver-visible C3 / C4 / matcher /
# seams), timed end to end.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
start=$(date +%s)
timeout -k 10 900 python bench.py > gpurun_out/bench_all.log 2>&1 || { tail -20 gpurun_out/bench_all.log; exit 1; }
echo "bench seconds $(( $(date +%s) - start ))"
tail -1 gpurun_out/bench_all.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('C2', d['value'], d['ms_per_step'], d['max_abs_diff'])
for k,v in d.get('also',{}).items(): print(k, json.dumps(v)[:400])"
