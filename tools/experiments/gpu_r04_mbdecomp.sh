# Round 4: where the multi-band launch's time goes -- variants built with MCS_EXP_MB (1 serial,
# 2 no blend, 3 no band pass, 4 neither) beside main, two alternations, then a kernel trace of the
# serial variant (standalone kernel durations).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for v in main mb1 mb2 mb3 mb4; do
    if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/dec_$v.log 2>&1 || { tail -20 gpurun_out/dec_$v.log; exit 1; }
    tail -1 gpurun_out/dec_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d.get('max_abs_diff'))"
  done
done
export MCS_LIBRARY="$R/variants/mb1.so"
rm -rf "$R/gpurun_out/trace_mb1"
(cd /tmp && MCS_BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/trace_mb1" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-also --no-paste-ref > "$R/gpurun_out/trace_mb1.log" 2>&1) || exit $?
python tools/trace_stats.py gpurun_out/trace_mb1 --out gpurun_out/trace_stats_mb1.json > /dev/null || exit 1
python -c "
import json; d=json.load(open('gpurun_out/trace_stats_mb1.json'))
for w in d['windows']:
    print(w['window'], w['launch_span_us_mean'])
    for k,v in w['kernels'].items(): print('  ', k, v['dispatches'], v['mean_us'])
"
