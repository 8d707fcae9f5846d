# Kernel traces of the timed launches for the main library and variants/<name>.so (arguments):
# per variant the bench line's launch time and every kernel's mean duration inside the marker
# window (tools/trace_stats.py).  Extra bench flags in $BENCH_ARGS.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
  rm -rf "$R/gpurun_out/tr_$v"
  (cd /tmp && MCS_BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/tr_$v" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-also --no-paste-ref $BENCH_ARGS > "$R/gpurun_out/tr_$v.log" 2>&1) || { tail -20 "$R/gpurun_out/tr_$v.log"; exit 1; }
  python tools/trace_stats.py gpurun_out/tr_$v --out gpurun_out/tr_stats_$v.json > /dev/null || exit 1
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.load(open(f"gpurun_out/tr_stats_{v}.json"))
line = [l for l in open(f"gpurun_out/tr_{v}.log") if l.startswith('{"metric"')]
ln = json.loads(line[-1]) if line else {}
w = d["windows"][0]
print(v, "span", w["launch_span_us_mean"], "bench", ln.get("value"), ln.get("max_abs_diff"),
      " ".join(f"{k}={x['mean_us']}x{x['dispatches']}" for k, x in w["kernels"].items()))
PY
done
