# Round 3: C3 serial latency -- rig job device chain (graph on / off) vs the per-call path, and a
# kernel trace of the serial loop.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "MCS_RIG_GRAPH=1" "MCS_RIG_GRAPH=0" "MCS_RIG_PATH=calls"; do
  env $cfg timeout -k 10 300 python tools/estimate_bench.py --stitch --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/c3s.log 2>&1 || { tail -20 gpurun_out/c3s.log; exit 1; }
  tail -1 gpurun_out/c3s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['value'], d['stage_ms_per_capture'])"
done
rm -rf "$R/gpurun_out/c3s_trace"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/c3s_trace" -o run -- python3 "$R/tools/estimate_bench.py" --stitch --steps 50 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/c3s_trace.log" 2>&1) || exit $?
echo traced
