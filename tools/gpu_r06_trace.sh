# Round 6: kernel trace (rocprofv3, marker-bracketed timed launches) of the C2 multi-band bench
# line, then per-kernel durations (tools/trace_stats.py).  Args: rig (chain|cylinder).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
rig=${1:-chain}
(cd /tmp && MCS_BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/tr6_$rig" -o run -- python3 "$R/bench.py" --rig $rig --steps 6 --warmup 2 --no-cpu-baseline --no-also --no-paste-ref > "$R/gpurun_out/tr6_$rig.log" 2>&1) || { tail -20 "$R/gpurun_out/tr6_$rig.log"; exit 1; }
python3 tools/trace_stats.py "$R/gpurun_out/tr6_$rig" > "$R/gpurun_out/tr6_${rig}_stats.txt" 2>&1; tail -40 "$R/gpurun_out/tr6_${rig}_stats.txt"
