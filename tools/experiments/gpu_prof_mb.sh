# kernel trace + stats of the multi-band bench (band pass on and off)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_mb" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-paste-ref > "$R/gpurun_out/prof_mb.log" 2>&1 || exit $?
MCS_MB_CONCURRENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_mb_serial" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-paste-ref > "$R/gpurun_out/prof_mb_serial.log" 2>&1 || exit $?
echo done
