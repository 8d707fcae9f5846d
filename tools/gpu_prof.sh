# rocprofv3 kernel trace + stats of one bench run (no counters).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline "$@" > "$R/gpurun_out/prof.log" 2>&1
