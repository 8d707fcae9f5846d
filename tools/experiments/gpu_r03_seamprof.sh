# Round 3: kernel trace of the device seam max-flow (C4 plan).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf "$R/gpurun_out/seam_prof"
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/seam_prof" -o run -- python3 "$R/tools/seam_bench.py" --no-check --reps 1 > "$R/gpurun_out/seam_prof.log" 2>&1) || exit $?
tail -1 gpurun_out/seam_prof.log
