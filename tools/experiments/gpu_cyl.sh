# C4 (cylinder) bench line and its rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/profcyl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/profcyl" -o run -- python3 "$R/bench.py" --rig cylinder --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/profcyl.log" 2>&1 || exit $?
cd "$R" && timeout -k 10 300 python bench.py --rig cylinder > gpurun_out/bench_cyl.log 2>&1
