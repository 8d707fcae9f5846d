# Bench lines of record: C2 (default) and C4 (--rig cylinder), each with its rocprofv3 kernel
# stats; the PMC traffic of the C2 launch (tools/gpu_pmc.sh) feeds the C2 line's roofline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof gpurun_out/profcyl
bash tools/gpu_prof.sh || exit $?
cd "$R" && bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || exit $?
cd "$R" && MCS_PMC_DIR="$R/gpurun_out/pmc" python tools/pmc_summary.py > gpurun_out/pmc_summary.log 2>&1 || exit $?
cp profiles/pmc_latest.json gpurun_out/pmc_latest.json
cd "$R" && timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/profcyl" -o run -- python3 "$R/bench.py" --rig cylinder --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/profcyl.log" 2>&1 || exit $?
cd "$R" && timeout -k 10 300 python bench.py --rig cylinder > gpurun_out/bench_cyl.log 2>&1
