# Round measurement: GPU parity suite, bench line, rocprofv3 kernel stats, PMC counter passes
# (HBM traffic per launch -> profiles/pmc_latest.json), then the bench line again (with traffic).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
nproc > gpurun_out/nproc.txt; lscpu | grep -i "model name" >> gpurun_out/nproc.txt || true
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
bash tools/gpu_prof.sh || exit $?
cd "$R" && bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || exit $?
cd "$R" && MCS_PMC_DIR="$R/gpurun_out/pmc" python tools/pmc_summary.py > gpurun_out/pmc_summary.log 2>&1 || exit $?
cp profiles/pmc_latest.json gpurun_out/pmc_latest.json
cd "$R" && timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
