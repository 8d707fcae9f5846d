# Round 5: counter passes only (C2 multi-band default workload + C4 cylinder) and their summaries
# (gpurun_out/pmc_summary*.txt, pmc_latest*.json) -- the counter half of tools/gpu_r05_final.sh a.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_pmc.sh || exit $?
MCS_PMC_DIR="$R/gpurun_out/pmc_cyl" bash tools/gpu_pmc.sh --rig cylinder || exit $?
WLC=$(grep -h "^{\"metric\"" gpurun_out/pmc_cyl/pass1.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())[\"roofline\"][\"traffic_workload\"])") || exit 1
MCS_PMC_DIR="$R/gpurun_out/pmc_cyl" python3 tools/pmc_summary.py "$WLC" mcs_stream_c3,mcs_stream_big_c3,mcs_direct_c3,mcs_mb_bands,mcs_mb_blend_c3 profiles/pmc_latest_cyl.json > gpurun_out/pmc_summary_cyl.txt 2>&1 || { cat gpurun_out/pmc_summary_cyl.txt; exit 1; }
cp profiles/pmc_latest_cyl.json gpurun_out/pmc_latest_cyl.json
python3 tools/pmc_summary.py > gpurun_out/pmc_summary.txt 2>&1 || { cat gpurun_out/pmc_summary.txt; exit 1; }
cp profiles/pmc_latest.json gpurun_out/pmc_latest.json
echo done
