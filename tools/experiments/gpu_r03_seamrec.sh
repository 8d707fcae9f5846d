# Round 3: C4 seams per plan, device push-relabel (labels checked vs the oracle) and host Dinic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 150 python tools/seam_bench.py > gpurun_out/seam_dev.log 2>&1 || { tail -20 gpurun_out/seam_dev.log; exit 1; }
tail -1 gpurun_out/seam_dev.log
MCS_SEAM_FLOW=host timeout -k 10 150 python tools/seam_bench.py --no-check --reps 1 > gpurun_out/seam_host.log 2>&1 || { tail -20 gpurun_out/seam_host.log; exit 1; }
tail -1 gpurun_out/seam_host.log
