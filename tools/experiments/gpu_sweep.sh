set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python tools/sweep.py > gpurun_out/sweep.log 2>&1
