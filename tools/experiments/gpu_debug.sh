set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/debug_pixels.py > gpurun_out/dbg_pixels.log 2>&1
echo done
