# Round 3: device push-relabel seams -- parity (device vs host Dinic, and the plan path vs the
# oracle), then the C4 seam time per plan, device vs host Dinic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_seam.py -x -v --timeout 120 --timeout-method thread > gpurun_out/seam_tests.log 2>&1 || { tail -30 gpurun_out/seam_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/seam_tests.log | tail -20
timeout -k 10 150 python tools/seam_bench.py > gpurun_out/seam_dev.log 2>&1 || { tail -20 gpurun_out/seam_dev.log; exit 1; }
tail -1 gpurun_out/seam_dev.log
MCS_SEAM_FLOW=host timeout -k 10 150 python tools/seam_bench.py --no-check --reps 1 > gpurun_out/seam_host.log 2>&1 || { tail -20 gpurun_out/seam_host.log; exit 1; }
tail -1 gpurun_out/seam_host.log
