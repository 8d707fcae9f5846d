# Round 3: device seam max-flow -- parity tests, then a tuning sweep (push launches / push rounds
# / relabel rounds; LDS-tiled relabel rounds via MCS_SEAM_RELABEL_LDS_ITERS).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_seam.py -x -q --timeout 120 --timeout-method thread > gpurun_out/seam_tests.log 2>&1 || { tail -30 gpurun_out/seam_tests.log; exit 1; }
tail -1 gpurun_out/seam_tests.log
for cfg in ${CFGS:-"8 16 32 1" "32 16 32 1" "32 16 16 1" "32 16 64 1" "32 16 64 0"}; do
  set -- $cfg
  MCS_SEAM_PUSH_LAUNCHES=$1 MCS_SEAM_PUSH_ITERS=$2 MCS_SEAM_RELABEL_LDS_ITERS=$3 MCS_SEAM_RELABEL_LDS=$4 MCS_SEAM_RELABEL_BATCH=${5:-8} timeout -k 10 120 python tools/seam_bench.py --no-check > gpurun_out/seamtune.log 2>&1 || { tail -20 gpurun_out/seamtune.log; exit 1; }
  tail -1 gpurun_out/seamtune.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['ms_per_plan'], d['stats_pairs_push_relabel_globalrelabels_us'])"
done
