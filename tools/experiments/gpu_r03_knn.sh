# Round 3: kNN-2 variants (block-count target, queries per lane), matcher pairs/s.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for v in ${VARS:-qpl1 main qpl4}; do
    if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
    timeout -k 10 200 python tools/match_bench.py > gpurun_out/knn_$v.log 2>&1 || { tail -20 gpurun_out/knn_$v.log; exit 1; }
    tail -1 gpurun_out/knn_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', [(s['n_query'], s['ms_per_call'], s['pairs_per_s'], s['popcount_util'], s.get('max_abs_diff_vs_cpu')) for s in d['sizes']])"
  done
done
