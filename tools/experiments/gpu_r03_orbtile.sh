# Round 3: ORB level tile height (MCS_ORB_TILE_H 16 / 32) -- ORB + estimate parity with the
# 32-row variant, then C3 (frames resident and uploaded) alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MCS_LIBRARY="$R/variants/oty32.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_estimate.py -x -q --timeout 120 --timeout-method thread > gpurun_out/orbt_tests.log 2>&1 || { tail -30 gpurun_out/orbt_tests.log; exit 1; }
tail -1 gpurun_out/orbt_tests.log
for i in 1 2; do
  for v in main oty32; do
    if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
    for res in "--resident" ""; do
      timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap $res --depth 4 --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/orbt.log 2>&1 || { tail -20 gpurun_out/orbt.log; exit 1; }
      tail -1 gpurun_out/orbt.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $res', d['value'], 'latency', d['latency_ms_upload_to_homographies'], 'h2d', d.get('h2d_gb_per_s'), d.get('h2d_link_ceiling_gb_per_s'), d.get('frac_of_h2d_link'), d['max_abs_diff_vs_cpu_render'])"
    done
  done
done
