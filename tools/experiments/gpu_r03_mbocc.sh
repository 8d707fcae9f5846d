# Round 3: multi-band co-residency variants (blend / band VGPR budgets that fit beside the
# streaming kernel's 6 waves per SIMD), multi-band bench lines alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_blend.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mbocc_tests.log 2>&1 || { tail -30 gpurun_out/mbocc_tests.log; exit 1; }
tail -1 gpurun_out/mbocc_tests.log
for i in 1 2; do
  for v in "$@"; do
    if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
    timeout -k 10 200 python bench.py --blend multiband --no-cpu-baseline --no-paste-ref > gpurun_out/var_$v.log 2>&1 || { tail -20 gpurun_out/var_$v.log; exit 1; }
    tail -1 gpurun_out/var_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
  done
done
