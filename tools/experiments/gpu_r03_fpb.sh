# Round 3: blend captures per block (MCS_MB_BL_FPB) -- parity of the 2-capture variant, then the
# multi-band lines (C2, C4) alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MCS_LIBRARY="$R/variants/fpb2.so" timeout -k 10 600 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fpb_tests.log 2>&1 || { tail -30 gpurun_out/fpb_tests.log; exit 1; }
tail -1 gpurun_out/fpb_tests.log
for i in 1 2; do
  for v in main fpb2 fpb4; do
    if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
    for rig in chain cylinder; do
      timeout -k 10 300 python bench.py --rig $rig --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/fpb.log 2>&1 || { tail -20 gpurun_out/fpb.log; exit 1; }
      tail -1 gpurun_out/fpb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $rig', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
    done
  done
done
