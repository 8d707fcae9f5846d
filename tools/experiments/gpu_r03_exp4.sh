# Round 3 experiment 4: tail-split launch lists (MCS_STREAM_TAIL = 96 default vs 0 = off) on the
# main build and on the 40 KiB / 64-VGPR variants; the multi-band tests for the new lists.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_parity.py tests/test_gpu_stream.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 || { tail -30 gpurun_out/pytest_sel.log; exit 1; }
tail -1 gpurun_out/pytest_sel.log
for i in 1 2; do
  for v in main lds40 cores; do
    for t in 96 0 48; do
      unset MCS_LIBRARY
      [ $v = main ] || export MCS_LIBRARY="$R/variants/$v.so"
      for b in none multiband; do
        MCS_STREAM_TAIL=$t timeout -k 10 200 python bench.py --blend $b --no-cpu-baseline --no-paste-ref > gpurun_out/var_$v.log 2>&1 || { tail -20 gpurun_out/var_$v.log; exit 1; }
        tail -1 gpurun_out/var_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v tail=$t $b', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
      done
    done
  done
done
