# Round 3: row-chunked band pass + blend (blend of chunk c beside the bands of chunk c+1):
# multi-band GPU tests, then the C2 / C4 multi-band lines for 1 (unchunked) .. 6 chunks.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py tests/test_gpu_seam.py -x -q --timeout 300 --timeout-method thread > gpurun_out/rc_tests.log 2>&1 || { tail -30 gpurun_out/rc_tests.log; exit 1; }
tail -1 gpurun_out/rc_tests.log
for i in 1 2; do
  for c in ${CHUNKS:-1 2 3 4 6}; do
    MCS_MB_ROW_CHUNKS=$c timeout -k 10 300 python bench.py --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/rc.log 2>&1 || { tail -20 gpurun_out/rc.log; exit 1; }
    tail -1 gpurun_out/rc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('chunks $c', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
  done
done
for c in 1 3; do
  MCS_MB_ROW_CHUNKS=$c timeout -k 10 300 python bench.py --rig cylinder --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/rc.log 2>&1 || { tail -20 gpurun_out/rc.log; exit 1; }
  tail -1 gpurun_out/rc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cyl chunks $c', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
done
