# Round 6: the large-footprint streaming launch split into capture ranges (MCS_BIG_PARTS) --
# cylinder / seam GPU tests, then C4 seam and multi-band bench lines for parts 1 / 2 / 4 / 8,
# alternating twice (same box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cylinder.py tests/test_gpu_seam.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_big.log 2>&1 || { tail -30 gpurun_out/pytest_big.log; exit 1; }
tail -1 gpurun_out/pytest_big.log
for i in 1 2; do
  for parts in 1 2 4 8; do
    for b in seam multiband; do
      MCS_BIG_PARTS=$parts timeout -k 10 200 python bench.py --rig cylinder --blend $b --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/big_$parts.log 2>&1 || { tail -20 gpurun_out/big_$parts.log; exit 1; }
      tail -1 gpurun_out/big_$parts.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('parts $parts $b', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
    done
  done
done
