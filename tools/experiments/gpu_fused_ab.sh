# RETIRED (round 4): libmcs no longer reads MCS_MB_BANDS_FUSED -- the knob was stripped
# from the product path, so this script now times the same build on both sides of its A/B.
# Kept as the record of how the numbers DESIGN.md cites were taken; to repeat such an A/B,
# build the variants as compile-time defines with tools/build_variant.py (MCS_LIBRARY=...).
# interior + edge bands in one launch (MCS_MB_BANDS_FUSED=1) vs two: parity of the blend / stream
# paths, then C2 and C4 bench lines alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_ingest.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1 || { tail -30 gpurun_out/pytest_fused.log; exit 1; }
tail -1 gpurun_out/pytest_fused.log
for i in 1 2; do
  for v in 1 0; do
    for r in chain cylinder; do
      MCS_MB_BANDS_FUSED=$v timeout -k 10 200 python bench.py --rig $r --no-cpu-baseline > gpurun_out/split_$v.log 2>&1 || { tail -20 gpurun_out/split_$v.log; exit 1; }
      tail -1 gpurun_out/split_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r FUSED=$v', d['value'], 'launch', d['kernels']['launch_ms'])"
    done
  done
done
