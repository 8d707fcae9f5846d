# RETIRED (round 4): libmcs no longer reads MCS_STREAM_B32 -- the knob was stripped
# from the product path, so this script now times the same build on both sides of its A/B.
# Kept as the record of how the numbers DESIGN.md cites were taken; to repeat such an A/B,
# build the variants as compile-time defines with tools/build_variant.py (MCS_LIBRARY=...).
# A/B of the streaming kernel's DMA form: buffer resource (default) vs 64-bit global addresses
# (MCS_STREAM_B32=0), paste-only bench lines, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for v in 1 0; do
    MCS_STREAM_B32=$v timeout -k 10 200 python bench.py --blend none --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || { tail -20 gpurun_out/ab_$v.log; exit 1; }
    tail -1 gpurun_out/ab_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B32=$v', d['value'], 'ms', d['ms_per_step'], 'launch', d['kernels'])"
  done
done
