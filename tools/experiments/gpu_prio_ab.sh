# RETIRED (round 4): libmcs no longer reads MCS_MB_PRIORITY -- the knob was stripped
# from the product path, so this script now times the same build on both sides of its A/B.
# Kept as the record of how the numbers DESIGN.md cites were taken; to repeat such an A/B,
# build the variants as compile-time defines with tools/build_variant.py (MCS_LIBRARY=...).
# multi-band side stream at the greatest priority (MCS_MB_PRIORITY=1) vs default: C2 and C4 bench lines
# alternating (timing only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for v in -1 0; do
    for r in chain cylinder; do
      MCS_MB_PRIORITY=$v timeout -k 10 200 python bench.py --rig $r --no-cpu-baseline > gpurun_out/split_$v.log 2>&1 || { tail -20 gpurun_out/split_$v.log; exit 1; }
      tail -1 gpurun_out/split_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r PRIO=$v', d['value'], 'launch', d['kernels']['launch_ms'])"
    done
  done
done
