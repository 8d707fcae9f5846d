# RETIRED (round 4): libmcs no longer reads MCS_MB_CONCURRENT -- the knob was stripped
# from the product path, so this script now times the same build on both sides of its A/B.
# Kept as the record of how the numbers DESIGN.md cites were taken; to repeat such an A/B,
# build the variants as compile-time defines with tools/build_variant.py (MCS_LIBRARY=...).
# serial multi-band kernel stats per library variant (no parity tests: timing experiments)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
  rm -rf "$R/gpurun_out/prof_$v"
  (cd /tmp && MCS_MB_CONCURRENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$v" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-paste-ref > "$R/gpurun_out/prof_$v.log" 2>&1) || exit $?
  echo "== $v"; python3 "$R/tools/kstats.py" "$R/gpurun_out/prof_$v" | grep "bands\|blend_c\|stream"
done
