# RETIRED (round 4): libmcs no longer reads MCS_MB_BAND_ALIGNED, MCS_MB_BAND_LDS, MCS_MB_CONCURRENT -- the knob was stripped
# from the product path, so this script now times the same build on both sides of its A/B.
# Kept as the record of how the numbers DESIGN.md cites were taken; to repeat such an A/B,
# build the variants as compile-time defines with tools/build_variant.py (MCS_LIBRARY=...).
# band pass window alignment: serial kernel times and concurrent multi-band lines per variant
# (main; unaligned = main with MCS_MB_BAND_ALIGNED=0; noring = MCS_MB_BAND_LDS=0; else
# variants/<name>.so; timing only:
# the aligned-test variant computes wrong pixels on purpose)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  unset MCS_LIBRARY MCS_MB_BAND_ALIGNED MCS_MB_BAND_LDS
  case "$v" in main) ;; unaligned) export MCS_MB_BAND_ALIGNED=0 ;; noring) export MCS_MB_BAND_LDS=0 ;; *) export MCS_LIBRARY="$R/variants/$v.so" ;; esac
  rm -rf "$R/gpurun_out/prof_$v"
  (cd /tmp && MCS_MB_CONCURRENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$v" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-paste-ref --no-also > "$R/gpurun_out/prof_$v.log" 2>&1) || exit $?
  echo "== $v serial"; python3 "$R/tools/kstats.py" "$R/gpurun_out/prof_$v" | grep "bands\|blend_c\|stream"
done
for i in 1 2; do
  for v in "$@"; do
    unset MCS_LIBRARY MCS_MB_BAND_ALIGNED MCS_MB_BAND_LDS
    case "$v" in main) ;; unaligned) export MCS_MB_BAND_ALIGNED=0 ;; noring) export MCS_MB_BAND_LDS=0 ;; *) export MCS_LIBRARY="$R/variants/$v.so" ;; esac
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/var_$v.log 2>&1 || { tail -20 gpurun_out/var_$v.log; exit 1; }
    tail -1 gpurun_out/var_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
  done
done
