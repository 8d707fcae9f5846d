# bench lines (paste-only and multi-band; $RIG chain|cylinder, $BLENDS) for the main library and
# variants/<name>.so given as arguments, alternating twice (timing only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for v in "$@"; do
    if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
    for b in ${BLENDS:-none multiband}; do
      timeout -k 10 200 python bench.py --rig ${RIG:-chain} --blend $b --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/var_$v.log 2>&1 || { tail -20 gpurun_out/var_$v.log; exit 1; }
      tail -1 gpurun_out/var_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $b', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
    done
  done
done
