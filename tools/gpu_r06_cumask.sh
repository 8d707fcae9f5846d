# Round 6: CU mask of the band-pass + blend stream (MCS_MB_CUMASK, A/B only) -- C2 and C4
# multi-band bench lines on one box, none (default) first and last.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
F=ffffffff
run() {  # name mask rig
  local name=$1 mask=$2 rig=$3
  if [ "$mask" = none ]; then unset MCS_MB_CUMASK; else export MCS_MB_CUMASK=$mask; fi
  timeout -k 10 200 python bench.py --rig $rig --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/cm_$name.log 2>&1 || { tail -20 gpurun_out/cm_$name.log; exit 1; }
  tail -1 gpurun_out/cm_$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name $rig', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
}
for rig in chain cylinder; do
  run none none $rig || exit 1
  run all $F,$F,$F,$F,$F,$F,$F,$F $rig || exit 1
  run half5 55555555,55555555,55555555,55555555,55555555,55555555,55555555,55555555 $rig || exit 1
  run q3 77777777,77777777,77777777,77777777,77777777,77777777,77777777,77777777 $rig || exit 1
  run q1 11111111,11111111,11111111,11111111,11111111,11111111,11111111,11111111 $rig || exit 1
  run halfw $F,0,$F,0,$F,0,$F,0 $rig || exit 1
  run none2 none $rig || exit 1
done
