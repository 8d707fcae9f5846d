# Round 6: CU masks balanced over the shader engines (word w of MCS_MB_CUMASK = CU w of every SE,
# as the CU-mask bits are dealt round-robin over the engines): the band-pass + blend stream on
# 1 / 2 / 4 / 6 of each engine's 8 CUs.  C2 + C4 bench lines, then C2 timelines for w2 / w4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
F=ffffffff
mask() { case $1 in none) echo "";; w1) echo $F,0,0,0,0,0,0,0;; w2) echo $F,$F,0,0,0,0,0,0;;
  w4) echo $F,$F,$F,$F,0,0,0,0;; w6) echo $F,$F,$F,$F,$F,$F,0,0;; w7) echo $F,$F,$F,$F,$F,$F,$F,0;; esac; }
for rig in chain cylinder; do
  for v in none w1 w2 w4 w6 w7 none; do
    m=$(mask $v); if [ -z "$m" ]; then unset MCS_MB_CUMASK; else export MCS_MB_CUMASK=$m; fi
    timeout -k 10 200 python bench.py --rig $rig --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/cm2_$v.log 2>&1 || { tail -20 gpurun_out/cm2_$v.log; exit 1; }
    tail -1 gpurun_out/cm2_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $rig', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
  done
done
for v in w2 w4; do
  export MCS_MB_CUMASK=$(mask $v)
  (cd /tmp && MCS_BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/cmt2_$v" -o run -- python3 "$R/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --no-also --no-paste-ref > "$R/gpurun_out/cmt2_$v.log" 2>&1) || { tail -20 "$R/gpurun_out/cmt2_$v.log"; exit 1; }
  echo "== $v"; python3 tools/timeline.py "$R/gpurun_out/cmt2_$v" 9
done
