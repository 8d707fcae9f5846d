# Round 6: kernel traces of the C2 multi-band launch with the band-pass + blend stream on a CU
# mask (MCS_MB_CUMASK): none / 1 CU in 4 / 1 CU in 8 -- per-launch timelines (tools/timeline.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
for v in none q1 x8; do
  case $v in
    none) unset MCS_MB_CUMASK ;;
    q1) export MCS_MB_CUMASK=11111111,11111111,11111111,11111111,11111111,11111111,11111111,11111111 ;;
    x8) export MCS_MB_CUMASK=01010101,01010101,01010101,01010101,01010101,01010101,01010101,01010101 ;;
  esac
  (cd /tmp && MCS_BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/cmt_$v" -o run -- python3 "$R/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --no-also --no-paste-ref > "$R/gpurun_out/cmt_$v.log" 2>&1) || { tail -20 "$R/gpurun_out/cmt_$v.log"; exit 1; }
  echo "== $v"; tail -1 "$R/gpurun_out/cmt_$v.log" | cut -c1-200
  python3 tools/timeline.py "$R/gpurun_out/cmt_$v" 9
done
