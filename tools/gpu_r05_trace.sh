# Round 5: marker-bracketed kernel traces of the timed launches (C2 multi-band and C4
# multi-band) for the main library and, optionally, one variant (variants/<name>.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
for v in main "$@"; do
  if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
  for rig in chain cylinder; do
    (cd /tmp && MCS_BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/tr_${v}_$rig" -o run -- python3 "$R/bench.py" --rig $rig --steps 6 --warmup 2 --no-cpu-baseline --no-also --no-paste-ref > "$R/gpurun_out/tr_${v}_$rig.log" 2>&1) || { tail -20 "$R/gpurun_out/tr_${v}_$rig.log"; exit 1; }
  done
done
