# Round 3 experiment 5: band-pass descriptor ring depth (variants desc4 / desc6: the dependent
# descriptor -> window loads get 2 / 4 rows of slack instead of 1), fused and unfused band
# launches; serial kernel times (MCS_MB_CONCURRENT=0) from marker-bracketed traces.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for v in main desc4 desc6 desc6u; do
    unset MCS_LIBRARY MCS_MB_BANDS_FUSED
    case $v in main) ;; desc6u) export MCS_LIBRARY="$R/variants/desc6.so" MCS_MB_BANDS_FUSED=0 ;; *) export MCS_LIBRARY="$R/variants/$v.so" ;; esac
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-paste-ref > gpurun_out/var_$v.log 2>&1 || { tail -20 gpurun_out/var_$v.log; exit 1; }
    tail -1 gpurun_out/var_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v multiband', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
  done
done
for v in main desc6; do
  unset MCS_LIBRARY
  [ $v = main ] || export MCS_LIBRARY="$R/variants/$v.so"
  rm -rf "$R/gpurun_out/ser_$v"
  (cd /tmp && MCS_MB_CONCURRENT=0 MCS_BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/ser_$v" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-paste-ref > "$R/gpurun_out/ser_$v.log" 2>&1) || exit $?
  python tools/trace_stats.py gpurun_out/ser_$v | python -c "import json,sys; d=json.load(sys.stdin); w=d['windows'][0]; print('$v serial', w['launch_span_us_mean'], {k: v['mean_us'] for k, v in w['kernels'].items()})"
done
# C3 host-side breakdown: serial stages, and the pipelined forms with more host threads
timeout -k 10 300 python tools/estimate_bench.py --stitch --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/c3_serial.log 2>&1 || exit $?
tail -1 gpurun_out/c3_serial.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 serial', d['value'], d.get('stage_ms_per_capture'))"
timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --threads 8 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/c3_ov8.log 2>&1 || exit $?
tail -1 gpurun_out/c3_ov8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 overlap t8', d['value'])"
timeout -k 10 300 python tools/estimate_bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/c3_est.log 2>&1 || exit $?
tail -1 gpurun_out/c3_est.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 estimate only', d['value'], d.get('stage_ms_per_capture'))"
