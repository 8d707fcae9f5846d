# multi-band variants: parity tests on the main build, then bench + serial kernel stats per variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_mb.log 2>&1 || { tail -40 gpurun_out/pytest_mb.log; exit 1; }
tail -1 gpurun_out/pytest_mb.log
for v in main "$@"; do
  if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$v.log 2>&1 || { tail -20 gpurun_out/bench_$v.log; exit 1; }
  echo "== $v"; tail -1 gpurun_out/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'], 'paste', d['kernels'])"
  rm -rf "$R/gpurun_out/prof_$v"
  (cd /tmp && MCS_MB_CONCURRENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$v" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-paste-ref > "$R/gpurun_out/prof_$v.log" 2>&1) || exit $?
  python3 "$R/tools/kstats.py" "$R/gpurun_out/prof_$v" | grep -v "footprint\|prepare\|prep_\|owner\|classify\|bdesc"
done
