# A/B of env settings on the multi-band bench: parity tests once, then serial kernel stats per
# setting (each argument: NAME=VALUE or "base")
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_mb.log 2>&1 || { tail -40 gpurun_out/pytest_mb.log; exit 1; }
tail -1 gpurun_out/pytest_mb.log
for v in "$@"; do
  tag=$(echo "$v" | tr '=' '_')
  rm -rf "$R/gpurun_out/prof_$tag"
  (cd /tmp && env $( [ "$v" = base ] || echo "$v" ) MCS_MB_CONCURRENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$tag" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-paste-ref > "$R/gpurun_out/prof_$tag.log" 2>&1) || exit $?
  echo "== $v"; python3 "$R/tools/kstats.py" "$R/gpurun_out/prof_$tag" | grep "bands\|blend_c\|stream"
  env $( [ "$v" = base ] || echo "$v" ) timeout -k 10 300 python bench.py --no-cpu-baseline --no-paste-ref > gpurun_out/bench_$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'])"
done
