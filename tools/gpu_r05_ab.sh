# Round 5: full -m gpu suite, then the C2 (multi-band, paste) and C4 bench lines of this build
# (kernels + roofline fields printed); argument "quick" skips the suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
if [ "${1:-full}" != quick ]; then
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
fi
for a in "--no-also" "--blend none --no-also" "--rig cylinder --no-also"; do
  n=$(echo "$a" | tr -d ' -' )
  timeout -k 10 300 python bench.py --no-cpu-baseline $a > gpurun_out/ab_$n.log 2>&1 || { tail -20 gpurun_out/ab_$n.log; exit 1; }
  grep -h '^{"metric"' gpurun_out/ab_$n.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('$n', d['value'], d['kernels'], 'frac', r['frac'], 'touched', r['touched']['frac'], 'diff', d['max_abs_diff'])"
done
