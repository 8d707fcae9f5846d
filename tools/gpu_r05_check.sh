set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{"metric"' gpurun_out/bench.log > gpurun_out/bench_line.json
python3 -c "
import json; d=json.load(open('gpurun_out/bench_line.json'))
print(d['value'], d['kernels'], d['max_abs_diff'], d['checked_captures'])
for k,v in d['also'].items(): print(k, json.dumps(v)[:400])
"
