# Round 5: full -m gpu suite; C3 lines (rig-job stitch vs Python-built stitch); same-box bench A/B
# of main against the variants named as arguments (C2 paste + multi-band, C4 seam + multi-band).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for v in "" "--python-stitch"; do
  n=c3res$(echo "$v" | tr -d ' -')
  timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth 4 --steps 400 --warmup 20 --no-cpu-baseline $v > gpurun_out/$n.log 2>&1 || { tail -20 gpurun_out/$n.log; exit 1; }
  tail -1 gpurun_out/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], 'diff', d['max_abs_diff_vs_cpu_render'])"
done
RIG=chain BLENDS="none multiband" bash tools/gpu_var_bench.sh main "$@" || exit 1
RIG=cylinder BLENDS="seam multiband" bash tools/gpu_var_bench.sh main "$@" || exit 1
