# Round 5: C3 GPU tests, then the resident and uploaded C3 lines with the capture's geometry,
# plan and stitch inside the rig job (mcs_rig_job_wait_stitch) and, for comparison, built in
# Python (--python-stitch), depth 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_estimate.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_c3.log 2>&1 || { tail -30 gpurun_out/pytest_c3.log; exit 1; }
tail -1 gpurun_out/pytest_c3.log
for v in "" "--python-stitch"; do
  for r in "--resident" ""; do
    n=c3$(echo "$v$r" | tr -d ' -')
    timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap $r --depth ${DEPTH:-4} --steps 400 --warmup 20 --no-cpu-baseline $v > gpurun_out/$n.log 2>&1 || { tail -20 gpurun_out/$n.log; exit 1; }
    tail -1 gpurun_out/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], 'diff', d['max_abs_diff_vs_cpu_render'], d['config']['workload'][-60:])"
  done
done
