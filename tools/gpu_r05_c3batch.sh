# Round 5: multi-capture rig jobs (mcs_rig_job_create_batch) -- estimate GPU tests, then the C3
# resident and uploaded lines at 1 / 2 / 3 captures per job (depth 4), alternating twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_estimate.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_c3batch.log 2>&1 || { tail -30 gpurun_out/pytest_c3batch.log; exit 1; }
tail -1 gpurun_out/pytest_c3batch.log
for SS in "" --stitch-streams; do
  for b in 1 2 3; do
    timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth 4 --steps 600 --warmup 24 --no-cpu-baseline --batch $b $SS > gpurun_out/c3b_res_$b.log 2>&1 || { tail -20 gpurun_out/c3b_res_$b.log; exit 1; }
    tail -1 gpurun_out/c3b_res_$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$SS batch $b resident', d['value'], 'diff', d['max_abs_diff_vs_cpu_render'])"
  done
  for b in 1 2; do
    timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --depth 4 --steps 400 --warmup 20 --no-cpu-baseline --batch $b $SS > gpurun_out/c3b_up_$b.log 2>&1 || { tail -20 gpurun_out/c3b_up_$b.log; exit 1; }
    tail -1 gpurun_out/c3b_up_$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$SS batch $b uploaded', d['value'], 'link', d['frac_of_h2d_link'], 'diff', d['max_abs_diff_vs_cpu_render'])"
  done
done
