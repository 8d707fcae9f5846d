# Round 4: FAST cardinal pre-test + interior-tile staging in mcs_orb_level -- ORB / estimate GPU
# tests, the resident C3 line at depth 4 and 1, and a kernel-statistics pass at depth 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_estimate.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_orb.log 2>&1 || { tail -30 gpurun_out/pytest_orb.log; exit 1; }
tail -1 gpurun_out/pytest_orb.log
for d in 4 1; do
  timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth $d --no-cpu-baseline --steps 300 > gpurun_out/c3_res_d$d.log 2>&1 || { tail -20 gpurun_out/c3_res_d$d.log; exit 1; }
  tail -1 gpurun_out/c3_res_d$d.log | cut -c1-250
done
rm -rf "$R/gpurun_out/c3prof_d1"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/c3prof_d1" -o run -- python3 "$R/tools/estimate_bench.py" --stitch --pipelined --overlap --resident --depth 1 --no-cpu-baseline --steps 200 > "$R/gpurun_out/c3prof_d1.log" 2>&1) || exit 1
