# Round 4: one-launch kNN-2 (quad DPP + LDS merge, no atomics / memset / finalize) -- matcher,
# rig-job and estimate GPU tests, the matcher bench, the resident C3 line and its kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $KNN_TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_knn.log 2>&1 || { tail -30 gpurun_out/pytest_knn.log; exit 1; }
tail -1 gpurun_out/pytest_knn.log
timeout -k 10 200 python tools/match_bench.py > gpurun_out/match_knn.log 2>&1 || { tail -20 gpurun_out/match_knn.log; exit 1; }
tail -1 gpurun_out/match_knn.log | cut -c1-700
timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth 4 --no-cpu-baseline --steps 300 > gpurun_out/c3_res_knn.log 2>&1 || { tail -20 gpurun_out/c3_res_knn.log; exit 1; }
tail -1 gpurun_out/c3_res_knn.log | cut -c1-250
rm -rf "$R/gpurun_out/c3prof_knn"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/c3prof_knn" -o run -- python3 "$R/tools/estimate_bench.py" --stitch --pipelined --overlap --resident --depth 1 --no-cpu-baseline --steps 200 > "$R/gpurun_out/c3prof_knn.log" 2>&1) || exit 1
