# Round 4: resident C3 (estimate + stitch per capture, frames in HBM): lines at depth 4 and
# depth 1, and kernel statistics of each (rocprofv3 --kernel-trace --stats).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for d in 4 1; do
  timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth $d --no-cpu-baseline --steps 300 > gpurun_out/c3_res_d$d.log 2>&1 || { tail -20 gpurun_out/c3_res_d$d.log; exit 1; }
  tail -1 gpurun_out/c3_res_d$d.log | cut -c1-300
  rm -rf "$R/gpurun_out/c3prof_d$d"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/c3prof_d$d" -o run -- python3 "$R/tools/estimate_bench.py" --stitch --pipelined --overlap --resident --depth $d --no-cpu-baseline --steps 200 > "$R/gpurun_out/c3prof_d$d.log" 2>&1) || { tail -20 "$R/gpurun_out/c3prof_d$d.log"; exit 1; }
done
