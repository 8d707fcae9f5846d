# Round 3: Hamming matcher pairs/s + VALU utilisation, its kernel stats and one
# PMC pass; C3 with the frames resident in HBM (GPU-bound rate) beside the uploaded form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python tools/match_bench.py > gpurun_out/match.log 2>&1 || { tail -20 gpurun_out/match.log; exit 1; }
tail -1 gpurun_out/match.log
rm -rf "$R/gpurun_out/match_trace" "$R/gpurun_out/match_pmc"
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/match_trace" -o run -- python3 "$R/tools/match_bench.py" > "$R/gpurun_out/match_trace.log" 2>&1) || exit $?
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/match_pmc" -o run -- python3 "$R/tools/match_bench.py" > "$R/gpurun_out/match_pmc.log" 2>&1) || exit $?
for D in 3 4; do
  timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth $D --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/c3_res$D.log 2>&1 || { tail -20 gpurun_out/c3_res$D.log; exit 1; }
  tail -1 gpurun_out/c3_res$D.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 resident depth $D', d['value'], 'latency', d['latency_ms_upload_to_homographies'], d['max_abs_diff_vs_cpu_render'])"
done
