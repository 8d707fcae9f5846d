# Round-6 final record on one build (argument a: tests, smoke, counters, bench lines; b: traces,
# C3, matcher, seams, C5, probe; none: both): full -m gpu suite, smoke, PMC counter passes over the default bench
# workload (-> profiles/pmc_latest.json on the box, copied to gpurun_out/), the default bench line
# (roofline.traffic from those counters, the full CPU-baseline protocol), paste-only and cylinder
# lines, marker-bracketed kernel traces of the timed launches (tools/trace_stats.py), C3 lines and
# trace, the matcher, C4 seams, the C5 stream and the HBM copy probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "${1:-all}" != b ]; then
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
echo smoke ok
bash tools/gpu_pmc.sh || exit $?
MCS_PMC_DIR="$R/gpurun_out/pmc_cyl" bash tools/gpu_pmc.sh --rig cylinder || exit $?
WLC=$(grep -h "^{\"metric\"" gpurun_out/pmc_cyl/pass1.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())[\"roofline\"][\"traffic_workload\"])") || exit 1
MCS_PMC_DIR="$R/gpurun_out/pmc_cyl" python3 tools/pmc_summary.py "$WLC" mcs_stream_c3,mcs_stream_big_c3,mcs_direct_c3,mcs_mb_bands,mcs_mb_blend_c3 profiles/pmc_latest_cyl.json > gpurun_out/pmc_summary_cyl.txt 2>&1 || { cat gpurun_out/pmc_summary_cyl.txt; exit 1; }
cp profiles/pmc_latest_cyl.json gpurun_out/pmc_latest_cyl.json
python3 tools/pmc_summary.py > gpurun_out/pmc_summary.txt 2>&1 || { cat gpurun_out/pmc_summary.txt; exit 1; }
cp profiles/pmc_latest.json gpurun_out/pmc_latest.json
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{"metric"' gpurun_out/bench.log > gpurun_out/bench_line.json
timeout -k 10 300 python bench.py --blend none --no-also > gpurun_out/bench_paste.log 2>&1 || exit $?
grep '^{"metric"' gpurun_out/bench_paste.log > gpurun_out/bench_line_paste.json
timeout -k 10 300 python bench.py --rig cylinder --no-also > gpurun_out/bench_cyl.log 2>&1 || exit $?
grep '^{"metric"' gpurun_out/bench_cyl.log > gpurun_out/bench_line_cyl.json
[ "${1:-all}" = a ] && { echo done a; exit 0; }
fi
for w in "mb:" "paste:--blend none" "cyl:--rig cylinder"; do
  n=${w%%:*}; a=${w#*:}
  rm -rf "$R/gpurun_out/trace_$n"
  (cd /tmp && MCS_BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/trace_$n" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-also $a > "$R/gpurun_out/trace_$n.log" 2>&1) || exit $?
  grep '^{"metric"' gpurun_out/trace_$n.log > gpurun_out/trace_${n}_line.json
  python tools/trace_stats.py gpurun_out/trace_$n --bench-line gpurun_out/trace_${n}_line.json --out gpurun_out/trace_stats_$n.json > /dev/null || exit 1
done
timeout -k 10 300 python tools/estimate_bench.py --stitch --no-cpu-baseline > gpurun_out/c3_serial.log 2>&1 || exit $?
timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --depth 4 --steps 400 --warmup 20 > gpurun_out/c3_overlap.log 2>&1 || exit $?
timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth 4 --steps 400 --warmup 20 --no-cpu-baseline --python-stitch > gpurun_out/c3_resident_pystitch.log 2>&1 || exit $?
timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth 4 --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/c3_resident.log 2>&1 || exit $?
timeout -k 10 300 python tools/estimate_bench.py > gpurun_out/c3_estimate.log 2>&1 || exit $?
tail -1 gpurun_out/c3_overlap.log | cut -c1-300
rm -rf "$R/gpurun_out/trace_c3"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/trace_c3" -o run -- python3 "$R/tools/estimate_bench.py" --stitch --pipelined --overlap --depth 4 --steps 200 --warmup 10 --no-cpu-baseline > "$R/gpurun_out/trace_c3.log" 2>&1) || exit $?
timeout -k 10 200 python tools/match_bench.py > gpurun_out/match.log 2>&1 || exit $?
timeout -k 10 200 python tools/seam_bench.py > gpurun_out/seam.log 2>&1 || exit $?
timeout -k 10 300 python tools/stream_bench.py --summary > gpurun_out/stream.log 2>&1 || exit $?
timeout -k 10 120 ./tools/probes/copy_probe > gpurun_out/copy_probe.txt 2>&1 || exit $?
echo done
echo done
