# Round-2 record on the final build: full -m gpu suite, smoke, rocprofv3 counter passes over the
# default bench workload, their summary (profiles/pmc_latest.json on the box, copied to
# gpurun_out/), the default bench line (roofline.traffic from those counters), kernel stats of
# the bench (multi-band, paste-only, cylinder), the C4 cylinder bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
echo smoke ok
bash tools/gpu_pmc.sh || exit $?
python3 tools/pmc_summary.py > gpurun_out/pmc_summary.txt 2>&1 || { cat gpurun_out/pmc_summary.txt; exit 1; }
cp profiles/pmc_latest.json gpurun_out/pmc_latest.json
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log > gpurun_out/bench_line.json
for w in "mb:" "paste:--blend none" "cyl:--rig cylinder"; do
  n=${w%%:*}; a=${w#*:}
  rm -rf "$R/gpurun_out/prof_$n"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$n" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline $a > "$R/gpurun_out/prof_$n.log" 2>&1) || exit $?
done
timeout -k 10 300 python bench.py --rig cylinder > gpurun_out/bench_cyl.log 2>&1 || exit $?
tail -1 gpurun_out/bench_cyl.log > gpurun_out/bench_line_cyl.json
echo done
