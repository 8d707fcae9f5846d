# ORB iteration: parity (orb, match, ransac, estimate), single-frame probe, C3 bench lines,
# kernel stats of the serial single-frame probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_estimate.py tests/test_gpu_match.py tests/test_gpu_ransac.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_orb.log 2>&1 || { tail -40 gpurun_out/pytest_orb.log; exit 1; }
tail -1 gpurun_out/pytest_orb.log
timeout -k 10 200 python tools/orb_probe.py > gpurun_out/orb_probe.json 2> gpurun_out/orb_probe.err || { tail gpurun_out/orb_probe.err; exit 1; }
tail -1 gpurun_out/orb_probe.json
timeout -k 10 300 python tools/estimate_bench.py --steps 200 --warmup 20 > gpurun_out/c3.json 2> gpurun_out/c3.err || { tail gpurun_out/c3.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c3.json')); print('C3', d['value'], d['stage_ms_per_capture'], d.get('cpu_baseline',{}).get('value'))"
timeout -k 10 300 python tools/estimate_bench.py --stitch --steps 100 --warmup 10 > gpurun_out/c3_stitch.json 2> gpurun_out/c3_stitch.err || { tail gpurun_out/c3_stitch.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c3_stitch.json')); print('C3 e2e', d['value'], d['stage_ms_per_capture'], d['max_abs_diff_vs_cpu_render'])"
rm -rf "$R/gpurun_out/prof_orb"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_orb" -o run -- python3 "$R/tools/estimate_bench.py" --steps 50 --warmup 5 --threads 1 --no-cpu-baseline > "$R/gpurun_out/prof_orb.log" 2>&1) || exit 1
python3 tools/kstats.py gpurun_out/prof_orb
