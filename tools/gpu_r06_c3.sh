# Round 6: C3 record on the build with 64 x 32 ORB tiles: ORB / estimate / match / ransac GPU tests,
# then the C3 lines of tools/gpu_r06_final.sh (uploaded depth 4, resident, serial, estimation only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_estimate.py tests/test_gpu_match.py tests/test_gpu_ransac.py tests/test_gpu_l2match.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_c3.log 2>&1 || { tail -30 gpurun_out/pytest_c3.log; exit 1; }
tail -1 gpurun_out/pytest_c3.log
timeout -k 10 300 python tools/estimate_bench.py --stitch --no-cpu-baseline > gpurun_out/c3_serial.log 2>&1 || exit $?
timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --depth 4 --steps 400 --warmup 20 > gpurun_out/c3_overlap.log 2>&1 || exit $?
timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth 4 --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/c3_resident.log 2>&1 || exit $?
timeout -k 10 300 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth 4 --steps 400 --warmup 20 --no-cpu-baseline --batch 2 > gpurun_out/c3_resident_b2.log 2>&1 || exit $?
timeout -k 10 300 python tools/estimate_bench.py > gpurun_out/c3_estimate.log 2>&1 || exit $?
for f in c3_serial c3_overlap c3_resident c3_resident_b2 c3_estimate; do echo "$f $(tail -1 gpurun_out/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('max_abs_diff_vs_cpu_render'))")"; done
