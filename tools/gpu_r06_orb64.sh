# Round 6: 64 x 64 ORB tiles (variants/orb64.so, MCS_ORB_TILE_H=64) vs the 64 x 32 default
# (variants/orb32main.so = the main build): ORB / estimate GPU tests on the variant, then C3
# resident estimate + stitch alternating three times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
MCS_LIBRARY="$R/variants/orb64.so" timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_estimate.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_orb64.log 2>&1 || { tail -30 gpurun_out/pytest_orb64.log; exit 1; }
tail -1 gpurun_out/pytest_orb64.log
for i in 1 2 3; do
  for v in orb32main orb64; do
    export MCS_LIBRARY="$R/variants/$v.so"
    timeout -k 10 200 python tools/estimate_bench.py --stitch --pipelined --overlap --resident --depth 4 --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/o64_$v.log 2>&1 || { tail -20 gpurun_out/o64_$v.log; exit 1; }
    echo "$v resident $(tail -1 gpurun_out/o64_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['max_abs_diff_vs_cpu_render'])")"
  done
done
