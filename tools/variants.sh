# Kernel experiments on the GPU box: parity of the main library, then bench lines for it and for
# every variant library under build/variants/ (built by multicamera_stitching_amd.build(lib=...)).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/variants
[ -n "$NO_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/variants/main.log 2>&1 && \
for v in build/variants/*.so; do
  [ -e "$v" ] || continue
  n=$(basename "$v" .so)
  MCS_LIBRARY="$PWD/$v" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "gpurun_out/variants/$n.log" 2>&1 || exit $?
done
