# multiband experiment: parity of the blend tests, bench line of the main library and of each
# variant; *prof* variants print in-kernel phase cycle counts (MCS_MB_PROF).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/variants
rm -f gpurun_out/variants/*.log
[ -n "$NO_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/variants/main.log 2>&1 || exit $?
for v in build/variants/*.so; do
  [ -e "$v" ] || continue
  n=$(basename "$v" .so)
  case "$n" in *prof*) a="--steps 1 --warmup 1";; *) a="--steps 20 --warmup 3";; esac
  MCS_LIBRARY="$PWD/$v" timeout -k 10 200 python bench.py $a --no-cpu-baseline > "gpurun_out/variants/$n.log" 2>&1 || exit $?
done
