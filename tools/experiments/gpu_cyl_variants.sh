# C4 (cylinder) bench lines and the C2 launch probe for the main library and every
# build/variants/*.so (kernel experiments).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cylv
rm -f gpurun_out/cylv/*.log
timeout -k 10 200 python bench.py --rig cylinder --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/cylv/main.log 2>&1 || exit $?
timeout -k 10 200 python tools/mb_probe.py > gpurun_out/cylv/main_c2.log 2>&1 || exit $?
for v in build/variants/*.so; do
  [ -e "$v" ] || continue
  n=$(basename "$v" .so)
  MCS_LIBRARY="$PWD/$v" timeout -k 10 200 python bench.py --rig cylinder --steps 10 --warmup 2 --no-cpu-baseline > "gpurun_out/cylv/$n.log" 2>&1 || exit $?
  MCS_LIBRARY="$PWD/$v" timeout -k 10 200 python tools/mb_probe.py > "gpurun_out/cylv/${n}_c2.log" 2>&1 || exit $?
done
