# multi-band probe (tools/mb_probe.py) with the main library and every build/variants/*.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mbv
rm -f gpurun_out/mbv/*.log
timeout -k 10 200 python tools/mb_probe.py > gpurun_out/mbv/main.log 2>&1 || exit $?
for v in build/variants/*.so; do
  [ -e "$v" ] || continue
  n=$(basename "$v" .so)
  MCS_LIBRARY="$PWD/$v" timeout -k 10 200 python tools/mb_probe.py > "gpurun_out/mbv/$n.log" 2>&1 || exit $?
done
