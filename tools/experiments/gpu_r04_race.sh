# Round 4: which build introduced a nondeterministic multi-band mismatch (tools/debug_mb_race.py
# over the builds of commits 8487f70 and 89afb1e and the working tree).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARS:-c89 e1 e12 eall main}; do
  if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$GRAFT_REPO_ROOT/variants/$v.so"; fi
  timeout -k 10 300 python -u tools/debug_mb_race.py 3 > gpurun_out/race_$v.log 2>&1; echo "$v rc=$?"; grep "px differ\|== rep" gpurun_out/race_$v.log | cut -c1-60
done
