# Round 4: isolate a multi-band parity failure (C2 full size) over debug variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in main d_dpp d_mad6 d_win d_all main; do
  if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$GRAFT_REPO_ROOT/variants/$v.so"; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_blend.py -m gpu -q --timeout 300 --timeout-method thread -k "c2_full" > gpurun_out/iso_$v.log 2>&1; echo "$v rc=$?"; grep -o "assert [0-9]* == 0" gpurun_out/iso_$v.log | head -2
done
