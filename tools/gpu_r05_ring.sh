# Round 5: band-pass LDS ring depth A/B (C2 and C4 multi-band lines; LDS-ring band counts),
# main against the variants given, alternating twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do
  for v in main "$@"; do
    if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$GRAFT_REPO_ROOT/variants/$v.so"; fi
    for rig in chain cylinder; do
      timeout -k 10 200 python bench.py --rig $rig --blend multiband --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/ring_$v.log 2>&1 || { tail -20 gpurun_out/ring_$v.log; exit 1; }
      tail -1 gpurun_out/ring_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $rig', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'], 'lds_bands', d['plan']['mb_bands_lds_ring'], 'of', d['plan']['mb_bands'])"
    done
  done
done
