# Round 3 experiment 3: co-residency of the multi-band kernels with the streaming kernel --
# variants/lds40.so (40 KiB streaming blocks: room for a 36 KiB blend block per CU),
# variants/cores.so (the same + 64 VGPRs: room for the blend's 112), and the XCD-contiguous
# band mapping (MCS_MB_BAND_XCD=1) on the main build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for v in main main_xcd lds40 cores; do
    unset MCS_LIBRARY MCS_MB_BAND_XCD
    case $v in main) ;; main_xcd) export MCS_MB_BAND_XCD=1 ;; *) export MCS_LIBRARY="$R/variants/$v.so" ;; esac
    for b in none multiband; do
      timeout -k 10 200 python bench.py --blend $b --no-cpu-baseline --no-paste-ref > gpurun_out/var_$v.log 2>&1 || { tail -20 gpurun_out/var_$v.log; exit 1; }
      tail -1 gpurun_out/var_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $b', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
    done
  done
done
