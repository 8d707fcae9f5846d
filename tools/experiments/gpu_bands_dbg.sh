cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MCS_DEBUG_BANDS=1 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-paste-ref > gpurun_out/bands_dbg.log 2> gpurun_out/bands_dbg.err
grep -c "^band" gpurun_out/bands_dbg.err
