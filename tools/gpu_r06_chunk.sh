# Round 6: multi-band scratch chunk (MCS_MB_CHUNK, A/B): band pass then blend per chunk of 16 / 32
# captures on the side stream (the blend reads the scratch its chunk's band pass has just written)
# vs one 64-capture chunk.  C2 + C4 multi-band lines alternating twice, blend tests at chunk 16.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
MCS_MB_CHUNK=16 timeout -k 10 400 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not sweep" > gpurun_out/pytest_chunk.log 2>&1 || { tail -30 gpurun_out/pytest_chunk.log; exit 1; }
tail -1 gpurun_out/pytest_chunk.log
for i in 1 2; do
  for rig in chain cylinder; do
    for v in 64 32 16; do
      MCS_MB_CHUNK=$v timeout -k 10 200 python bench.py --rig $rig --no-cpu-baseline --no-paste-ref --no-also > gpurun_out/ch_$v.log 2>&1 || { tail -20 gpurun_out/ch_$v.log; exit 1; }
      tail -1 gpurun_out/ch_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('chunk=$v $rig', d['value'], 'launch', d['kernels']['launch_ms'], 'diff', d['max_abs_diff'])"
    done
  done
done
(cd /tmp && MCS_MB_CHUNK=16 MCS_BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/cht_16" -o run -- python3 "$R/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --no-also --no-paste-ref > "$R/gpurun_out/cht_16.log" 2>&1) || { tail -20 "$R/gpurun_out/cht_16.log"; exit 1; }
echo "== chunk=16"; python3 tools/timeline.py "$R/gpurun_out/cht_16" 12
