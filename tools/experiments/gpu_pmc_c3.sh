# rocprofv3 counter passes over the C3 estimation bench (ORB + kNN-2 + RANSAC per capture), one
# counter group per pass (bench flags in $C3_ARGS: the resident rig-job path with
# C3_ARGS='--stitch --pipelined --overlap --resident --depth 1 --steps 20 --warmup 2');
# summarise with: python tools/pmc_c3_summary.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
rm -rf "$R/gpurun_out/pmc_c3"; mkdir -p "$R/gpurun_out/pmc_c3"
cd /tmp
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
         "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  echo "$c" > "$R/gpurun_out/pmc_c3/pass$i.txt"
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc_c3/pass$i" -o run -- python3 "$R/tools/estimate_bench.py" ${C3_ARGS:---steps 10 --warmup 2 --threads 1} --no-cpu-baseline > "$R/gpurun_out/pmc_c3/pass$i.log" 2>&1 || exit $?
done
echo done
