set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
R="$GRAFT_REPO_ROOT"
cd /tmp
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_WAIT_INST_LDS" "TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" "SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT TA_BUSY_avr"; do
  n=$(echo $c | tr ' ' '_' | cut -c1-60)
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc/$n" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --frames 64 --no-cpu-baseline > "$R/gpurun_out/pmc/$n.log" 2>&1 || echo "fail $c" >> "$R/gpurun_out/pmc/fails.txt"
done
echo done
