# RETIRED (round 4): libmcs no longer reads MCS_MB_CONCURRENT -- the knob was stripped
# from the product path, so this script now times the same build on both sides of its A/B.
# Kept as the record of how the numbers DESIGN.md cites were taken; to repeat such an A/B,
# build the variants as compile-time defines with tools/build_variant.py (MCS_LIBRARY=...).
# PMC passes over the serial multi-band launch (band kernel alone); per-kernel averages with
#   MCS_PMC_DIR=gpurun_out/pmc_bands python tools/pmc_kernel.py mcs_mb_bands_all_a_c3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
rm -rf "$R/gpurun_out/pmc_bands"; mkdir -p "$R/gpurun_out/pmc_bands"
cd /tmp
i=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM" \
         "TA_BUSY_avr TA_BUSY_max" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
         "FETCH_SIZE"; do
  i=$((i+1))
  echo "$c" > "$R/gpurun_out/pmc_bands/pass$i.txt"
  MCS_MB_CONCURRENT=0 timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc_bands/pass$i" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-paste-ref > "$R/gpurun_out/pmc_bands/pass$i.log" 2>&1 || echo "pass $i failed"
done
echo done
