# Round 6: where the C3 direct stitch (mcs_direct_c3_i1_o32) spends its time: kernel trace of the
# serial C3 run (standalone durations), then SQ counter passes (one group per pass) over it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
P="$R/gpurun_out/pmc_direct"; mkdir -p "$P"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/dtrace" -o run -- python3 "$R/tools/estimate_bench.py" --stitch --steps 60 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/dtrace.log" 2>&1) || { tail -20 "$R/gpurun_out/dtrace.log"; exit 1; }
head -12 "$R"/gpurun_out/dtrace/run_kernel_stats.csv | cut -d, -f1-4,6,7
i=0
for c in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
         "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum" "FETCH_SIZE"; do
  i=$((i+1))
  echo "$c" > "$P/pass$i.txt"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$P/pass$i" -o run -- python3 "$R/tools/estimate_bench.py" --stitch --steps 20 --warmup 2 --no-cpu-baseline > "$P/pass$i.log" 2>&1) || { tail -5 "$P/pass$i.log"; exit 1; }
done
MCS_PMC_DIR="$P" python3 tools/pmc_kernel.py mcs_direct_c3 > "$R/gpurun_out/pmc_direct.json" 2>&1; head -60 "$R/gpurun_out/pmc_direct.json"
MCS_PMC_DIR="$P" python3 tools/pmc_kernel.py mcs_orb_level > "$R/gpurun_out/pmc_orblevel.json" 2>&1; head -60 "$R/gpurun_out/pmc_orblevel.json"
