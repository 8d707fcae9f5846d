# rocprofv3 counter passes (one counter group per pass, no tracing domains) over the default bench
# workload (extra bench flags as arguments; output dir $MCS_PMC_DIR, default gpurun_out/pmc);
# stops at the first failing pass.  Summarise with: python tools/pmc_summary.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
P="${MCS_PMC_DIR:-$R/gpurun_out/pmc}"
mkdir -p "$P"
cd /tmp
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
         "TCC_HIT_sum TCC_MISS_sum" \
         "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"; do
  i=$((i+1))
  echo "$c" > "$P/pass$i.txt"
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$P/pass$i" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-paste-ref --no-also "$@" > "$P/pass$i.log" 2>&1 || exit $?
done
echo done
