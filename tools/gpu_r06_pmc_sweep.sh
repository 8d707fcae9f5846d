# Round 6: two counter passes (wave / instruction mix) over the C2 multi-band bench, for the sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; P="$R/gpurun_out/pmc6"; mkdir -p "$P"; cd /tmp
i=0
for c in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d "$P/pass$i" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-paste-ref --no-also "$@" > "$P/pass$i.log" 2>&1 || exit $?
done
MCS_PMC_DIR="$P" python3 "$R/tools/pmc_kernel.py" mcs_mb_sweep
