# Utilisation counters of the streaming kernel (paste-only bench): VALU / LDS / VMEM issue
# activity against busy CU cycles, one counter pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/pmcbusy"
rm -rf "$R/gpurun_out/pmcbusy/pass"*
cd /tmp
i=0
for c in "SQ_WAVES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
         "SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmcbusy/pass$i" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-paste-ref "$@" > "$R/gpurun_out/pmcbusy/pass$i.log" 2>&1 || exit $?
done
