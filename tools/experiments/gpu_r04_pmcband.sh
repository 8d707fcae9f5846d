# Round 4: counters of the serial band pass / blend (variant s_main = MCS_EXP_MB=1) after the
# XCD-grouped launches: traffic and L2 hit rate per kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
export MCS_LIBRARY="$R/variants/s_main.so"
mkdir -p "$R/gpurun_out/pmcb"
cd /tmp
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
         "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
         "TA_BUSY_avr TA_BUSY_max TD_BUSY_avr TD_BUSY_max"; do
  i=$((i+1))
  echo "$c" > "$R/gpurun_out/pmcb/pass$i.txt"
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmcb/pass$i" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-paste-ref --no-also > "$R/gpurun_out/pmcb/pass$i.log" 2>&1 || exit $?
done
cd "$R"
for k in mcs_mb_bands mcs_mb_blend mcs_stream_c3; do MCS_PMC_DIR=gpurun_out/pmcb python tools/pmc_kernel.py $k > gpurun_out/pmcb/$k.json || exit 1; done
python - <<'PY'
import json
for k in ("mcs_mb_bands", "mcs_mb_blend", "mcs_stream_c3"):
    d = json.load(open(f"gpurun_out/pmcb/{k}.json"))
    c = d["counters"]
    print(k, {x: round(c.get(x, 0)) for x in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum", "SQ_WAVES", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "TA_BUSY_avr", "TD_BUSY_avr", "GRBM_GUI_ACTIVE")})
    print("   derived", {x: (round(v, 3) if isinstance(v, float) else v) for x, v in d["derived"].items()})
PY
