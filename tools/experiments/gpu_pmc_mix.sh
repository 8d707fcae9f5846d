# VALU instruction mix of the multi-band kernels (one counter pass, small bench run).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/pmcmix"
cd /tmp
rocprofv3 -L > "$R/gpurun_out/pmcmix/avail.txt" 2>&1 || true
i=0
for c in "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU" \
         "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F16 SQ_INSTS_VALU_MUL_F16 SQ_INSTS_VALU_FMA_F16 SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmcmix/pass$i" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-paste-ref "$@" > "$R/gpurun_out/pmcmix/pass$i.log" 2>&1 || exit $?
done
