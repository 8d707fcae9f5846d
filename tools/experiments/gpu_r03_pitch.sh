# Round 3: LDS row pitch of the streaming footprints (multiple of 128 B: bank-conflict-free window
# reads) -- full GPU suite on the new default, then paste / multi-band lines for the variants
# and the LDS bank-conflict counter of the streaming kernel (default vs packed rows).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pitch_tests.log 2>&1 || { tail -30 gpurun_out/pitch_tests.log; exit 1; }
tail -1 gpurun_out/pitch_tests.log
BLENDS="none multiband" bash tools/gpu_var_bench.sh p0 main p128l48 p128l52 || exit 1
for v in p0 main; do
  if [ "$v" = main ]; then unset MCS_LIBRARY; else export MCS_LIBRARY="$R/variants/$v.so"; fi
  rm -rf "$R/gpurun_out/pitch_pmc_$v"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d "$R/gpurun_out/pitch_pmc_$v" -o run -- python3 "$R/bench.py" --blend none --steps 2 --warmup 1 --no-cpu-baseline --no-paste-ref > "$R/gpurun_out/pitch_pmc_$v.log" 2>&1) || exit $?
done
unset MCS_LIBRARY
python3 - <<'PY'
import csv, glob, collections
for v in ("p0", "main"):
    f = glob.glob(f"gpurun_out/pitch_pmc_{v}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if not r["Kernel_Name"].startswith("mcs_stream_c3"):
            continue
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    big = [c for c in agg.values() if c["SQ_WAVES"] > 20000]
    bc = sum(c["SQ_LDS_BANK_CONFLICT"] for c in big); act = sum(c["SQ_LDS_IDX_ACTIVE"] for c in big)
    print(v, "stream dispatches", len(big), "lds_bank_conflict_frac", round(bc / act, 4) if act else None)
PY
