# RETIRED (round 4): libmcs no longer reads MCS_DEBUG_BANDS, MCS_MB_CONCURRENT -- the knob was stripped
# from the product path, so this script now times the same build on both sides of its A/B.
# Kept as the record of how the numbers DESIGN.md cites were taken; to repeat such an A/B,
# build the variants as compile-time defines with tools/build_variant.py (MCS_LIBRARY=...).
# serial kernel stats of the C4 cylinder bench (multi-band levels on the caller's stream)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf "$R/gpurun_out/prof_cylser"
(cd /tmp && MCS_MB_CONCURRENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_cylser" -o run -- python3 "$R/bench.py" --rig cylinder --steps 10 --warmup 2 --no-cpu-baseline --no-paste-ref > "$R/gpurun_out/prof_cylser.log" 2>&1) || exit $?
python3 "$R/tools/kstats.py" "$R/gpurun_out/prof_cylser" | grep "bands\|blend\|stream\|levels"
MCS_DEBUG_BANDS=1 timeout -k 10 120 python3 bench.py --rig cylinder --steps 1 --warmup 0 --no-cpu-baseline --no-paste-ref 2> gpurun_out/cyl_bands.txt > /dev/null || exit $?
grep -c "^band" gpurun_out/cyl_bands.txt; grep -c "^tile" gpurun_out/cyl_bands.txt
