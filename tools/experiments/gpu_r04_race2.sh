# Round 4: the descriptor-slot race fix (s_waitcnt lgkmcnt(0) before the slot's refill), parity
# over repeated full-size C2 stitches, then kernel traces of the fixed build, the in-kernel-weights
# build and their serial-decomposition variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
VARS="main e1w" bash tools/experiments/gpu_r04_race.sh || exit 1
bash tools/gpu_trace_variants.sh main e1w c89 mbx e1mbx
