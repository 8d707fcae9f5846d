# Round 4: blend work lists grouped by parity class (zero-weight taps skipped by whole waves) --
# the blend GPU tests, the serial kernel trace (standalone band pass / blend), the band-pass
# decomposition variants (MCS_EXP_BAND_PART, serial band pass only), the C2 line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_blend.log 2>&1 || { tail -30 gpurun_out/pytest_blend.log; exit 1; }
tail -1 gpurun_out/pytest_blend.log
bash tools/gpu_trace_variants.sh s_main bp0 bp1 bp2 bp4 bp7 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-also > gpurun_out/b_mb.log 2>&1 || { tail -20 gpurun_out/b_mb.log; exit 1; }
grep '^{"metric"' gpurun_out/b_mb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', d['value'], d['kernels'], d['max_abs_diff'])"
