# Round 4: band-pass VALU diet (ring windows without the third-dword select, shift-add 6x,
# bound_ctrl DPP, doubled weights packed by v_perm, ring descriptors carrying precomputed
# weights) -- multi-band GPU tests, serial kernel trace, C2 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blend.py tests/test_gpu_cylinder.py tests/test_gpu_seam.py tests/test_gpu_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_valu.log 2>&1 || { tail -30 gpurun_out/pytest_valu.log; exit 1; }
tail -1 gpurun_out/pytest_valu.log
bash tools/gpu_trace_variants.sh s_main || exit 1
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-also > gpurun_out/b_mb.log 2>&1 || { tail -20 gpurun_out/b_mb.log; exit 1; }
grep '^{"metric"' gpurun_out/b_mb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', d['value'], d['kernels'], d['max_abs_diff'], d['plan'].get('mb_mixed_px_per_capture'), d['plan'].get('mb_r1_entries_per_capture'))"
done
timeout -k 10 300 python bench.py --rig cylinder --no-cpu-baseline --no-also > gpurun_out/b_cyl.log 2>&1 || { tail -20 gpurun_out/b_cyl.log; exit 1; }
grep '^{"metric"' gpurun_out/b_cyl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C4', d['value'], d['kernels'], d['max_abs_diff'])"
