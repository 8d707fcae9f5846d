# Round 4: the large-footprint streaming launch (C4's top / bottom tiles), the parallel host
# staging copies of the stream pipeline and the parity-sorted blend lists -- the GPU tests that
# touch them, the C4 bench line (graph-cut seams + multi-band), the C5 stream lines, the serial
# kernel trace (standalone band pass / blend times) and the C2 line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_remap.py tests/test_gpu_cylinder.py tests/test_gpu_seam.py tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_ingest.py tests/test_gpu_blend.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_c4.log 2>&1 || { tail -30 gpurun_out/pytest_c4.log; exit 1; }
tail -1 gpurun_out/pytest_c4.log
timeout -k 10 400 python bench.py --rig cylinder --no-also > gpurun_out/bench_cyl_gc.log 2>&1 || { tail -20 gpurun_out/bench_cyl_gc.log; exit 1; }
grep '^{"metric"' gpurun_out/bench_cyl_gc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['max_abs_diff'], d['plan'], d['kernels'], d['roofline']['frac'], d['roofline']['touched']['frac'], d['config']['workload'])"
timeout -k 10 300 python tools/stream_bench.py --summary > gpurun_out/stream_r04.log 2>&1 || { tail -20 gpurun_out/stream_r04.log; exit 1; }
grep -v summary gpurun_out/stream_r04.log | cut -c1-300
bash tools/gpu_trace_variants.sh s_main || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-also > gpurun_out/b_mb.log 2>&1 || { tail -20 gpurun_out/b_mb.log; exit 1; }
grep '^{"metric"' gpurun_out/b_mb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', d['value'], d['kernels'], d['max_abs_diff'])"
