# Round 3: where the streaming kernel's time goes (paste-only launch, variants/*.so built by
# tools/build_variant.py: nocomp = DMA + stores, nodma = compute + stores, nostore = DMA only),
# the box's host CPU (for the CPU baseline protocol), and the device-to-device copy ceiling.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
{ echo "nproc $(nproc)"; python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; lscpu | grep -i "model name\|socket\|core\|thread\|NUMA node(s)\|flags" | cut -c1-300; env | grep -i "OMP\|MAX_JOBS"; } > gpurun_out/host.txt 2>&1
BLENDS=none bash tools/gpu_var_bench.sh main nocomp nodma nostore > gpurun_out/decomp.txt 2>&1 || { cat gpurun_out/decomp.txt; exit 1; }
cat gpurun_out/decomp.txt
timeout -k 10 120 python tools/copy_bw.py > gpurun_out/copy_bw.json 2>&1 || exit 1
cat gpurun_out/copy_bw.json gpurun_out/host.txt
# tail / prologue share: the paste launch at 64, 128 and 256 captures per launch
for F in 128 256; do
  timeout -k 10 200 python bench.py --blend none --frames $F --no-cpu-baseline > gpurun_out/frames_$F.log 2>&1 || exit 1
  tail -1 gpurun_out/frames_$F.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('F=$F', d['value'], 'ms', d['ms_per_step'], d['kernels'])"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_blend.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_blend.log 2>&1; tail -3 gpurun_out/pytest_blend.log
