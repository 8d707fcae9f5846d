set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 ./tools/probes/copy_probe > gpurun_out/copy_probe_r04.txt 2>&1 || exit $?
timeout -k 10 200 ./tools/probes/copy_probe 4096 > gpurun_out/copy_probe_r04_4g.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-also --no-cpu-baseline > gpurun_out/b_mb.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --blend none --no-also --no-cpu-baseline > gpurun_out/b_paste.log 2>&1 || exit $?
grep '^{' gpurun_out/b_mb.log | cut -c1-400
grep '^{' gpurun_out/b_paste.log | cut -c1-400
