# C2 / C4 multi-band bench lines for settings of one environment variable, alternating twice:
#   bash tools/experiments/gpu_env_ab.sh VAR value1 value2 ...   ("-" = unset)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
var=$1; shift
for i in 1 2; do
  for v in "$@"; do
    for r in chain cylinder; do
      if [ "$v" = - ]; then unset $var; else export $var=$v; fi
      timeout -k 10 200 python bench.py --rig $r --no-cpu-baseline > gpurun_out/envab.log 2>&1 || { tail -20 gpurun_out/envab.log; exit 1; }
      tail -1 gpurun_out/envab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r $var=$v', d['value'], 'launch', d['kernels']['launch_ms'])"
    done
  done
done
