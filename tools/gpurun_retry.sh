#!/bin/bash
# Runs one gpurun call, retrying ONLY when no box was available or the box failed while being
# prepared (infrastructure: exit 3 / "transient"); never retries a command that ran.
# usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
log=$1; to=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient\|no free box\|backing off" "$log"; then
    echo "[retry $i: rc $rc, infrastructure]" >> "$log.tries"; sleep 100; continue
  fi
  exit $rc
done
exit 3
