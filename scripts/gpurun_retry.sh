#!/bin/bash
# Host-side helper: run one gpurun call, retrying ONLY while the pool reports no free box / slot (exit 3,
# nothing ran, nothing charged).  Any other outcome -- success, a failing or faulting command -- is final.
#   scripts/gpurun_retry.sh LOG TIMEOUT 'command'
log=$1; to=$2; cmd=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 120
done
echo "exit=$rc" >> "$log"
exit $rc
