#!/bin/bash
# Runs one gpurun call, retrying only when no box was obtained (nothing ran:
# exit 3, or a transient acquisition failure); never re-runs a command that
# ran. Usage: tools/gpu_try.sh LOG TIMEOUT CMD...
log=$1; to=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|has no free box\|stopped responding while being prepared\|backing off" $log && ! grep -q "status=ok" $log; then
    sleep 45; continue
  fi
  if [ $rc -eq 3 ]; then sleep 45; continue; fi
  exit $rc
done
exit 99
