#!/bin/bash
# Host-side helper: gpurun, waiting out pool capacity only (busy / no free box /
# backing off: nothing ran, nothing charged); a command that ran is never re-run.
log=$1; shift
for n in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun "$@" > $log 2>&1; rc=$?
  if grep -q "nothing was charged\|no free box\|backing off" $log && ! grep -q "merged" $log; then sleep 90; continue; fi
  exit $rc
done
exit $rc
