#!/bin/bash
# round-4: precision diagnostics + the table / parity GPU tests + a pipe A/B
# against the round-3 library (build/ab/src)
set -o pipefail
out=gpurun_out/${1:-r4t5}
mkdir -p $out
[ -n "$DIAG" ] && { timeout -k 10 300 python -u tools/fld_precision.py 2 > $out/fld.log 2>&1 || exit $?; }
[ -n "$DIAG" ] && { timeout -k 10 300 python -u tools/ck_precision.py 0 1 > $out/ck.log 2>&1 || exit $?; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_table.py tests/test_gpu_table_grad.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $out/tests.log 2>&1
rc=$?; echo "rc=$rc" >> $out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  BS=256,64 DESIGN=checkpoints TAG=new timeout -k 10 120 python -u tools/time_call.py >> $out/ab.log 2>&1 || exit $?
  LT_ROOT=build/ab/src BS=256,64 DESIGN=checkpoints TAG=r3 timeout -k 10 120 python -u tools/time_call.py >> $out/ab.log 2>&1 || exit $?
done
