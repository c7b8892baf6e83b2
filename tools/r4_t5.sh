#!/bin/bash
# round-4: GPU tests (table, gradients, parity, full size) + A/B timings
# (checkpointing pair, Viterbi) against the round-3 library (build/ab/src)
set -o pipefail
out=gpurun_out/${1:-r4t7}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_table.py tests/test_gpu_table_grad.py tests/test_gpu_parity.py tests/test_gpu_full_size.py -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $out/tests.log 2>&1
rc=$?; echo "rc=$rc" >> $out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  TAG=new timeout -k 10 120 python -u tools/vit_time.py >> $out/ab.log 2>&1 || exit $?
  LT_ROOT=build/ab/src TAG=r3 timeout -k 10 120 python -u tools/vit_time.py >> $out/ab.log 2>&1 || exit $?
  BS=256,64 DESIGN=checkpoints TAG=new timeout -k 10 120 python -u tools/time_call.py >> $out/ab.log 2>&1 || exit $?
  LT_ROOT=build/ab/src BS=256,64 DESIGN=checkpoints TAG=r3 timeout -k 10 120 python -u tools/time_call.py >> $out/ab.log 2>&1 || exit $?
done
