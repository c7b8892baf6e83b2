#!/bin/bash
# Viterbi follower-sleep variants: bit-exact cfg4 check + timing for each
set -o pipefail
out=gpurun_out/${1:-r5vv}
mkdir -p $out
TAG=prod timeout -k 10 120 python -u tools/vit_time.py >> $out/vit.log 2>&1 || exit $?
for v in ${VARS:-nap4 nap16 nap64 nap1p8}; do
  LT_LIB_PATH=build/var/vit_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_full_size.py -q -k "cfg4" --timeout 200 --timeout-method thread -p no:cacheprovider > $out/t_$v.log 2>&1
  rc=$?; echo "$v rc=$rc" >> $out/vit.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  for i in 1 2; do
    LT_LIB_PATH=build/var/vit_$v.so TAG=$v timeout -k 10 120 python -u tools/vit_time.py >> $out/vit.log 2>&1 || exit $?
  done
done
TAG=prod timeout -k 10 120 python -u tools/vit_time.py >> $out/vit.log 2>&1 || exit $?
