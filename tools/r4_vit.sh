#!/bin/bash
# round-4 Viterbi: the bit-exact Viterbi tests, A/B timing vs round 3, stamps
set -o pipefail
out=gpurun_out/${1:-r4v}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -q -k "viterbi or Viterbi or forward_gradients or den_forward" --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $out/tests.log 2>&1
rc=$?; echo "rc=$rc" >> $out/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  TAG=new timeout -k 10 120 python -u tools/vit_time.py >> $out/ab.log 2>&1 || exit $?
  LT_ROOT=build/ab/src TAG=r3 timeout -k 10 120 python -u tools/vit_time.py >> $out/ab.log 2>&1 || exit $?
done
timeout -k 5 120 python tools/vit_stamps.py > $out/stamps.log 2>&1
