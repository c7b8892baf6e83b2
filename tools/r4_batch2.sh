#!/bin/bash
# round-4 batch 2: Viterbi (weights two deep) + producer backward (parallel reduce)
set -o pipefail
out=gpurun_out/${1:-r4b2}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_producer.py -q -k "viterbi or Viterbi or forward_gradients or den_forward or producer or joint or backward" --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $out/tests.log 2>&1
rc=$?; echo "rc=$rc" >> $out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do
  TAG=new timeout -k 10 120 python -u tools/vit_time.py >> $out/vit.log 2>&1 || exit $?
done
HS=32,64,128 timeout -k 10 300 python -u tools/fusion_crossover.py > $out/cross.log 2>&1 || exit $?
