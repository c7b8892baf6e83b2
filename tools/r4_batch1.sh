#!/bin/bash
# round-4 batch: Viterbi (pair loader) tests + timings, producer backward
# tests + the crossover timings at small H
set -o pipefail
out=gpurun_out/${1:-r4b1}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_producer.py -q -k "viterbi or Viterbi or forward_gradients or den_forward or producer or joint or backward" --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $out/tests.log 2>&1
rc=$?; echo "rc=$rc" >> $out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  TAG=new timeout -k 10 120 python -u tools/vit_time.py >> $out/vit.log 2>&1 || exit $?
done
for d in 0 1 2 3; do
  LT_LIB_PATH=build/diag/liblt_lattice_diag.so LT_VIT_DBG=$d TAG=abl$d timeout -k 10 120 python -u tools/vit_time.py >> $out/vit.log 2>&1 || exit $?
done
HS=32,64,128 timeout -k 10 300 python -u tools/fusion_crossover.py > $out/cross.log 2>&1 || exit $?
LT_ROOT=build/ab/src HS=32,64,128 timeout -k 10 300 python -u tools/fusion_crossover.py > $out/cross_r3.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -q -k "trigram or random or golden_loss" --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $out/tri_tests.log 2>&1
rc=$?; echo "rc=$rc" >> $out/tri_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  TAG=new timeout -k 10 120 python -u tools/cfg5_time.py >> $out/cfg5.log 2>&1 || exit $?
  LT_ROOT=build/ab/src timeout -k 10 120 python -u tools/cfg5_time.py >> $out/cfg5.log 2>&1 || exit $?
done
