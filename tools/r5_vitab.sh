#!/bin/bash
# Viterbi build-macro variants: the GPU Viterbi tests on each build/var/vit_*.so,
# then cfg4 timings of the product and every variant, three interleaved rounds.
set -o pipefail
out=gpurun_out/r5vab; rm -rf $out; mkdir -p $out
export TMPDIR=/tmp
for v in build/var/vit_*.so; do
  LT_LIB_PATH=$v timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "viterbi or cfg4" --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $out/tests_$(basename $v .so).log 2>&1 || { tail -20 $out/tests_$(basename $v .so).log; exit 1; }
  tail -1 $out/tests_$(basename $v .so).log
done
for i in 1 2 3; do
  TAG=prod timeout -k 10 120 python -u tools/vit_time.py >> $out/vit.log 2>&1 || exit $?
  for v in build/var/vit_*.so; do
    LT_LIB_PATH=$v TAG=$(basename $v .so) timeout -k 10 120 python -u tools/vit_time.py >> $out/vit.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $out/vit.log
