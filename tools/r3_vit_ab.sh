#!/bin/bash
# two-wave Viterbi: the progress store with (product) or without (vitnw) the
# LDS wait + release fence before it; the cfg4 bit-exact test on both
set -o pipefail
out=gpurun_out/${1:-r3vitab}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_full_size.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "cfg4" > $out/gpu.log 2>&1 || exit $?
LT_LIB_PATH=build/var/vitnw.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "cfg4 or viterbi or shortest" > $out/gpu_nw.log 2>&1 || exit $?
for r in 1 2; do
  TAG=wait timeout -k 10 200 python -u tools/vit_time.py >> $out/vit.txt 2>&1 || exit $?
  TAG=nowait LT_LIB_PATH=build/var/vitnw.so timeout -k 10 200 python -u tools/vit_time.py >> $out/vit.txt 2>&1 || exit $?
done
