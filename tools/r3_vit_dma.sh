#!/bin/bash
# Viterbi A/B: the product library against a variant build (build/var/vitbp2.so:
# two backpointer waves); bit-exact tests on both, times, chain stamps
set -o pipefail
out=gpurun_out/${1:-r3vitdma}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "cfg4 or viterbi or shortest or vit or max_tropical or golden" > $out/gpu.log 2>&1 || exit $?
LT_LIB_PATH=build/var/vitbp2.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "cfg4 or viterbi or shortest" > $out/gpu_var.log 2>&1 || exit $?
for r in 1 2; do
  TAG=product timeout -k 10 200 python -u tools/vit_time.py >> $out/vit.txt 2>&1 || exit $?
  TAG=variant LT_LIB_PATH=build/var/vitbp2.so timeout -k 10 200 python -u tools/vit_time.py >> $out/vit.txt 2>&1 || exit $?
done
timeout -k 10 200 python -u tools/vit_stamps.py > $out/stamps.txt 2>&1 || exit $?
