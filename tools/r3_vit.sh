#!/bin/bash
# two-wave Viterbi (chain / backpointers) and the per-slice marginal tiles:
# parity (bit-exact Viterbi, trigram and golden loss + grad), then cfg4 times
# against the one-wave kernel (build/var/vit1.so) and cfg5 times, kernel trace
set -o pipefail
out=gpurun_out/${1:-r3vit}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "viterbi or shortest or vit or cfg4 or trigram or cfg5 or golden or den_grad or loss_grad or north_star" > $out/gpu.log 2>&1 || exit $?
for r in 1 2; do
  TAG=split timeout -k 10 200 python -u tools/vit_time.py >> $out/vit.txt 2>&1 || exit $?
  TAG=one LT_LIB_PATH=build/var/vit1.so timeout -k 10 200 python -u tools/vit_time.py >> $out/vit.txt 2>&1 || exit $?
  timeout -k 10 200 python -u tools/cfg5_time.py >> $out/cfg5.txt 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/ktv -o run -- python tools/vit_time.py > $out/ktv.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt5 -o run -- python tools/cfg5_time.py > $out/kt5.log 2>&1 || exit $?
