#!/bin/bash
# Viterbi A/B: the GPU Viterbi tests on the product library, then cfg4
# timings of the product library and each build/var/vit_*.so, interleaved.
set -o pipefail
out=gpurun_out/${1:-r4vab}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -k "viterbi or shortest or cfg4 or vit" --timeout 200 \
  --timeout-method thread -p no:cacheprovider -rf > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do
  TAG=prod timeout -k 10 120 python -u tools/vit_time.py >> $out/vit.log 2>&1 || exit $?
  for v in build/var/vit_*.so; do
    LT_LIB_PATH=$v TAG=$(basename $v .so) timeout -k 10 120 python -u tools/vit_time.py >> $out/vit.log 2>&1 || exit $?
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt4 -o run -- python tools/vit_time.py > $out/kt4.log 2>&1 || exit $?
echo done >> $out/vit.log
