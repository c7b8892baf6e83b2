#!/bin/bash
set -o pipefail
out=gpurun_out/${1:-r3c}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
  -p no:cacheprovider --deselect tests/test_gpu_full_size.py > $out/gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_full_size.py -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $out/full.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/vit_time.py > $out/vit.txt 2>&1 || exit $?
bash tools/r3_prof.sh $1p
