#!/bin/bash
# Mid-mode fused pipe (in-workgroup marginals): parity on the fused design,
# the design query, the full-size B=256 tests, call times per batch size.
set -o pipefail
out=gpurun_out/${1:-r3mid}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "fused" > $out/par.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/par.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "design_query or b256 or 256" > $out/full.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for d in auto checkpoints; do
  DESIGN=$d BS=128,192,256,384 N=10 timeout -k 10 300 python -u tools/time_call.py >> $out/times.txt 2>&1 || exit $?
done
DESIGN=auto BS=256 N=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt -o run -- python tools/time_call.py > $out/kt.log 2>&1 || exit $?
