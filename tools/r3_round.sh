#!/bin/bash
# Round-3 GPU pass: GPU suite (full-size file verbosely), bench line, kernel
# trace of the bench. Test failures (rc 1) continue; a crash or time limit stops.
set -o pipefail
out=gpurun_out/${1:-r3d}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
  -p no:cacheprovider --deselect tests/test_gpu_full_size.py > $out/gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_full_size.py -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $out/full.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/ktb -o run -- python bench.py --steps 20 --warmup 5 > $out/ktb.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit $?
BS=256 N=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt256 -o run -- python tools/time_call.py > $out/kt256.log 2>&1 || exit $?
