#!/bin/bash
# Round-3 GPU pass: the whole GPU suite, then the full-size parity file
# verbosely, then the realistic-weight sweep (with per-element error) and
# optionally the bench. Test failures (rc 1) continue; a crash or a time
# limit stops the call.
set -o pipefail
out=gpurun_out/${1:-r3b}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
  -p no:cacheprovider --deselect tests/test_gpu_full_size.py > $out/gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_full_size.py -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $out/full.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/weights_sweep.py --err > $out/ws.jsonl 2> $out/ws.err || exit $?
if [ -n "$2" ]; then
  timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err
fi
