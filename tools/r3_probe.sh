#!/bin/bash
# Round-3 probe: full-size parity under the per-element marginal bound, the
# realistic-weight sweep and the bench, in one GPU call. Test failures
# (rc 1) continue; a crash or a time limit stops the call.
set -o pipefail
out=gpurun_out/${1:-r3a}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_full_size.py -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $out/full.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/weights_sweep.py --err > $out/ws.jsonl 2> $out/ws.err || exit $?
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err
