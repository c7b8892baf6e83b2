#!/bin/bash
# Round-5 GPU tests: the suite (full-size file verbosely) and smoke. Test
# failures (rc 1) continue; a crash or time limit stops the script.
set -o pipefail
out=gpurun_out/${1:-r5t}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 540 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 300 --timeout-method thread \
  -p no:cacheprovider --deselect tests/test_gpu_full_size.py -rfs > $out/gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_gpu_full_size.py -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider -rf > $out/full.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
