#!/bin/bash
# round-4 targeted GPU pass: table kernels + gradients, the checkpointing
# path's rounding budget (tools/ck_precision.py), the full-size parity tests
set -o pipefail
out=gpurun_out/${1:-r4t2}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_table.py tests/test_gpu_table_grad.py -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $out/table.log 2>&1
rc=$?; echo "rc=$rc" >> $out/table.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ck_precision.py 0 1 2 7 > $out/ck.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -k "full_size" --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $out/parity.log 2>&1
rc=$?; echo "rc=$rc" >> $out/parity.log
