#!/bin/bash
# mid mode (3 marginal waves) as the explicit fused design: its parity and
# the B=256 / design tests, then call times fused (3 and 2 waves) against the
# checkpointing pair (auto) at B = 128, 192, 256
set -o pipefail
out=gpurun_out/${1:-r3mid3}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider -k "fused or design or b256 or 256" \
  > $out/par.log 2>&1 || exit $?
for r in 1 2; do
  DESIGN=fused TAG=mid3 BS=128,192,256 N=10 timeout -k 10 300 python -u tools/time_call.py >> $out/times.txt 2>&1 || exit $?
  LT_LIB_PATH=build/var/mid2.so TAG=mid2 DESIGN=fused BS=128,192,256 N=10 timeout -k 10 300 python -u tools/time_call.py >> $out/times.txt 2>&1 || exit $?
  DESIGN=auto TAG=checkpoints BS=128,192,256 N=10 timeout -k 10 300 python -u tools/time_call.py >> $out/times.txt 2>&1 || exit $?
done
