#!/bin/bash
# A/B: lt_loss_grad call time of the in-tree library against build/var/old.so
# (same box, interleaved), then the phase-C stamps of the diagnostic build.
set -o pipefail
out=gpurun_out/${1:-ab}
mkdir -p $out
for i in 1 2; do
  BS=${BS:-64,256} N=20 TAG=new timeout -k 10 200 python -u tools/time_call.py >> $out/times.txt 2>&1 || exit $?
  LT_LIB_PATH=build/var/old.so BS=${BS:-64,256} N=20 TAG=old timeout -k 10 200 python -u tools/time_call.py >> $out/times.txt 2>&1 || exit $?
done
