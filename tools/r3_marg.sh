#!/bin/bash
# marginal pass: one workgroup per trigram frame (slices in turn over one row
# load). Parity of every marg_kernel user, then cfg5 and B=256 call times for
# the product (prefetching the next slice) and build/var/nopf.so
set -o pipefail
out=gpurun_out/${1:-r3marg}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "trigram or cfg5 or golden or fourgram or den_grad or loss_grad or north_star or two-call or recursion or table" > $out/gpu.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python -u tools/cfg5_time.py >> $out/cfg5.txt 2>&1 || exit $?
  LT_LIB_PATH=build/var/nopf.so timeout -k 10 200 python -u tools/cfg5_time.py >> $out/cfg5_nopf.txt 2>&1 || exit $?
  DESIGN=auto TAG=product BS=64,256 N=10 timeout -k 10 300 python -u tools/time_call.py >> $out/times.txt 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt5 -o run -- python tools/cfg5_time.py > $out/kt5.log 2>&1 || exit $?
BS=256 N=10 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt256 -o run -- python tools/time_call.py > $out/kt256.log 2>&1 || exit $?
