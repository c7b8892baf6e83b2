#!/bin/bash
# Diagnostic: kernel times of the chunked path for walk ring depths
# (build/var/w<N>.so, diagnostic builds) fused into A's launch and unfused
# (LT_CHUNK_FUSE=0: ck_combine_kernel after A).
set -o pipefail
out=gpurun_out/${1:-wd}
mkdir -p $out
export TMPDIR=/tmp
for n in ${SLOTS:-3 6 9}; do
  for fu in 1 0; do
    LT_LIB_PATH=build/var/w$n.so LT_CHUNK_FUSE=$fu DESIGN=chunk BS=${BS:-64} N=10 TAG=w$n-f$fu \
      timeout -k 10 120 rocprofv3 --kernel-trace -d $out/w$n-f$fu -o run -- python -u tools/time_call.py >> $out/times.txt 2>&1 || exit $?
  done
done
