#!/bin/bash
# B=256 (the north star, checkpointing pair) per-call time for the product
# library and the pipe nap variants, three interleaved rounds.
set -o pipefail
O=gpurun_out/r5nap; rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  for lib in last_torch_amd/liblt_lattice.so build/var/*.so; do
    BS=256 N=40 LT_LIB_PATH=$lib timeout -k 10 120 python3 -u tools/time_call.py >> $O/t.txt 2>&1 || { tail -20 $O/t.txt; exit 1; }
  done
done
cat $O/t.txt
