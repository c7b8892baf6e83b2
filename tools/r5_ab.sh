#!/bin/bash
# Per-call time (tools/time_call.py) of the product library and every
# build/var/*.so, three interleaved rounds, at batch sizes BS (default 64).
set -o pipefail
O=gpurun_out/r5ab; rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  for lib in last_torch_amd/liblt_lattice.so build/var/*.so; do
    BS=${BS:-64} N=40 LT_LIB_PATH=$lib timeout -k 10 120 python3 -u tools/time_call.py >> $O/t.txt 2>&1 || { tail -20 $O/t.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/t.txt
