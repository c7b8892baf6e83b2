#!/bin/bash
# Marginal-pass A/B: cfg5 and B=256 per-call time for the product library and
# every build/var/*.so, three interleaved rounds.
set -o pipefail
O=gpurun_out/r5mab; rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  for lib in last_torch_amd/liblt_lattice.so build/var/*.so; do
    BS=256 N=20 LT_LIB_PATH=$lib timeout -k 10 120 python3 -u tools/time_call.py >> $O/t.txt 2>&1 || { tail -20 $O/t.txt; exit 1; }
    WARM=10 N=20 LT_LIB_PATH=$lib timeout -k 10 120 python3 -u tools/cfg5_time.py 2>&1 | sed "s|^|$(basename $lib) cfg5 |" >> $O/t.txt || exit 1
  done
done
grep -v amdgpu.ids $O/t.txt
