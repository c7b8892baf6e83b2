#!/bin/bash
# Diagnostic GPU call: tools/time_call.py for the product library and each
# build/var/*.so, two interleaved rounds, one process per library.
set -o pipefail
O=gpurun_out/libab; mkdir -p $O
for r in 1 2; do
  for lib in last_torch_amd/liblt_lattice.so build/var/*.so; do
    LT_LIB_PATH=$lib timeout -k 10 120 python3 -u tools/time_call.py >> $O/t.txt 2>&1 || { tail -20 $O/t.txt; exit 1; }
    if [ "${CFG5:-0}" = 1 ]; then
      LT_LIB_PATH=$lib timeout -k 10 120 python3 -u tools/cfg5_time.py 2>&1 | sed "s|^|$(basename $lib) cfg5 |" >> $O/t.txt || exit 1
    fi
  done
done
grep ms $O/t.txt
