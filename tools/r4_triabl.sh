#!/bin/bash
# Trigram (cfg5) role ablations in the diagnostic build (LT_DBG bits: 1 skip
# den compute, 2 skip numerator, 4 loaders issue nothing, 8 no barrier);
# timing only, the results are wrong by design. Kernel trace of each.
set -o pipefail
out=gpurun_out/${1:-r4ta}
mkdir -p $out
D=build/diag/liblt_lattice_diag.so
for d in 0 16 32 1 2 4 5 3 7; do
  LT_LIB_PATH=$D LT_DBG=$d timeout -k 10 120 python3 -u tools/cfg5_time.py 2>&1 | sed "s/^/dbg=$d /" >> $out/t.txt || exit 1
done
for d in 0 16 32; do
  LT_LIB_PATH=$D LT_DBG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt$d -o run -- python3 tools/cfg5_time.py > $out/kt$d.log 2>&1 || exit 1
done
