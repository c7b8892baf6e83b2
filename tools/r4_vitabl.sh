#!/bin/bash
# Viterbi chain ablations in the diagnostic build (timing only)
set -o pipefail
out=gpurun_out/${1:-r4va}
mkdir -p $out
for d in 0 1 2 6 3 7; do
  LT_LIB_PATH=build/diag/liblt_lattice_diag.so LT_VIT_DBG=$d TAG=abl$d timeout -k 10 120 python -u tools/vit_time.py >> $out/abl.log 2>&1 || exit $?
done
timeout -k 10 120 python -u tools/vit_stamps.py >> $out/stamps.log 2>&1 || exit $?
