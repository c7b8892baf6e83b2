#!/bin/bash
# Diagnostic GPU call: chunk parity, then lt_loss_grad timing (walk_sweep) for
# the batch sizes in BS (default 64,256).
set -o pipefail
O=gpurun_out/qa; mkdir -p $O
timeout -k 10 300 python -u tools/chunk_check.py > $O/check.log 2>&1 || { tail -30 $O/check.log; exit 1; }
tail -1 $O/check.log
BS=${BS:-64,256} timeout -k 10 200 python -u tools/walk_sweep.py > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 1; }
grep -E "nofuse|default" $O/sweep.log
if [ -f build/w4/liblt_lattice_w4.so ]; then
  echo "-- 4 waves per SIMD variant"
  LT_LIB_PATH=build/w4/liblt_lattice_w4.so BS=${BS:-64,256} timeout -k 10 200 python -u tools/walk_sweep.py > $O/sweep_w4.log 2>&1 || { tail -20 $O/sweep_w4.log; exit 1; }
  grep -E "nofuse|default" $O/sweep_w4.log
fi
