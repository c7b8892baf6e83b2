#!/bin/bash
# Diagnostic GPU call: lt_loss_grad at B=256 (checkpointing pipe + marginal
# pass) and cfg5 for LT_MARG_UNITS (16-byte units per thread and tile).
set -o pipefail
for u in 5 4 3 2; do
  LT_MARG_UNITS=$u TAG=units$u BS=256 timeout -k 10 100 python3 -u tools/time_call.py || exit 1
  LT_MARG_UNITS=$u timeout -k 10 100 python3 -u tools/cfg5_time.py | sed "s/^/units$u /" || exit 1
done
