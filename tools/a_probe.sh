#!/bin/bash
# Diagnostic GPU call: chunk parity, lt_loss_grad timing (B=64), phase C
# stamps, and one PMC pass of SQ counters over the unfused phase-A launch.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ap; mkdir -p $O
timeout -k 10 300 python -u tools/chunk_check.py > $O/check.log 2>&1 || { tail -30 $O/check.log; exit 1; }
tail -2 $O/check.log
BS=64 timeout -k 10 120 python -u tools/walk_sweep.py > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 1; }
head -3 $O/sweep.log
timeout -k 10 100 python -u tools/chunk_stamps.py > $O/stamps_c.log 2>&1 || { tail -20 $O/stamps_c.log; exit 1; }
cat $O/stamps_c.log
rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" $O/counters.txt | sort -u | tr '\n' ' ' > $O/sq_counters.txt || true
echo
LT_CHUNK_FUSE=0 N=5 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA --output-format csv -d $O/pmc1 -o run -- python3 tools/chunk_prof.py > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 1; }
echo done
