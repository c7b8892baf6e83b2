#!/bin/bash
# Round-3 profile pass: per-design call times, kernel traces (B=64 auto,
# B=256 auto and chunk) and SQ PMC passes on the chunked kernels at B=64.
set -o pipefail
out=gpurun_out/${1:-r3p}
mkdir -p $out
export TMPDIR=/tmp
rocprofv3 -L > $out/counters.txt 2>&1 || true
for d in auto chunk checkpoints; do
  DESIGN=$d BS=64,128,192,256 N=10 timeout -k 10 300 python -u tools/time_call.py >> $out/times.txt 2>&1 || exit $?
done
DESIGN=auto BS=64 N=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt64 -o run -- python tools/time_call.py > $out/kt64.log 2>&1 || exit $?
DESIGN=auto BS=256 N=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt256 -o run -- python tools/time_call.py > $out/kt256.log 2>&1 || exit $?
DESIGN=chunk BS=256 N=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt256c -o run -- python tools/time_call.py > $out/kt256c.log 2>&1 || exit $?
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  DESIGN=auto BS=64 N=3 timeout -s KILL 120 rocprofv3 --pmc $pmc -d $out/pmc$i -o run -- python tools/time_call.py > $out/pmc$i.log 2>&1 || { rc=$?; echo "pmc pass $i rc=$rc" >> $out/pmc_fail.txt; exit $rc; }
done
