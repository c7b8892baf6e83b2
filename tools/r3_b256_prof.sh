#!/bin/bash
# North-star B=256: kernel trace and SQ/TCC PMC passes of pipe_kernel and
# marg_kernel (the design lt_loss_grad picks there).
set -o pipefail
out=gpurun_out/${1:-r3b256}
mkdir -p $out
export TMPDIR=/tmp
DESIGN=auto BS=256 N=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt -o run -- python tools/time_call.py > $out/kt.log 2>&1 || exit $?
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  DESIGN=auto BS=256 N=3 timeout -s KILL 120 rocprofv3 --pmc $pmc -d $out/pmc_$i -o run -- python tools/time_call.py > $out/pmc_$i.log 2>&1 || { rc=$?; echo "pmc pass $i rc=$rc" >> $out/pmc_fail.txt; exit $rc; }
done
