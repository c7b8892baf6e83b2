#!/bin/bash
# Where phase C's time goes at the bench shape: role ablations and s_memtime
# marks (diagnostic build), then two SQ PMC passes of the product call.
set -o pipefail
out=gpurun_out/r5ck; rm -rf $out; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/chunk_stamps.py > $out/stamps.txt 2>&1 || exit $?
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  N=5 timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $out/ck_$i -o run -- python3 tools/time_call.py > $out/ck_$i.log 2>&1 || exit $?
done
echo done > $out/done.txt
