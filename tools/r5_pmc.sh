#!/bin/bash
# SQ counter passes (one --pmc run each, within the per-block limits) of the
# cfg5 trigram call and the cfg4 Viterbi call.
set -o pipefail
out=gpurun_out/${1:-r5pmc}
mkdir -p $out
export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  N=2 WARM=1 timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $out/cfg5_$i -o run -- python3 tools/cfg5_time.py > $out/cfg5_$i.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $out/vit_$i -o run -- python3 tools/vit_time.py > $out/vit_$i.log 2>&1 || exit $?
done
echo done > $out/done.txt
