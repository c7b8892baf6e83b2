#!/bin/bash
# Trigram den roles (lt_tri.hip): parity tests touching the trigram
# checkpointing path, cfg5 timing, kernel trace + PMC of the new kernel.
set -o pipefail
out=gpurun_out/${1:-r3tri2}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "trigram or cfg5 or golden_loss_and_grad or fourgram" > $out/gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/cfg5_time.py > $out/cfg5.txt 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt5 -o run -- python tools/cfg5_time.py > $out/kt5.log 2>&1 || exit $?
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $out/pmc5_$i -o run -- python tools/cfg5_time.py > $out/pmc5_$i.log 2>&1 || { rc=$?; echo "pmc pass $i rc=$rc" >> $out/pmc_fail.txt; exit $rc; }
done
