#!/bin/bash
# Trigram den roles + NW-wave Viterbi: parity tests on both paths, cfg5 time,
# Viterbi cfg4 times for the product (NW = 2) and build/var/vit{1,4}.so,
# kernel trace + SQ PMC of the trigram call.
set -o pipefail
out=gpurun_out/${1:-r3m}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "trigram or cfg5 or golden_loss_and_grad or fourgram or viterbi or vit" > $out/gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/cfg5_time.py > $out/cfg5.txt 2>&1 || exit $?
for r in 1 2; do
  for lib in last_torch_amd/liblt_lattice.so build/var/vit1.so build/var/vit4.so; do
    TAG=$(basename $lib) LT_LIB_PATH=$lib timeout -k 10 120 python -u tools/vit_time.py >> $out/vit.txt 2>&1 || exit $?
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt5 -o run -- python tools/cfg5_time.py > $out/kt5.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt4 -o run -- python tools/vit_time.py > $out/kt4.log 2>&1 || exit $?
bash tools/r3_b256_prof.sh ${1:-r3m}_b256 || exit $?
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $out/pmc5_$i -o run -- python tools/cfg5_time.py > $out/pmc5_$i.log 2>&1 || { rc=$?; echo "pmc pass $i rc=$rc" >> $out/pmc_fail.txt; exit $rc; }
done
