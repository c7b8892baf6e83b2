#!/bin/bash
# Viterbi after the publish/poll change: the full-size file (cfg4 every
# utterance, T=2400/4500 routes) and the parity file's Viterbi cases, timing,
# kernel trace and the two SQ passes.
set -o pipefail
out=gpurun_out/${1:-r5vit}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_full_size.py tests/test_gpu_parity.py -q -k "viterbi or cfg4 or shortest" --timeout 280 --timeout-method thread -p no:cacheprovider > $out/t.log 2>&1 || exit $?
for i in 1 2 3; do timeout -k 10 120 python -u tools/vit_time.py >> $out/vit.log 2>&1 || exit $?; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt4 -o run --output-format csv -- python tools/vit_time.py > $out/kt4.log 2>&1 || exit $?
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $out/vit_$i -o run -- python3 tools/vit_time.py > $out/vit_$i.log 2>&1 || exit $?
done
echo done > $out/done.txt
