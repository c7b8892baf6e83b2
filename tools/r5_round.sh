#!/bin/bash
# Round-5 GPU pass: GPU suite (full-size file verbosely), smoke, bench line and
# its kernel trace, B=256 trace, Viterbi (cfg4) trace + SQ PMC, trigram (cfg5)
# trace, FETCH/WRITE passes of the bench call, joint-step timings. Test
# failures (rc 1) continue; a crash or time limit stops the script.
set -o pipefail
out=gpurun_out/${1:-r5r}
mkdir -p $out
export TMPDIR=/tmp
R=$(pwd)
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 300 --timeout-method thread \
    -p no:cacheprovider --deselect tests/test_gpu_full_size.py -rf > $out/gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $out/gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 900 python -u -m pytest tests/test_gpu_full_size.py -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider -rf > $out/full.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $out/full.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/ktb -o run -- python bench.py --steps 20 --warmup 5 > $out/ktb.log 2>&1 || exit $?
BS=256 N=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt256 -o run -- python tools/time_call.py > $out/kt256.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/vit_time.py > $out/vit.txt 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt4 -o run -- python tools/vit_time.py > $out/kt4.log 2>&1 || exit $?
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $out/pmc4_$i -o run -- python tools/vit_time.py > $out/pmc4_$i.log 2>&1 || { rc=$?; echo "pmc4 pass $i rc=$rc" >> $out/pmc_fail.txt; exit $rc; }
done
timeout -k 10 200 python -u tools/cfg5_time.py > $out/cfg5.txt 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt5 -o run -- python tools/cfg5_time.py > $out/kt5.log 2>&1 || exit $?
(cd /tmp && N=5 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$out/pmc_fetch -o run -- \
  python3 $R/tools/chunk_prof.py > $R/$out/pmc_fetch.log 2>&1) || exit $?
(cd /tmp && N=5 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$out/pmc_write -o run -- \
  python3 $R/tools/chunk_prof.py > $R/$out/pmc_write.log 2>&1) || exit $?
HS=32,64,128,512 timeout -k 10 300 python -u tools/joint_step_bench.py > $out/joint_step.jsonl 2> $out/joint_step.err || exit $?
echo done > $out/done.txt
timeout -k 10 300 python3 -u tools/table_bench.py > $out/table_bench.jsonl 2> $out/table_bench.err || exit $?
echo done2 >> $out/done.txt
