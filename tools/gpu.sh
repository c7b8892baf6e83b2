#!/bin/bash
# One GPU pass, parameterised (replaces the per-round r4_* / r5_* one-offs).
#
#   tools/gpu.sh OUT STEP [STEP ...]      (run through gpurun, from the repo root)
#
# Writes under gpurun_out/OUT. Steps run in order; a test step whose tests fail
# (pytest rc 1) continues, any other failure -- a crash, an abort, a time limit --
# ends the pass there (no further GPU step runs after a fault).
#
# Steps:
#   tests      GPU suite (the full-size file apart, verbosely), then smoke()
#   full       the full-size file alone
#   k=EXPR     pytest -m gpu -k EXPR (e.g. k=cfg4)
#   bench      bench.py at the driver's flags (--warmup 5 --steps 20) and at its defaults
#   trace      rocprofv3 --kernel-trace --stats: the bench call, B=256, cfg4 Viterbi, cfg5 trigram
#   pmc        SQ counter passes of the bench call, cfg4 and cfg5; FETCH_SIZE / WRITE_SIZE of
#              the bench call (tools/chunk_prof.py) and of B=256
#   ab         per-call time of the product library and every build/var/*.so, three interleaved
#              rounds (tools/time_call.py; BS batch size, default 64)
#   vitvar     every build/var/vit_*.so: the cfg4 / long-utterance Viterbi tests
#   vart=EXPR  every build/var/*.so: pytest -m gpu -k EXPR (a variant's parity before its timing)
#   cfg5       tools/cfg5_time.py, product and every build/var/*.so interleaved
#   vit        tools/vit_time.py, product and every build/var/*.so interleaved
#   joint      tools/joint_step_bench.py (HS hidden sizes, default 32,64,128,512)
#   table      tools/table_bench.py
set -o pipefail
[ $# -ge 2 ] || { sed -n 2,30p "$0"; exit 2; }
out=gpurun_out/$1; shift
mkdir -p $out
export TMPDIR=/tmp
R=$(pwd)
PYT="python -u -m pytest --timeout 300 --timeout-method thread -p no:cacheprovider -rfs"

# a test run: rc 0 / 1 go on, anything else stops the pass
t_run() {  # t_run LOG SECONDS ARGS...
  local log=$1 sec=$2; shift 2
  timeout -k 10 $sec $PYT "$@" > $out/$log 2>&1
  local rc=$?; echo "pytest rc=$rc" >> $out/$log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
libs() { echo last_torch_amd/liblt_lattice.so; ls build/var/*.so 2>/dev/null; }
sq_passes=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR")

for step in "$@"; do
  echo "== $step $(date +%T)" >> $out/steps.txt
  case $step in
    tests)
      t_run gpu.log 600 tests -m gpu -q --maxfail=30 --deselect tests/test_gpu_full_size.py
      t_run full.log 500 tests/test_gpu_full_size.py -v
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > $out/smoke.log 2>&1 || exit $?
      ;;
    full) t_run full.log 500 tests/test_gpu_full_size.py -v ;;
    k=*) t_run k_$(echo "${step#k=}" | tr -c 'A-Za-z0-9_\n' _).log 500 tests -m gpu -v -k "${step#k=}" ;;
    bench)
      timeout -k 10 400 python -u bench.py --warmup 5 --steps 20 > $out/bench_driver_flags.json \
        2> $out/bench_driver_flags.err || exit $?
      timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || exit $?
      ;;
    trace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/ktb -o run -- python bench.py \
        --steps 20 --warmup 5 --no-joint --no-weights --cpu-utts 0 --cpu-ref-utts 0 \
        --cpu-twin-utts 0 > $out/ktb.log 2>&1 || exit $?
      BS=256 N=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt256 -o run -- \
        python tools/time_call.py > $out/kt256.log 2>&1 || exit $?
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt4 -o run -- \
        python tools/vit_time.py > $out/kt4.log 2>&1 || exit $?
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt5 -o run -- \
        python tools/cfg5_time.py > $out/kt5.log 2>&1 || exit $?
      ;;
    pmc)
      i=0
      for pmc in "${sq_passes[@]}"; do
        i=$((i+1))
        (cd /tmp && N=5 timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $R/$out/ck_sq$i \
          -o run -- python3 $R/tools/chunk_prof.py > $R/$out/ck_sq$i.log 2>&1) || exit $?
        timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $out/vit_sq$i -o run -- \
          python3 tools/vit_time.py > $out/vit_sq$i.log 2>&1 || exit $?
        N=2 WARM=1 timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $out/cfg5_sq$i \
          -o run -- python3 tools/cfg5_time.py > $out/cfg5_sq$i.log 2>&1 || exit $?
      done
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && N=5 timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $R/$out/pmc_$c \
          -o run -- python3 $R/tools/chunk_prof.py > $R/$out/pmc_$c.log 2>&1) || exit $?
        (cd /tmp && BS=256 N=5 timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv \
          -d $R/$out/pmc256_$c -o run -- python3 $R/tools/time_call.py > $R/$out/pmc256_$c.log 2>&1) || exit $?
      done
      ;;
    ab)
      for r in 1 2 3; do
        for lib in $(libs); do
          BS=${BS:-64} N=40 LT_LIB_PATH=$lib timeout -k 10 120 python3 -u tools/time_call.py \
            >> $out/ab.txt 2>&1 || exit $?
        done
      done
      ;;
    vitvar)
      for lib in build/var/vit_*.so; do
        v=$(basename $lib .so)
        LT_LIB_PATH=$lib t_run t_$v.log 300 tests/test_gpu_full_size.py -v -k "cfg4 or viterbi_long"
      done
      ;;
    vart=*)
      for lib in build/var/*.so; do
        v=$(basename $lib .so)
        LT_LIB_PATH=$lib t_run vart_$v.log 500 tests -m gpu -q -k "${step#vart=}"
      done
      ;;
    cfg5|vit)
      for r in 1 2; do
        for lib in $(libs); do
          LT_LIB_PATH=$lib TAG=$(basename $lib .so) timeout -k 10 200 python3 -u tools/${step}_time.py \
            >> $out/$step.txt 2>&1 || exit $?
        done
      done
      ;;
    joint)
      HS=${HS:-32,64,128,512} timeout -k 10 300 python -u tools/joint_step_bench.py \
        > $out/joint_step.jsonl 2> $out/joint_step.err || exit $?
      ;;
    table)
      timeout -k 10 300 python3 -u tools/table_bench.py > $out/table_bench.jsonl \
        2> $out/table_bench.err || exit $?
      ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo done >> $out/steps.txt
