#!/bin/bash
# Round-5 measurement pass: the bench line at the driver's flags and at the
# defaults, its kernel trace, B=256 trace, Viterbi (cfg4) and trigram (cfg5)
# traces, FETCH/WRITE passes of the bench call.
set -o pipefail
out=gpurun_out/${1:-r5b}
mkdir -p $out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > $out/bench_driver_flags.json 2> $out/bench1.err || exit $?
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ktb -o run --output-format csv -- python bench.py --steps 20 --warmup 5 > $out/ktb.log 2>&1 || exit $?
BS=256 N=10 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt256 -o run --output-format csv -- python tools/time_call.py > $out/kt256.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/vit_time.py > $out/vit.txt 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt4 -o run --output-format csv -- python tools/vit_time.py > $out/kt4.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/cfg5_time.py > $out/cfg5.txt 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt5 -o run --output-format csv -- python tools/cfg5_time.py > $out/kt5.log 2>&1 || exit $?
(cd /tmp && N=5 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$out/pmc_fetch -o run -- \
  python3 $R/tools/chunk_prof.py > $R/$out/pmc_fetch.log 2>&1) || exit $?
(cd /tmp && N=5 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$out/pmc_write -o run -- \
  python3 $R/tools/chunk_prof.py > $R/$out/pmc_write.log 2>&1) || exit $?
echo done > $out/done.txt
