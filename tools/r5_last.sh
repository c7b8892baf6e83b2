#!/bin/bash
# Last check of the round: GPU suite, full-size file, smoke, and the bench at
# the driver's flags.
set -o pipefail
out=gpurun_out/r5last; rm -rf $out; mkdir -p $out
export TMPDIR=/tmp
tools/r5_tests.sh r5last || exit $?
timeout -k 10 400 python -u bench.py --warmup 5 --steps 20 > $out/bench_driver_flags.json 2> $out/bench.err || exit $?
echo done > $out/done.txt
