#!/bin/bash
set -o pipefail
out=gpurun_out/${1:-r4t4}
mkdir -p $out
timeout -k 10 300 python -u tools/fld_precision.py 2 > $out/fld.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ck_precision.py 0 1 > $out/ck.log 2>&1 || exit $?
