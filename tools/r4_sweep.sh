#!/bin/bash
set -o pipefail
out=gpurun_out/${1:-r4sw}
mkdir -p $out
D=build/diag/liblt_lattice_diag.so
TAG=prod timeout -k 10 120 python3 -u tools/time_call.py >> $out/t.txt 2>&1 || exit $?
TAG=diag LT_LIB_PATH=$D timeout -k 10 120 python3 -u tools/time_call.py >> $out/t.txt 2>&1 || exit $?
for L in 4 5 7 8; do
  TAG=len$L LT_LIB_PATH=$D LT_CHUNK_LEN=$L LT_CHUNK_LDS=98304 timeout -k 10 120 python3 -u tools/time_call.py >> $out/t.txt 2>&1 || exit $?
done
for A in 0 10 40 60; do
  TAG=walk$A LT_LIB_PATH=$D LT_CHUNK_WALK_AT=$A timeout -k 10 120 python3 -u tools/time_call.py >> $out/t.txt 2>&1 || exit $?
done
for P in 4096 8192; do
  TAG=pad$P LT_LIB_PATH=$D LT_CK_LDS_PAD=$P timeout -k 10 120 python3 -u tools/time_call.py >> $out/t.txt 2>&1 || exit $?
done
TAG=diag LT_LIB_PATH=$D timeout -k 10 120 python3 -u tools/time_call.py >> $out/t.txt 2>&1 || exit $?
echo done >> $out/t.txt
