#!/bin/bash
# Trigram mid mode: parity (ragged + cfg5 + parity-file trigram cases), then
# cfg5 timing with and without the workers (diag build, LT_TRI_MID) and a
# kernel trace.
set -o pipefail
out=gpurun_out/${1:-r4mid}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "trigram" -rf > $out/t_full.log 2>&1
rc=$?; echo "rc=$rc" >> $out/t_full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "32-2 or trigram or n2" -rf > $out/t_par.log 2>&1
rc=$?; echo "rc=$rc" >> $out/t_par.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 120 python -u tools/cfg5_time.py >> $out/cfg5.txt 2>&1 || exit $?
  LT_LIB_PATH=build/diag/liblt_lattice_diag.so LT_TRI_MID=0 timeout -k 10 120 python -u tools/cfg5_time.py >> $out/cfg5.txt 2>&1 || exit $?
  LT_LIB_PATH=build/diag/liblt_lattice_diag.so LT_TRI_MID=1 timeout -k 10 120 python -u tools/cfg5_time.py >> $out/cfg5.txt 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt5 -o run -- python tools/cfg5_time.py > $out/kt5.log 2>&1 || exit $?
