#!/bin/bash
# Chunked-scan change check: the GPU suite (full-size file too), then the
# bench-shape call time of the product library against build/var/*.so,
# interleaved (tools/lib_ab.sh).
set -o pipefail
out=gpurun_out/${1:-r4ck}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 300 --timeout-method thread \
  -p no:cacheprovider -rf > $out/gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2 3; do
  for lib in last_torch_amd/liblt_lattice.so build/var/*.so; do
    LT_LIB_PATH=$lib timeout -k 10 120 python3 -u tools/time_call.py >> $out/t.txt 2>&1 || exit $?
  done
done
echo done >> $out/t.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt -o run -- python tools/chunk_prof.py > $out/kt.log 2>&1 || exit $?
