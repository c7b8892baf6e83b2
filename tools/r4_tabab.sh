#!/bin/bash
# Table-kernel change check: the table / general-lattice GPU tests, then
# tools/table_bench.py for the product library and build/var/*.so.
set -o pipefail
out=gpurun_out/${1:-r4tab}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_table.py tests/test_gpu_table_grad.py tests/test_gpu_api.py -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for lib in last_torch_amd/liblt_lattice.so build/var/*.so; do
  echo "== $lib" >> $out/t.jsonl
  LT_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/table_bench.py >> $out/t.jsonl 2>> $out/err.txt || exit $?
done
