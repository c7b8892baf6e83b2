#!/bin/bash
# Trigram change check: the trigram GPU tests, then cfg5 lt_loss_grad time of
# the product library and each build/var/*.so, interleaved.
set -o pipefail
out=gpurun_out/${1:-r4tri}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "trigram or tri or cfg5 or n2 or random" --timeout 300 \
  --timeout-method thread -p no:cacheprovider -rf > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2 3; do
  for lib in last_torch_amd/liblt_lattice.so build/var/*.so; do
    LT_LIB_PATH=$lib timeout -k 10 120 python3 -u tools/cfg5_time.py >> $out/t.txt 2>&1 || exit $?
  done
done
