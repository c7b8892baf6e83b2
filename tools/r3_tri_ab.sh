#!/bin/bash
# trigram loader-wave A/B: parity of the product path, cfg5 time per library
set -o pipefail
out=gpurun_out/${1:-r3tab}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "trigram or cfg5 or golden_loss_and_grad or fourgram or viterbi or vit" > $out/gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2; do
  for lib in last_torch_amd/liblt_lattice.so build/var/tri2.so build/var/tri3.so; do
    LT_LIB_PATH=$lib timeout -k 10 120 python -u tools/cfg5_time.py 2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $lib) |" >> $out/t.txt || exit 1
  done
done
timeout -k 10 120 python -u tools/vit_time.py >> $out/t.txt 2>&1 || exit $?
