#!/bin/bash
# Split staging in phase C: chunk-path GPU tests on the variant library
# (LT_LIB_PATH), then the A/B timing against the product.
set -o pipefail
out=gpurun_out/r5split; rm -rf $out; mkdir -p $out
export TMPDIR=/tmp
LT_LIB_PATH=build/var/chunk_split1.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_api.py tests/test_gpu_graph.py -m gpu -q -x \
  -k "chunk or grad or cfg2 or loss" --timeout 120 --timeout-method thread -p no:cacheprovider > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -2 $out/t.log
tools/r5_ab.sh
