#!/bin/bash
# Diagnostic GPU call: per-kernel durations (rocprofv3 kernel trace of
# tools/chunk_prof.py) for the product library and each build/var/*.so,
# fused and unfused, on one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/vt; rm -rf $O; mkdir -p $O
for lib in last_torch_amd/liblt_lattice.so build/var/*.so; do
  n=$(basename $lib .so)
  for F in 1 0; do
    LT_LIB_PATH=$lib LT_CHUNK_FUSE=$F timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$n$F -o run -- python3 tools/chunk_prof.py > $O/$n$F.log 2>&1 || { tail -20 $O/$n$F.log; exit 1; }
    python3 tools/prof_stats.py $O/$n$F | grep "ck_" | cut -d, -f1,4 | sed "s/^/$n fuse=$F /"
  done
done
