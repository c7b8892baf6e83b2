#!/bin/bash
# Diagnostic GPU call: per-kernel durations of lt_loss_grad at the bench
# shape (B from $B, default 64), fused and unfused, for the product library
# and (if present) the variant in $VARIANT_LIB.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/kt; rm -rf $O; mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$name -o run -- python3 tools/chunk_prof.py > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }
  python3 tools/prof_stats.py $O/$name | grep "ck_" | cut -d, -f1,2,4 | sed "s/^/$name /"
}
run fused LT_CHUNK_FUSE=1 && run unfused LT_CHUNK_FUSE=0 || exit 1
if [ -n "$VARIANT_LIB" ]; then
  run vfused LT_LIB_PATH=$VARIANT_LIB LT_CHUNK_FUSE=1 && run vunfused LT_LIB_PATH=$VARIANT_LIB LT_CHUNK_FUSE=0 || exit 1
fi
if [ -n "$PMC" ]; then
  LT_CHUNK_FUSE=0 N=5 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc2 -o run -- python3 tools/chunk_prof.py > $O/pmc2.log 2>&1 || { tail -20 $O/pmc2.log; exit 1; }
  python3 tools/pmc_stats.py $O/pmc2 ck_
fi
