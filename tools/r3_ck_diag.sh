#!/bin/bash
# phase C (ck_marg_kernel) at cfg2: s_memtime segments per workgroup, call
# times with role ablations (diagnostic build), and a kernel trace of the
# product call
set -o pipefail
out=gpurun_out/${1:-r3ckdiag}
mkdir -p $out
export LT_LIB_PATH=build/diag/liblt_lattice_diag.so
timeout -k 10 200 python -u tools/chunk_stamps.py > $out/stamps.txt 2>&1 || exit $?
for d in 0 4 8 12 16 28; do
  LT_CK_DBG=$d TAG=dbg$d BS=64 N=20 timeout -k 10 200 python -u tools/time_call.py >> $out/abl.txt 2>&1 || exit $?
done
unset LT_LIB_PATH
cd /tmp && export TMPDIR=/tmp
BS=64 N=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/time_call.py > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || exit $?
