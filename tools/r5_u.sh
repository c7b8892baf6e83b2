set -o pipefail
O=gpurun_out/r5u; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=build/diag/liblt_lattice_diag.so
for r in 1 2; do
for u in 5 4 3 2; do
  TAG=units$u BS=256 N=20 LT_LIB_PATH=$D LT_MARG_UNITS=$u timeout -k 10 120 python3 -u tools/time_call.py >> $O/t.txt 2>&1 || exit $?
done
done
for u in 5 3; do
  TAG=cfg5_units$u LT_LIB_PATH=$D LT_MARG_UNITS=$u timeout -k 10 120 python3 -u tools/cfg5_time.py >> $O/t.txt 2>&1 || exit $?
done
