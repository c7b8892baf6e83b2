set -o pipefail
O=gpurun_out/r5q; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=build/diag/liblt_lattice_diag.so
for r in 1 2; do
for dn in 1 0; do
  TAG=dense$dn BS=256 N=20 LT_LIB_PATH=$D LT_MARG_DENSE=$dn timeout -k 10 120 python3 -u tools/time_call.py >> $O/t.txt 2>&1 || exit $?
done
done
LT_LIB_PATH=$D LT_MARG_DENSE=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "checkpoint" > $O/par.txt 2>&1
