set -o pipefail
O=gpurun_out/r5w; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=build/diag/liblt_lattice_diag.so
for r in 1 2; do
for m in 1 2 0; do
  TAG=nmode$m BS=256 N=20 LT_LIB_PATH=$D LT_MARG_NMODE=$m timeout -k 10 120 python3 -u tools/time_call.py >> $O/t.txt 2>&1 || exit $?
  TAG=nmode$m LT_LIB_PATH=$D LT_MARG_NMODE=$m timeout -k 10 120 python3 -u tools/cfg5_time.py >> $O/t.txt 2>&1 || exit $?
done
done
LT_LIB_PATH=$D LT_MARG_NMODE=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_full_size.py -k "checkpoint or b256 or cfg5 or trigram or marg" > $O/par.txt 2>&1
