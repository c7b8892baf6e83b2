set -o pipefail
O=gpurun_out/r5z; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=build/diag/liblt_lattice_diag.so
for r in 1 2 3; do
for x in 1 0; do
  TAG=xcd$x LT_LIB_PATH=$D LT_MARG_XCD=$x timeout -k 10 120 python3 -u tools/cfg5_time.py >> $O/t.txt 2>&1 || exit $?
done
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_full_size.py -k "checkpoint or cfg5 or trigram" > $O/par.txt 2>&1
