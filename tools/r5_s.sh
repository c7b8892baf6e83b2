set -o pipefail
O=gpurun_out/r5s; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
LT_LIB_PATH=build/diag/liblt_lattice_diag.so timeout -k 10 200 python3 -u tools/vit_stamps.py > $O/vst.txt 2>&1
