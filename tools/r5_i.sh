set -o pipefail
O=gpurun_out/r5i; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u tools/joint_stamps.py > $O/stamps.txt 2>&1
