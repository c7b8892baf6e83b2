set -o pipefail
mkdir -p gpurun_out/r5g
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u tools/joint_stamps.py > gpurun_out/r5g/stamps.txt 2>&1
