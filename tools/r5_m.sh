set -o pipefail
O=gpurun_out/r5m; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o cfg5 --output-format csv -- python3 tools/cfg5_time.py > $O/cfg5.txt 2>&1
