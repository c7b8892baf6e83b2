set -o pipefail
O=gpurun_out/r5y; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $O/full.log 2>&1
