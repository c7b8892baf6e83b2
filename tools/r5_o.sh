set -o pipefail
O=gpurun_out/r5o; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_diag.py tests/test_gpu_parity.py -k "trigram or diag or random_checkpointing" > $O/t.txt 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/cfg5_time.py > $O/cfg5.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_full_size.py -k cfg5 > $O/cfg5_test.txt 2>&1
