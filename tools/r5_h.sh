set -o pipefail
O=gpurun_out/r5h; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_joint_fused.py > $O/joint.txt 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/joint_stamps.py > $O/stamps.txt 2>&1 || exit $?
timeout -k 10 300 python3 tools/joint_fused_bench.py --batches 64 256 --hidden 32 128 --reps 5 --warmup 2 > $O/jf.jsonl 2> $O/jf.err
