set -o pipefail
mkdir -p gpurun_out/r5f
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_joint_fused.py > gpurun_out/r5f/joint.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f/prof -o jf --output-format csv -- python3 tools/joint_fused_bench.py --batches 64 --hidden 32 128 --reps 3 --warmup 1 > gpurun_out/r5f/jf.jsonl 2> gpurun_out/r5f/jf.err
