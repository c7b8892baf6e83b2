set -o pipefail
mkdir -p gpurun_out/r5e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5e/prof -o jf -- python3 tools/joint_fused_bench.py --batches 64 --hidden 32 128 --reps 3 --warmup 1 > gpurun_out/r5e/jf.jsonl 2> gpurun_out/r5e/jf.err
r=$?
find gpurun_out/r5e/prof -name "*stats*" | head
exit $r
