set -o pipefail
O=gpurun_out/r5j; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u tools/joint_fused_bench.py --batches 64 256 --hidden 32 64 128 --reps 10 --warmup 3 > $O/joint_step.jsonl 2> $O/jf.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o jf --output-format csv -- python3 tools/joint_fused_bench.py --batches 64 --hidden 32 --reps 5 --warmup 2 > $O/prof.jsonl 2> $O/prof.err
