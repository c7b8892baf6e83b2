set -o pipefail
O=gpurun_out/r5r; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > $O/bench_driver_flags.json 2> $O/b1.err || exit $?
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --settle-ms 0 > $O/bench_nosettle.json 2> $O/b2.err
