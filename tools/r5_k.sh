set -o pipefail
O=gpurun_out/r5k; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u tools/clock_probe.py > $O/clock.jsonl 2> $O/clock.err || exit $?
(rocm-smi --showclocks > $O/smi_clocks.txt 2>&1 || true)
