set -o pipefail
O=gpurun_out/r5p; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u tools/table_bench.py > $O/table_bench.jsonl 2> $O/tb.err || exit $?
ONLY=fld2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o fld2 --output-format csv -- python3 tools/table_bench.py > $O/trace.txt 2>&1 || exit $?
ONLY=fld2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o fld2 --output-format csv -- python3 tools/table_bench.py > $O/pf.txt 2>&1 || exit $?
ONLY=fld2 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o fld2 --output-format csv -- python3 tools/table_bench.py > $O/pw.txt 2>&1
