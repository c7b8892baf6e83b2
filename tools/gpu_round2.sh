#!/bin/bash
# One GPU call: GPU tests, the bench, its kernel trace and the PMC passes of
# the timed launch. Outputs under gpurun_out/r02/; summaries are copied into
# profiles/ afterwards (tools/pmc_summary.py, tools/prof_stats.py).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step tests
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $OUT/gputest.log 2>&1 || { tail -30 $OUT/gputest.log; exit 1; }
  tail -3 $OUT/gputest.log
fi
step bench
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
step trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --steps 10 \
  --no-north-star --no-joint --cpu-utts 0 --cpu-ref-utts 0 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
step trace b256
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace256 -o run -- python3 bench.py --batch 256 \
  --steps 10 --no-north-star --no-joint --cpu-utts 0 --cpu-ref-utts 0 > $OUT/trace256.log 2>&1 || { tail -20 $OUT/trace256.log; exit 1; }
step pmc fetch
N=5 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  python3 tools/chunk_prof.py > $OUT/pmc_fetch.log 2>&1 || { tail -20 $OUT/pmc_fetch.log; exit 1; }
step pmc write
N=5 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  python3 tools/chunk_prof.py > $OUT/pmc_write.log 2>&1 || { tail -20 $OUT/pmc_write.log; exit 1; }

step configs
timeout -k 10 300 python3 -u tools/configs_bench.py > $OUT/configs.jsonl 2> $OUT/configs.err || { tail -20 $OUT/configs.err; exit 1; }
cat $OUT/configs.jsonl
step done
