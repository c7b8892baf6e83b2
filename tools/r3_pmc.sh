#!/bin/bash
# Round-3 HBM traffic of the bench call (cfg2 lt_loss_grad): FETCH_SIZE and
# WRITE_SIZE in separate passes (MI355X_MICROARCH.md), summarised by
# tools/pmc_summary.py into profiles/r03_pmc_summary.json afterwards
set -o pipefail
out=gpurun_out/${1:-r3pmc}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
N=5 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$out/pmc_fetch -o run -- \
  python3 $R/tools/chunk_prof.py > $R/$out/pmc_fetch.log 2>&1 || exit $?
N=5 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$out/pmc_write -o run -- \
  python3 $R/tools/chunk_prof.py > $R/$out/pmc_write.log 2>&1 || exit $?
