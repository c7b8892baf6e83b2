#!/bin/bash
# round 3: trigram marginal-pass parity + cfg5 time and kernel trace (the
# branch-free marg_tile den loop), then the producer fusion crossover
set -o pipefail
out=gpurun_out/${1:-r3x}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "trigram or cfg5 or golden_loss_and_grad or fourgram or den_grad or loss_grad" > $out/gpu.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/cfg5_time.py > $out/cfg5.txt 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt5 -o run -- python tools/cfg5_time.py > $out/kt5.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/fusion_crossover.py > $out/crossover.jsonl 2>&1 || exit $?
