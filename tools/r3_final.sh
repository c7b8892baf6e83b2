#!/bin/bash
# last GPU call of round 3: the two-backpointer-wave Viterbi A/B, then the
# full round pass (GPU suite, full-size tests, bench, smoke, kernel traces)
set -o pipefail
bash tools/r3_vit_dma.sh r3vitbp2 || exit $?
bash tools/r3_round.sh r3g || exit $?
