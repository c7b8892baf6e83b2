set -o pipefail
# Diagnostic GPU call: lt_loss_grad time (tools/time_call.py) across phase-C LDS budgets
# (LT_CHUNK_LDS, i.e. chunk lengths), B=64 and B=128.
for lds in 32768 40960 45056 49152 53248 57344 65536 81920; do
  LT_CHUNK_LDS=$lds TAG=lds$lds BS=64,128 timeout -k 10 100 python3 -u tools/time_call.py || exit 1
done
