set -o pipefail
for lds in 32768 40960 45056 49152 53248 57344 65536 81920; do
  LT_CHUNK_LDS=$lds TAG=lds$lds BS=64,128 timeout -k 10 100 python3 -u tools/time_call.py || exit 1
done
