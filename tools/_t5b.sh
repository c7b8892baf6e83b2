# cfg5: the overlap's timeline under diagnostic modes (DBG values in D; LIB2: a second library, DBG 0)
set -o pipefail
O=gpurun_out/${1:-r6p}; mkdir -p $O
for d in ${D:-0 2 32}; do
  DBG=$d timeout -k 10 200 python -u tools/tri_mix_timeline.py > $O/tl_$d.txt 2>&1 || exit $?
done
if [ -n "$LIB2" ]; then
  LT_LIB_PATH=$LIB2 timeout -k 10 200 python -u tools/tri_mix_timeline.py > $O/tl_lib2.txt 2>&1 || exit $?
fi
