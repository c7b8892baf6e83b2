# cfg5: per-call times, product and diagnostic build under LT_TRI_MIX_DBG values in D
set -o pipefail
O=gpurun_out/${1:-r6s}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python -u tools/cfg5_time.py 2>&1 | grep -v amdgpu.ids >> $O/t.txt || exit $?
  for d in ${D:-0}; do
    LT_TRI_MIX_DBG=$d LT_LIB_PATH=build/diag/liblt_lattice_diag.so timeout -k 10 200 python -u tools/cfg5_time.py 2>&1 | grep -v amdgpu.ids | sed "s/^/dbg=$d /" >> $O/t.txt || exit $?
  done
done
