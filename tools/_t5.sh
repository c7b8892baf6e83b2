# cfg5 kernel traces: the product library, the previous commit's (build/var/base.so) and
# the diagnostic build at each LT_TRI_MIX_DBG value in D (default "1 2")
set -o pipefail
O=gpurun_out/${1:-r6j}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt5 -o run -- python tools/cfg5_time.py > $O/kt5.log 2>&1 || exit $?
LT_LIB_PATH=build/var/base.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt5b -o run -- python tools/cfg5_time.py > $O/kt5b.log 2>&1 || exit $?
for d in ${D:-1 2}; do
  LT_TRI_MIX_DBG=$d LT_LIB_PATH=build/diag/liblt_lattice_diag.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
    -d $O/kt5d$d -o run -- python tools/cfg5_time.py > $O/kt5d$d.log 2>&1 || exit $?
done
for d in kt5 kt5b $(for d in ${D:-1 2}; do echo kt5d$d; done); do echo "== $d"; tail -1 $O/$d.log; python3 tools/prof_stats.py $O/$d; done > $O/stats.txt 2>&1
