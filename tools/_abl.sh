set -o pipefail
O=gpurun_out/r6c; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
D=${D:-0,1024,2048,3072,4,8,12,16,28}
DBGS=$D timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/chunk_ablate.py > $O/abl.txt 2>&1 || exit $?
f=$(find $O/kt -name "*kernel_trace.csv" | head -1); python3 tools/ck_abl_trace.py $f $D > $O/abl_kernels.txt 2>&1
