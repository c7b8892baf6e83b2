# Diagnostic GPU call: chunk parity (tools/chunk_check.py), then kernel traces
# of lt_loss_grad at B=64 and B=256, fused (LT_CHUNK_FUSE=1) and unfused.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fz; mkdir -p $O
timeout -k 10 300 python -u tools/chunk_check.py > $O/check.log 2>&1 || { tail -30 $O/check.log; exit 1; }
tail -3 $O/check.log
for F in 1 0; do
  export LT_CHUNK_FUSE=$F
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t$F -o run -- python3 tools/chunk_prof.py > $O/t$F.log 2>&1 || { tail -20 $O/t$F.log; exit 1; }
  B=256 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/b$F -o run -- python3 tools/chunk_prof.py > $O/b$F.log 2>&1 || { tail -20 $O/b$F.log; exit 1; }
done
echo done
