set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/vit
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "viterbi or Viterbi or cfg4 or Max or shortest or forward_gradients" > gpurun_out/vit/test.log 2>&1; tail -3 gpurun_out/vit/test.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/vit/tr -o run -- python3 tools/configs_bench.py > gpurun_out/vit/cfg.log 2>&1 || { tail -20 gpurun_out/vit/cfg.log; exit 1; }
grep config gpurun_out/vit/cfg.log
python3 tools/prof_stats.py gpurun_out/vit/tr > gpurun_out/vit/stats.csv; grep -E "vit_|backtrace|fwd_kernel<1" gpurun_out/vit/stats.csv | cut -c1-140 || true
