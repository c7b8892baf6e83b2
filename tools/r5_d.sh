set -o pipefail
mkdir -p gpurun_out/r5d
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_string_grad.py tests/test_gpu_table_grad.py tests/test_gpu_api.py > gpurun_out/r5d/t.txt 2>&1
r2=$?
timeout -k 10 300 python -u tools/joint_fused_bench.py > gpurun_out/r5d/jf.jsonl 2> gpurun_out/r5d/jf.err
r3=$?
echo "string=$r2 bench=$r3"
exit $((r2 | r3))
