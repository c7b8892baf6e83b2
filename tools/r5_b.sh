set -o pipefail
mkdir -p gpurun_out/r5b
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_string_grad.py tests/test_gpu_table_grad.py tests/test_gpu_api.py > gpurun_out/r5b/t.txt 2>&1
