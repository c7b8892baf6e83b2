set -o pipefail
mkdir -p gpurun_out/r5c
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_joint_fused.py > gpurun_out/r5c/joint.txt 2>&1
r1=$?
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_string_grad.py tests/test_gpu_table_grad.py tests/test_gpu_api.py > gpurun_out/r5c/t.txt 2>&1
r2=$?
echo "joint=$r1 string=$r2"
exit $((r1 | r2))
