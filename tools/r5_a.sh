set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_graph.py > gpurun_out/r5a/graph.txt 2>&1 && \
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r5a/gpu.txt 2>&1 && \
timeout -k 10 300 python bench.py --warmup 5 --steps 20 --no-joint > gpurun_out/r5a/bench.json 2> gpurun_out/r5a/bench.err
