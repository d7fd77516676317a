set -o pipefail
mkdir -p gpurun_out/s4j
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s4j/gpu_tests.txt 2>&1
