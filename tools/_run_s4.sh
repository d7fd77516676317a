set -o pipefail
mkdir -p gpurun_out/s4p
timeout -k 10 300 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s4p/tests.txt 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s4p/bench_default.json 2> gpurun_out/s4p/bench_default.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --timing 2 > gpurun_out/s4p/bench_t2.json 2> gpurun_out/s4p/bench_t2.err
