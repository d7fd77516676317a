set -o pipefail
mkdir -p gpurun_out/s4k
timeout -k 10 300 python -u -m pytest tests/test_gpu_defer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s4k/tests.txt 2>&1 && \
for t in 1 2 0; do timeout -k 10 300 python bench.py --no-cpu-baseline --timing $t > gpurun_out/s4k/bench_t$t.json 2> gpurun_out/s4k/bench_t$t.err || exit 1; done
