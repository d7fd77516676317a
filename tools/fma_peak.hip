// fp64 FMA throughput probe (gfx950): independent v_fma_f64 chains per lane,
// (a) all-VGPR operands, (b) one SGPR operand (the deferred pass's form).
// hipcc --offload-arch=gfx950 -O3 -o build/fma_peak tools/fma_peak.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CH, bool SG>
__global__ __launch_bounds__(256) void fma_kernel(double* out, const double* __restrict__ c, int iters) {
    double t[CH];
    const double p = 1.0 + threadIdx.x * 1e-9;
#pragma unroll
    for (int k = 0; k < CH; ++k) t[k] = k * 1e-3;
    const double cv = c[threadIdx.x & 7];
    for (int it = 0; it < iters; ++it) {
        const double s0 = SG ? c[it & 15] : cv;   // uniform address: scalar load
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int k = 0; k < CH; ++k) t[k] = __builtin_fma(-s0, p, t[k]);
    }
    double acc = 0;
#pragma unroll
    for (int k = 0; k < CH; ++k) acc += t[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int CH, bool SG>
static void run(double* out, double* c, int blocks) {
    const int iters = 2048;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    fma_kernel<CH, SG><<<blocks, 256>>>(out, c, 16);
    hipEventRecord(a);
    fma_kernel<CH, SG><<<blocks, 256>>>(out, c, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double flop = 2.0 * 16 * CH * (double)iters * blocks * 256;
    printf("{\"chains\": %d, \"sgpr_operand\": %d, \"blocks\": %d, \"ms\": %.4f, \"tflops\": %.2f}\n", CH, SG ? 1 : 0,
           blocks, ms, flop / ms / 1e9);
}

int main() {
    double *out, *c;
    hipMalloc(&out, sizeof(double) * 256 * 8192);
    hipMalloc(&c, sizeof(double) * 16);
    double h[16];
    for (int k = 0; k < 16; ++k) h[k] = 1e-6 * (k + 1);
    hipMemcpy(c, h, sizeof h, hipMemcpyHostToDevice);
    for (int blocks : {2048, 8192}) {
        run<4, false>(out, c, blocks);
        run<8, false>(out, c, blocks);
        run<8, true>(out, c, blocks);
        run<16, true>(out, c, blocks);
    }
    return 0;
}
