// mfma_probe.hip — does v_mfma_f64_16x16x4f64 round like four sequential fmas (k = 0..3)?
// Random A (16x4), B (4x16), C (16x16) with exponents over +-30; compares every element of
// D = mfma(A, B, C) with fma(a3,b3, fma(a2,b2, fma(a1,b1, fma(a0,b0, c)))) (fwd), the reverse
// order and a single rounding of the exact sum.  MFMA_DENORM=1: denormal-range operands,
// signed zeros and the smallest denormal mixed in.  Layouts (gfx950, wave64): A[l%16][l/16],
// B[l/16][l%16], C/D[l/16 + 4i][l%16] for the 4 doubles of lane l.
//   build: hipcc --offload-arch=gfx950 -O2 -ffp-contract=off -o tools/bin/mfma_probe tools/mfma_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <cmath>
#include <random>
typedef double d4 __attribute__((ext_vector_type(4)));
// per trial: A 16x4, B 4x16, C 16x16 row-major; D out 16x16
__global__ void k(const double* A, const double* B, const double* C, double* D, int trials) {
    const int l = threadIdx.x;
    for (int t = blockIdx.x; t < trials; t += gridDim.x) {
        const double* a = A + t * 64; const double* b = B + t * 64; const double* c = C + t * 256;
        double av = a[(l % 16) * 4 + (l / 16)];      // A[l%16][l/16]
        double bv = b[(l / 16) * 16 + (l % 16)];     // B[l/16][l%16]
        d4 cv;
        for (int i = 0; i < 4; ++i) cv[i] = c[((l / 16) + 4 * i) * 16 + (l % 16)];
        d4 dv = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, cv, 0, 0, 0);
        for (int i = 0; i < 4; ++i) D[t * 256 + ((l / 16) + 4 * i) * 16 + (l % 16)] = dv[i];
    }
}
int main() {
    const int trials = 200000;
    std::vector<double> A(trials * 64), B(trials * 64), C(trials * 256), D(trials * 256);
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> u(-1, 1);
    std::uniform_int_distribution<int> e(-30, 30);
    const int mode = getenv("MFMA_DENORM") ? 1 : 0;
    std::uniform_int_distribution<int> ed(-1040, -1000), ep(-20, 20);
    for (auto& x : A) x = std::ldexp(u(g), mode ? ed(g) + 1000 : e(g));
    for (auto& x : B) x = std::ldexp(u(g), mode ? -1000 - 10 + ep(g) / 4 : e(g));
    for (auto& x : C) x = std::ldexp(u(g), mode ? ed(g) : e(g) + 10);
    if (mode) {   // specials: signed zeros, infinities, NaN, denormals
        for (size_t i = 0; i < C.size(); i += 97) C[i] = (i / 97) % 2 ? -0.0 : 0.0;
        for (size_t i = 0; i < A.size(); i += 89) A[i] = (i / 89) % 3 == 0 ? -0.0 : 4.9e-324;
        for (size_t i = 0; i < B.size(); i += 101) B[i] = (i / 101) % 2 ? 0.0 : -0.0;
    }
    double *dA, *dB, *dC, *dD;
    hipMalloc(&dA, A.size() * 8); hipMalloc(&dB, B.size() * 8); hipMalloc(&dC, C.size() * 8); hipMalloc(&dD, D.size() * 8);
    hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
    k<<<1024, 64>>>(dA, dB, dC, dD, trials);
    hipMemcpy(D.data(), dD, D.size() * 8, hipMemcpyDeviceToHost);
    long seq_fwd = 0, seq_rev = 0, exact1 = 0, n = 0, pair = 0;
    for (int t = 0; t < trials; ++t)
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 16; ++j) {
                const double* a = &A[t * 64 + i * 4];
                double d = D[t * 256 + i * 16 + j];
                double s = C[t * 256 + i * 16 + j];
                for (int k = 0; k < 4; ++k) s = std::fma(a[k], B[t * 64 + k * 16 + j], s);
                double r = C[t * 256 + i * 16 + j];
                for (int k = 3; k >= 0; --k) r = std::fma(a[k], B[t * 64 + k * 16 + j], r);
                long double x = C[t * 256 + i * 16 + j];
                for (int k = 0; k < 4; ++k) x += (long double)a[k] * (long double)B[t * 64 + k * 16 + j];
                // pairwise: (c + (a0b0 + a1b1)) ... rough
                double p01 = std::fma(a[0], B[t*64 + j], a[1] * B[t*64+16+j]);
                seq_fwd += (memcmp(&d, &s, 8) == 0) || (d != d && s != s);
                seq_rev += (memcmp(&d, &r, 8) == 0);
                double xe = (double)x;
                exact1 += (memcmp(&d, &xe, 8) == 0);
                ++n;
            }
    printf("elements %ld  match seq-fma fwd %ld  rev %ld  ~single-rounding %ld\n", n, seq_fwd, seq_rev, exact1);
    return 0;
}
