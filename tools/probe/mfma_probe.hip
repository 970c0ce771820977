// Rounding behaviour of v_mfma_f32_16x16x32_f16 (and the bf16 / f32 variants):
// one wave per trial computes D = A B + C for random operands; the host compares
// with the exact sum (double) and reports the mean signed error split by the sign
// of the exact result -- round-to-nearest gives ~0 for both, truncation toward
// zero gives opposite signs, truncation toward -inf gives negative for both.
//   hipcc --offload-arch=gfx950 -O2 tools/probe/mfma_probe.hip -o /tmp/mfma_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef _Float16 f16;
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

// A [16][32], B [32][16] row-major, C/D [16][16]
__global__ void probe_kernel(const f16* A, const f16* B, const float* C, float* D, int trials) {
    const int t = blockIdx.x;
    if (t >= trials) return;
    const int lane = threadIdx.x;
    const f16* a = A + (size_t)t * 512;
    const f16* b = B + (size_t)t * 512;
    f16x8_t av, bv;
    // 16x16x32: lane l holds row (l % 16) of A, k = 8 (l / 16) .. +7; column (l % 16) of B, same k
    for (int e = 0; e < 8; ++e) {
        av[e] = a[(lane % 16) * 32 + 8 * (lane / 16) + e];
        bv[e] = b[(8 * (lane / 16) + e) * 16 + (lane % 16)];
    }
    f32x4_t acc;
    // D rows 4 (l / 16) + i, column l % 16
    for (int i = 0; i < 4; ++i) acc[i] = C[(size_t)t * 256 + (4 * (lane / 16) + i) * 16 + lane % 16];
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) D[(size_t)t * 256 + (4 * (lane / 16) + i) * 16 + lane % 16] = acc[i];
}

int main(int argc, char** argv) {
    const int trials = 4096;
    const double cmag = argc > 1 ? atof(argv[1]) : 0.0;     // |C| relative to a product
    std::mt19937 rng(7);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<f16> A(trials * 512), B(trials * 512);
    std::vector<float> C(trials * 256), D(trials * 256);
    for (auto& v : A) v = (f16)nd(rng);
    for (auto& v : B) v = (f16)nd(rng);
    for (auto& v : C) v = (float)(cmag * nd(rng));
    f16 *dA, *dB; float *dC, *dD;
    hipMalloc(&dA, A.size() * 2); hipMalloc(&dB, B.size() * 2);
    hipMalloc(&dC, C.size() * 4); hipMalloc(&dD, D.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe_kernel, dim3(trials), dim3(64), 0, 0, dA, dB, dC, dD, trials);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    double sp = 0, sn = 0, ap = 0, an = 0, rn = 0; long np = 0, nn = 0, exact = 0;
    for (int t = 0; t < trials; ++t)
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 16; ++j) {
                double s = C[t * 256 + i * 16 + j];
                for (int k = 0; k < 32; ++k) s += (double)(float)A[t * 512 + i * 32 + k] * (double)(float)B[t * 512 + k * 16 + j];
                const double d = D[t * 256 + i * 16 + j];
                const double ulp = std::ldexp(1.0, std::ilogb((float)s) - 23);   // fp32 ulp of the exact sum
                const double e = (d - s) / ulp;
                const double r = (double)(float)s;                                 // correctly rounded fp32
                if (d == r) ++exact;
                rn += std::fabs(d - r) / ulp;
                if (s > 0) { sp += e; ap += std::fabs(e); ++np; } else if (s < 0) { sn += e; an += std::fabs(e); ++nn; }
            }
    printf("|C|/product %.3g: mean signed error in fp32 ulps: exact>0 %+.4f (|e| %.4f)  exact<0 %+.4f (|e| %.4f)  "
           "correctly rounded %.4f  mean |D - rn(s)| %.4f ulp\n",
           cmag, sp / np, ap / np, sn / nn, an / nn, (double)exact / (trials * 256.0), rn / (trials * 256.0));
    return 0;
}
