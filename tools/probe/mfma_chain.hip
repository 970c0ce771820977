// Bias of the f16x3 conv's per-step product chain on the matrix core: one step
// (two taps) = x_h w_l + x_l w_h + x_h w_h per tap, six v_mfma_f32_16x16x32_f16
// into a fresh tile (conv3d_f16x3.inc, FOLD), compared with the exact sum of the
// same plane products.  Variants:
//   0  the kernel's order (hl, lh, hh, hl, lh, hh)
//   1  low-plane products first (hl, lh, hl, lh, hh, hh)
//   2  the kernel's order on negated A planes, the tile negated back
//   3  low-plane products and high-plane products in separate tiles, summed in fp32
//   hipcc --offload-arch=gfx950 -O2 tools/probe/mfma_chain.hip -o tools/probe/mfma_chain
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef _Float16 f16;
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ inline void mm(f32x4_t& c, f16x8_t a, f16x8_t b) { c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

// per trial: planes [tap 2][hi/lo 2][512] for A (16 x 32 row-major) and B (32 x 16 row-major)
__global__ void chain_kernel(const f16* A, const f16* B, float* D, int trials, int variant) {
    const int t = blockIdx.x;
    if (t >= trials) return;
    const int lane = threadIdx.x;
    f16x8_t a[2][2], b[2][2];
    for (int tap = 0; tap < 2; ++tap)
        for (int pl = 0; pl < 2; ++pl) {
            const f16* pa = A + ((size_t)t * 4 + tap * 2 + pl) * 512;
            const f16* pb = B + ((size_t)t * 4 + tap * 2 + pl) * 512;
            for (int e = 0; e < 8; ++e) {
                a[tap][pl][e] = pa[(lane % 16) * 32 + 8 * (lane / 16) + e];
                b[tap][pl][e] = pb[(8 * (lane / 16) + e) * 16 + (lane % 16)];
            }
            if (variant == 2) a[tap][pl] = -a[tap][pl];
        }
    f32x4_t c = (f32x4_t)0.0f, c2 = (f32x4_t)0.0f;
    if (variant == 0 || variant == 2) {
        for (int tap = 0; tap < 2; ++tap) { mm(c, a[tap][0], b[tap][1]); mm(c, a[tap][1], b[tap][0]); mm(c, a[tap][0], b[tap][0]); }
        if (variant == 2) c = -c;
    } else if (variant == 1) {
        for (int tap = 0; tap < 2; ++tap) { mm(c, a[tap][0], b[tap][1]); mm(c, a[tap][1], b[tap][0]); }
        for (int tap = 0; tap < 2; ++tap) mm(c, a[tap][0], b[tap][0]);
    } else {
        for (int tap = 0; tap < 2; ++tap) { mm(c2, a[tap][0], b[tap][1]); mm(c2, a[tap][1], b[tap][0]); }
        for (int tap = 0; tap < 2; ++tap) mm(c, a[tap][0], b[tap][0]);
        c += c2;
    }
    for (int i = 0; i < 4; ++i) D[(size_t)t * 256 + (4 * (lane / 16) + i) * 16 + lane % 16] = c[i];
}

int main(int argc, char** argv) {
    const int trials = 8192;
    const float xs = argc > 1 ? atof(argv[1]) : 1000.f, ws = argc > 2 ? atof(argv[2]) : 100.f;
    const float mean = argc > 3 ? atof(argv[3]) : 0.f;      // mean of the activations (ReLU'd data: > 0)
    std::mt19937 rng(11);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<f16> A((size_t)trials * 2048), B((size_t)trials * 2048);
    auto split = [](float v, f16& h, f16& l) { h = (f16)v; l = (f16)(v - (float)h); };
    for (size_t i = 0; i < A.size(); i += 1024)
        for (int k = 0; k < 512; ++k) {
            split(xs * (nd(rng) + mean), A[i + k], A[i + 512 + k]);
            split(ws * nd(rng), B[i + k], B[i + 512 + k]);
        }
    std::vector<double> ex((size_t)trials * 256, 0.0);
    for (int t = 0; t < trials; ++t)
        for (int tap = 0; tap < 2; ++tap) {
            const f16* ah = &A[((size_t)t * 4 + tap * 2) * 512]; const f16* al = ah + 512;
            const f16* bh = &B[((size_t)t * 4 + tap * 2) * 512]; const f16* bl = bh + 512;
            for (int i = 0; i < 16; ++i)
                for (int j = 0; j < 16; ++j) {
                    double s = 0;
                    for (int k = 0; k < 32; ++k) {
                        const double xh = (float)ah[i * 32 + k], xl = (float)al[i * 32 + k];
                        const double wh = (float)bh[k * 16 + j], wl = (float)bl[k * 16 + j];
                        s += xh * wl + xl * wh + xh * wh;
                    }
                    ex[(size_t)t * 256 + i * 16 + j] += s;
                }
        }
    double rms = 0;
    for (double v : ex) rms += v * v;
    rms = std::sqrt(rms / ex.size());
    f16 *dA, *dB; float* dD;
    hipMalloc(&dA, A.size() * 2); hipMalloc(&dB, B.size() * 2); hipMalloc(&dD, ex.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    std::vector<float> D(ex.size());
    for (int v = 0; v < 4; ++v) {
        hipLaunchKernelGGL(chain_kernel, dim3(trials), dim3(64), 0, 0, dA, dB, dD, trials, v);
        hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
        double sp = 0, sn = 0, sa = 0, sr = 0; long np = 0, nn = 0;
        for (size_t i = 0; i < ex.size(); ++i) {
            const double e = D[i] - ex[i];
            sa += std::fabs(e);
            sr += std::fabs((double)(float)ex[i] - ex[i]);
            if (ex[i] > 0) { sp += e; ++np; } else { sn += e; ++nn; }
        }
        const double u = rms * std::ldexp(1.0, -24);
        printf("x %g w %g mean %g variant %d: mean error / (rms 2^-24): exact>0 %+.4f  exact<0 %+.4f  all %+.4f   "
               "mean|e| %.4f (fp32 rounding %.4f)\n", xs, ws, mean, v, sp / np / u, sn / nn / u,
               (sp + sn) / (np + nn) / u, sa / ex.size() / u, sr / ex.size() / u);
    }
    return 0;
}
