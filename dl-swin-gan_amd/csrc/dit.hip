// Kernels of the DiT denoiser path (BASELINE config 5):
//   dit = dl_cs/models/DiT.py (reference), timm = timm.models.vision_transformer.
//
// * dlcs_mhsa_fwd / dlcs_mhsa_bwd -- the core of timm's Attention (qkv split into
//   [3, heads, hd], softmax(q k^T hd^-0.5) v) that DiTBlockFactor applies twice per
//   block (dit:336-345): over the H*W tokens of a frame (N = 1920 at the BASELINE
//   slice) and over the frames of a spatial position (N = 12).  Flash-style: K / V
//   streamed through LDS in 64-key chunks, scores and probabilities stay in
//   registers (one wave owns a 32-query (fwd, dQ) or 32-key (dK, dV) block on the
//   lanes of v_mfma_f32_32x32x2f32 tiles), online softmax in log2 units, the row
//   log-sum-exp saved for the backward, which recomputes P.  Head dims <= 32
//   (DiT: 384 / 16 = 24) contract in HD / 2 k-steps with no padding (lane half hh
//   supplies d = HD/2 * hh + j).
// * dlcs_conv3d_thin_im2col / _col2im -- the k3 convolutions with a 4-channel side
//   (DiTResNet's SFE 4 -> 384 and final 384 -> 4, dit:1297, :1302) as GEMMs: the
//   27-tap im2col of the thin side (108 columns) or the 27-tap gather-sum of a
//   thin GEMM output, on the patch-blocked channels-last layout.
// * small vector ops of the adaLN conditioning (dit:184-221, :324-331, :399-406):
//   SiLU and its gradient, 1 + scale, the sinusoidal timestep embedding, the
//   gate-folded Linear's parameter gradients, an embedding-row scatter-add.
#include "dlcs_common.h"

#include <algorithm>

namespace {

constexpr float kL2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

struct MhsaArgs {
    const float* qkv;    // [nseq * N, 3 * heads * hd]   (timm: reshape(B, N, 3, heads, hd))
    const float* o;      // [nseq * N, heads * hd]       (bwd)
    const float* dout;   // [nseq * N, heads * hd]       (bwd)
    float* out;          // [nseq * N, heads * hd]       (fwd)
    float* lse;          // [nseq, heads, N] natural log (fwd writes, bwd reads)
    float* dsum;         // [nseq, heads, N] rowsum(dO * O) (bwd workspace)
    float* dqkv;         // [nseq * N, 3 * heads * hd]   (bwd, every element written)
    int nseq, N, heads;
    float scale;
};

DLCS_DEV f32x16 mf(float a, float b, const f32x16& c) { return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0); }

constexpr int kKC = 64;      // keys (queries) per LDS chunk
constexpr int kCL = 40;      // row stride of the column-read images (4 * 40 = 32 mod 64: halves on disjoint banks)

// Chunk of rows [r0, r0 + kKC) of the head-h slice `part` (0 q, 1 k, 2 v) of qkv into
// a k-step image [kKC][HD + 2] (scaled by sc) and/or a column image [kKC][kCL]
// (columns >= HD zero); rows >= N are zero.
template <int HD>
DLCS_DEV void stage_rows(const float* src, long ld, int col0, int r0, int N, float* kimg, float sc, float* cimg) {
    constexpr int P4 = HD / 4, KLD = HD + 2;
    for (int i = threadIdx.x; i < kKC * P4; i += blockDim.x) {
        const int t = i / P4, c = i % P4;
        const bool ok = r0 + t < N;
        const float4 v = ok ? *reinterpret_cast<const float4*>(src + (long)(r0 + t) * ld + col0 + 4 * c)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
        if (kimg) {
            float2* kd = reinterpret_cast<float2*>(kimg + t * KLD + 4 * c);
            kd[0] = make_float2(v.x * sc, v.y * sc);
            kd[1] = make_float2(v.z * sc, v.w * sc);
        }
        if (cimg) *reinterpret_cast<float4*>(cimg + t * kCL + 4 * c) = v;
    }
}

template <int HD>
DLCS_DEV void zero_cols(float* cimg) {
    constexpr int Z = kCL - HD;
    for (int i = threadIdx.x; i < kKC * Z; i += blockDim.x) cimg[(i / Z) * kCL + HD + i % Z] = 0.0f;
}

// B operand of a k-step contraction (d = HD/2 * hh + j) from a global row
template <int HD>
DLCS_DEV void row_frag(float (&f)[HD / 2], const float* src, bool ok, int hh, float sc) {
    constexpr int H2 = HD / 2;
#pragma unroll
    for (int j = 0; j < H2; j += 2) {
        const float2 v = ok ? *reinterpret_cast<const float2*>(src + H2 * hh + j) : make_float2(0.f, 0.f);
        f[j] = v.x * sc;
        f[j + 1] = v.y * sc;
    }
}

// 32x32 tile: sum_j A(l31 row of img)[hh-half, j] B[j]
template <int HD>
DLCS_DEV f32x16 kstep_tile(const float* img, int row, const float (&b)[HD / 2], int hh) {
    constexpr int H2 = HD / 2, KLD = HD + 2;
    f32x16 acc = (f32x16)0.0f;
    const float* r = img + row * KLD + H2 * hh;
#pragma unroll
    for (int j = 0; j < H2; j += 2) {
        const float2 a = *reinterpret_cast<const float2*>(r + j);
        acc = mf(a.x, b[j], acc);
        acc = mf(a.y, b[j + 1], acc);
    }
    return acc;
}

// ---------------------------------------------------------------- forward
template <int HD>
__global__ void __launch_bounds__(256) mhsa_fwd_f32_kernel(MhsaArgs a) {
    constexpr int KLD = HD + 2;
    __shared__ __attribute__((aligned(16))) float Ks[kKC * KLD];
    __shared__ __attribute__((aligned(16))) float Vs[kKC * kCL];
    const int s = blockIdx.x / a.heads, h = blockIdx.x % a.heads;
    const int N = a.N, C = a.heads * HD;
    const long row0 = (long)s * N;
    const float* base = a.qkv + row0 * 3 * C;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hh = lane >> 5, l31 = lane & 31;
    const int qb = blockIdx.y * (blockDim.x >> 6) + wave;
    const int q = qb * 32 + l31;
    const bool qv = q < N;
    float qf[HD / 2];
    row_frag<HD>(qf, base + (long)min(q, N - 1) * 3 * C + h * HD, qv, hh, a.scale * kL2e);
    zero_cols<HD>(Vs);
    float m = -INFINITY, l = 0.0f;
    f32x16 z = (f32x16)0.0f;          // O^T: rows d, cols query
    for (int k0 = 0; k0 < N; k0 += kKC) {
        __syncthreads();
        stage_rows<HD>(base, 3 * C, C + h * HD, k0, N, Ks, 1.0f, nullptr);
        stage_rows<HD>(base, 3 * C, 2 * C + h * HD, k0, N, nullptr, 0.0f, Vs);
        __syncthreads();
        if (qb * 32 >= N) continue;
        for (int kb = 0; kb < kKC / 32 && k0 + kb * 32 < N; ++kb) {
            f32x16 sc = kstep_tile<HD>(Ks, kb * 32 + l31, qf, hh);     // S^T: rows key, cols query
            float tm = -INFINITY;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float v = (k0 + kb * 32 + acc_row(r, lane) < N) ? sc[r] : -INFINITY;
                sc[r] = v;
                tm = fmaxf(tm, v);
            }
            tm = xor32_max(tm);
            if (tm > m) {
                const float alpha = (m == -INFINITY) ? 0.0f : __builtin_amdgcn_exp2f(m - tm);
                z *= alpha;
                l *= alpha;
                m = tm;
            }
            float ps = 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float p = __builtin_amdgcn_exp2f(sc[r] - m);
                ps += p;
                z = mf(Vs[(kb * 32 + acc_row(r, lane)) * kCL + l31], p, z);
            }
            l += ps;
        }
    }
    if (qb * 32 >= N) return;
    const float lt = xor32_sum(l);
    if (!qv) return;
    const float inv = 1.0f / lt;
    float* dst = a.out + (row0 + q) * C + h * HD;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int d0 = 8 * g + 4 * hh;
        if (d0 < HD)
            *reinterpret_cast<float4*>(dst + d0) =
                make_float4(z[4 * g] * inv, z[4 * g + 1] * inv, z[4 * g + 2] * inv, z[4 * g + 3] * inv);
    }
    if (hh == 0) a.lse[((long)s * a.heads + h) * N + q] = m * kLn2 + __logf(lt);
}

// ---------------------------------------------------------------- backward
// D[s, h, q] = sum_d dO[q, h, d] O[q, h, d]
__global__ void mhsa_dsum_kernel(MhsaArgs a, int hd) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long total = (long)a.nseq * a.N * a.heads;
    if (i >= total) return;
    const int h = (int)(i % a.heads);
    const long row = i / a.heads;
    const int C = a.heads * hd;
    const float* o = a.o + row * C + h * hd;
    const float* d = a.dout + row * C + h * hd;
    float acc = 0.0f;
    for (int k = 0; k < hd; k += 4) {
        const float4 x = *reinterpret_cast<const float4*>(o + k), y = *reinterpret_cast<const float4*>(d + k);
        acc += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
    }
    const long s = row / a.N, q = row % a.N;
    a.dsum[(s * a.heads + h) * a.N + q] = acc;
}

// key-owned: dK, dV of a 32-key block per wave (keys on the lanes)
template <int HD>
__global__ void __launch_bounds__(256) mhsa_bwd_kv_f32_kernel(MhsaArgs a) {
    constexpr int KLD = HD + 2;
    __shared__ __attribute__((aligned(16))) float Qa[kKC * KLD];     // q * scale * log2e (k-step image)
    __shared__ __attribute__((aligned(16))) float dOa[kKC * KLD];    // dO (k-step image)
    __shared__ __attribute__((aligned(16))) float Qb[kKC * kCL];     // q (column image)
    __shared__ __attribute__((aligned(16))) float dOb[kKC * kCL];    // dO (column image)
    __shared__ float lse_s[kKC], D_s[kKC];
    const int s = blockIdx.x / a.heads, h = blockIdx.x % a.heads;
    const int N = a.N, C = a.heads * HD;
    const long row0 = (long)s * N;
    const float* base = a.qkv + row0 * 3 * C;
    const float* dob = a.dout + row0 * C;
    const long sh = ((long)s * a.heads + h) * N;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hh = lane >> 5, l31 = lane & 31;
    const int kb = blockIdx.y * (blockDim.x >> 6) + wave;
    const int key = kb * 32 + l31;
    const bool kv = key < N;
    float kf[HD / 2], vf[HD / 2];
    row_frag<HD>(kf, base + (long)min(key, N - 1) * 3 * C + C + h * HD, kv, hh, 1.0f);
    row_frag<HD>(vf, base + (long)min(key, N - 1) * 3 * C + 2 * C + h * HD, kv, hh, 1.0f);
    zero_cols<HD>(Qb);
    zero_cols<HD>(dOb);
    f32x16 dvt = (f32x16)0.0f, dkt = (f32x16)0.0f;      // rows d, cols key
    for (int q0 = 0; q0 < N; q0 += kKC) {
        __syncthreads();
        stage_rows<HD>(base, 3 * C, h * HD, q0, N, Qa, a.scale * kL2e, Qb);
        stage_rows<HD>(dob, C, h * HD, q0, N, dOa, 1.0f, dOb);
        for (int i = threadIdx.x; i < kKC; i += blockDim.x) {
            const bool ok = q0 + i < N;
            lse_s[i] = ok ? a.lse[sh + q0 + i] * kL2e : INFINITY;
            D_s[i] = ok ? a.dsum[sh + q0 + i] : 0.0f;
        }
        __syncthreads();
        if (kb * 32 >= N) continue;
        for (int qb = 0; qb < kKC / 32 && q0 + qb * 32 < N; ++qb) {
            const f32x16 sc = kstep_tile<HD>(Qa, qb * 32 + l31, kf, hh);     // S: rows query, cols key
            const f32x16 dp = kstep_tile<HD>(dOa, qb * 32 + l31, vf, hh);    // dP
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int qr = qb * 32 + acc_row(r, lane);
                const float p = __builtin_amdgcn_exp2f(sc[r] - lse_s[qr]);
                const float ds = p * (dp[r] - D_s[qr]);
                dvt = mf(dOb[qr * kCL + l31], p, dvt);
                dkt = mf(Qb[qr * kCL + l31], ds, dkt);
            }
        }
    }
    if (!kv) return;
    float* dk = a.dqkv + (row0 + key) * 3 * C + C + h * HD;
    float* dv = dk + C;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int d0 = 8 * g + 4 * hh;
        if (d0 < HD) {
            *reinterpret_cast<float4*>(dk + d0) = make_float4(dkt[4 * g] * a.scale, dkt[4 * g + 1] * a.scale,
                                                              dkt[4 * g + 2] * a.scale, dkt[4 * g + 3] * a.scale);
            *reinterpret_cast<float4*>(dv + d0) = make_float4(dvt[4 * g], dvt[4 * g + 1], dvt[4 * g + 2], dvt[4 * g + 3]);
        }
    }
}

// query-owned: dQ of a 32-query block per wave (queries on the lanes)
template <int HD>
__global__ void __launch_bounds__(256) mhsa_bwd_q_f32_kernel(MhsaArgs a) {
    constexpr int KLD = HD + 2;
    __shared__ __attribute__((aligned(16))) float Ka[kKC * KLD];
    __shared__ __attribute__((aligned(16))) float Va[kKC * KLD];
    __shared__ __attribute__((aligned(16))) float Kb[kKC * kCL];
    const int s = blockIdx.x / a.heads, h = blockIdx.x % a.heads;
    const int N = a.N, C = a.heads * HD;
    const long row0 = (long)s * N;
    const float* base = a.qkv + row0 * 3 * C;
    const long sh = ((long)s * a.heads + h) * N;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hh = lane >> 5, l31 = lane & 31;
    const int qb = blockIdx.y * (blockDim.x >> 6) + wave;
    const int q = qb * 32 + l31;
    const bool qv = q < N;
    const int qc = min(q, N - 1);
    float qf[HD / 2], dof[HD / 2];
    row_frag<HD>(qf, base + (long)qc * 3 * C + h * HD, qv, hh, a.scale * kL2e);
    row_frag<HD>(dof, a.dout + (row0 + qc) * C + h * HD, qv, hh, 1.0f);
    const float lse2 = qv ? a.lse[sh + q] * kL2e : INFINITY;
    const float Dq = qv ? a.dsum[sh + q] : 0.0f;
    zero_cols<HD>(Kb);
    f32x16 dqt = (f32x16)0.0f;                  // rows d, cols query
    for (int k0 = 0; k0 < N; k0 += kKC) {
        __syncthreads();
        stage_rows<HD>(base, 3 * C, C + h * HD, k0, N, Ka, 1.0f, Kb);
        stage_rows<HD>(base, 3 * C, 2 * C + h * HD, k0, N, Va, 1.0f, nullptr);
        __syncthreads();
        if (qb * 32 >= N) continue;
        for (int kb = 0; kb < kKC / 32 && k0 + kb * 32 < N; ++kb) {
            const f32x16 sc = kstep_tile<HD>(Ka, kb * 32 + l31, qf, hh);     // S^T: rows key, cols query
            const f32x16 dp = kstep_tile<HD>(Va, kb * 32 + l31, dof, hh);    // dP^T
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int kr = kb * 32 + acc_row(r, lane);
                const float p = (k0 + kr < N) ? __builtin_amdgcn_exp2f(sc[r] - lse2) : 0.0f;
                dqt = mf(Kb[kr * kCL + l31], p * (dp[r] - Dq), dqt);
            }
        }
    }
    if (qb * 32 >= N || !qv) return;
    float* dq = a.dqkv + (row0 + q) * 3 * C + h * HD;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int d0 = 8 * g + 4 * hh;
        if (d0 < HD)
            *reinterpret_cast<float4*>(dq + d0) = make_float4(dqt[4 * g] * a.scale, dqt[4 * g + 1] * a.scale,
                                                              dqt[4 * g + 2] * a.scale, dqt[4 * g + 3] * a.scale);
    }
}

template <int HD>
int mhsa_launch(const MhsaArgs& a, bool bwd, hipStream_t st) {
    const int nb = (a.N + 31) / 32;
    const int W = std::min(4, nb);
    const dim3 grid((unsigned)((long)a.nseq * a.heads), (unsigned)((nb + W - 1) / W)), block(W * 64);
    if (!bwd) {
        hipLaunchKernelGGL(mhsa_fwd_f32_kernel<HD>, grid, block, 0, st, a);
    } else {
        const long tot = (long)a.nseq * a.N * a.heads;
        hipLaunchKernelGGL(mhsa_dsum_kernel, dim3(cdiv(tot, 256)), dim3(256), 0, st, a, HD);
        hipLaunchKernelGGL(mhsa_bwd_kv_f32_kernel<HD>, grid, block, 0, st, a);
        hipLaunchKernelGGL(mhsa_bwd_q_f32_kernel<HD>, grid, block, 0, st, a);
    }
    return dlcs_launch_status();
}

int mhsa_dispatch(const MhsaArgs& a, int hd, bool bwd, hipStream_t st) {
    switch (hd) {
        case 8: return mhsa_launch<8>(a, bwd, st);
        case 16: return mhsa_launch<16>(a, bwd, st);
        case 20: return mhsa_launch<20>(a, bwd, st);
        case 24: return mhsa_launch<24>(a, bwd, st);
        case 32: return mhsa_launch<32>(a, bwd, st);
        default: return DLCS_ERR_UNSUPPORTED_SIZE;
    }
}

// ---------------------------------------------------------------- thin k3 convolutions
struct BlkGrid {
    int B, D, H, W, nT, nY, nX;
};

DLCS_DEV void blk_decode(long r, const BlkGrid& g, int& b, int& t, int& y, int& x) {
    const int inner = (int)(r & 63);
    long blk = r >> 6;
    const int x4 = (int)(blk % g.nX); blk /= g.nX;
    const int y4 = (int)(blk % g.nY); blk /= g.nY;
    const int t4 = (int)(blk % g.nT);
    b = (int)(blk / g.nT);
    t = 4 * t4 + (inner >> 4);
    y = 4 * y4 + ((inner >> 2) & 3);
    x = 4 * x4 + (inner & 3);
}

DLCS_DEV long blk_row(const BlkGrid& g, int b, int t, int y, int x) {
    return ((((long)b * g.nT + (t >> 2)) * g.nY + (y >> 2)) * g.nX + (x >> 2)) * 64 + (t & 3) * 16 + (y & 3) * 4 +
           (x & 3);
}

// neighbour row of (b, t, y, x) at sign * (kd - 1, kh - 1, kw - 1), or -1 outside the grid
DLCS_DEV long blk_nbr(const BlkGrid& g, int b, int t, int y, int x, int tap, int sign) {
    const int tt = t + sign * (tap / 9 - 1), yy = y + sign * ((tap / 3) % 3 - 1), xx = x + sign * (tap % 3 - 1);
    if (tt < 0 || tt >= g.D || yy < 0 || yy >= g.H || xx < 0 || xx >= g.W) return -1;
    return blk_row(g, b, tt, yy, xx);
}

// dst[v][tap * C + c] = src[nbr(v, tap)][c] (0 outside), columns [27 C, ldd) zero
__global__ void thin_im2col_kernel(const float* src, long lds, int C, float* dst, long ldd, int sign, BlkGrid g) {
    const long nrows = (long)g.B * g.D * g.H * g.W;
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrows * 28) return;
    const long v = i / 28;
    const int tap = (int)(i % 28);
    float* o = dst + v * ldd;
    if (tap == 27) {
        for (int c = 27 * C; c < ldd; ++c) o[c] = 0.0f;
        return;
    }
    int b, t, y, x;
    blk_decode(v, g, b, t, y, x);
    const long n = blk_nbr(g, b, t, y, x, tap, sign);
    for (int c = 0; c < C; ++c) o[tap * C + c] = n >= 0 ? src[n * lds + c] : 0.0f;
}

// out[v][c] (+)= bias[c] + sum_tap P[nbr(v, tap)][tap * C + c]   (c < C; columns [C, ldo) zero unless accumulate)
__global__ void thin_col2im_kernel(const float* P, long ldp, int C, float* out, long ldo, const float* bias, int sign,
                                   int accumulate, BlkGrid g) {
    const long nrows = (long)g.B * g.D * g.H * g.W;
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrows * ldo) return;
    const long v = i / ldo;
    const int c = (int)(i % ldo);
    if (c >= C) {
        if (!accumulate) out[i] = 0.0f;
        return;
    }
    int b, t, y, x;
    blk_decode(v, g, b, t, y, x);
    float acc = bias ? bias[c] : 0.0f;
    for (int tap = 0; tap < 27; ++tap) {
        const long n = blk_nbr(g, b, t, y, x, tap, sign);
        if (n >= 0) acc += P[n * ldp + tap * C + c];
    }
    out[i] = accumulate ? out[i] + acc : acc;
}

// ---------------------------------------------------------------- vectors
DLCS_DEV float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }

__global__ void dit_vec_kernel(int op, const float* a, const float* b, float* y, long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = a[i];
    float r;
    switch (op) {
        case 0: r = x * sigm(x); break;                                             // SiLU
        case 1: { const float sb = sigm(b[i]); r = x * sb * (1.0f + b[i] * (1.0f - sb)); break; }   // x * SiLU'(b)
        case 2: r = 1.0f + x; break;                                                // modulate gamma
        default: r = x + b[i]; break;                                               // sum
    }
    y[i] = r;
}

__global__ void timestep_embedding_kernel(const float* t, int B, int dim, float log_max_period, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * dim) return;
    const int b = i / dim, k = i % dim, half = dim / 2;
    if (k >= 2 * half) { out[i] = 0.0f; return; }
    const int kk = k < half ? k : k - half;
    const float f = expf(-log_max_period * (float)kk / (float)half);
    const float arg = t[b] * f;
    out[i] = k < half ? cosf(arg) : sinf(arg);
}

// per row n of a gate-folded Linear y = g * (x W^T + b):
//   dW[n,:] += g[n] G[n,:], db[n] += g[n] cs[n], dg[n] += W[n,:] . G[n,:] + b[n] cs[n]
__global__ void gated_linear_grad_kernel(const float* W, const float* bvec, const float* G, const float* cs,
                                         const float* gate, float* dW, float* db, float* dg, int K) {
    const int n = blockIdx.x;
    const float gn = gate[n];
    float acc = 0.0f;
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
        const float gv = G[(long)n * K + k];
        acc += W[(long)n * K + k] * gv;
        dW[(long)n * K + k] += gn * gv;
    }
    __shared__ float red[4];
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.0f;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
        const float c = cs[n];
        dg[n] += t + (bvec ? bvec[n] * c : 0.0f);
        if (db) db[n] += gn * c;
    }
}

__global__ void scale_rows_kernel(const float* W, const float* bvec, const float* gate, float* Wo, float* bo, int N,
                                  int K) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < (long)N * K) Wo[i] = gate[i / K] * W[i];
    if (i < N && bvec) bo[i] = gate[i] * bvec[i];
}

__global__ void rows_add_kernel(float* dst, const int32_t* idx, const float* src, long nrows, int C) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrows * C) return;
    const long r = i / C;
    const int c = (int)(i % C);
    const long d = idx ? (long)idx[r] : r;
    if (d >= 0) atomicAdd(dst + d * C + c, src[i]);
}

}  // namespace

int dlcs_mhsa_fwd_h3_internal(const float* qkv, float* out, float* lse, int nseq, int N, int heads, int hd,
                              float scale, hipStream_t st);
int dlcs_mhsa_bwd_h3_internal(const float* qkv, const float* dout, const float* lse, const float* dsum, float* dqkv,
                              int nseq, int N, int heads, int hd, float scale, hipStream_t st);

namespace {
bool mhsa_hd_h3(int64_t hd) { return hd == 8 || hd == 16 || hd == 20 || hd == 24 || hd == 32; }
}  // namespace

extern "C" {

int dlcs_mhsa_fwd(int dtype, const void* qkv, void* out, float* lse, int64_t nseq, int64_t N, int64_t heads,
                  int64_t head_dim, float scale, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(qkv && out && lse && nseq > 0 && N > 0 && heads > 0);
    if (dtype != DLCS_F32 || head_dim > 32 || head_dim % 4 || ((uintptr_t)qkv & 15) || ((uintptr_t)out & 15) ||
        nseq * heads > 0x7fffffffL)
        return DLCS_ERR_UNSUPPORTED_SIZE;
    MhsaArgs a{};
    a.qkv = (const float*)qkv; a.out = (float*)out; a.lse = lse;
    a.nseq = (int)nseq; a.N = (int)N; a.heads = (int)heads; a.scale = scale;
    // fp32 on fp16 matrix cores (three plane products, mhsa_h3.inc) by default;
    // DLCS_MHSA_H3=0 keeps the f32-MFMA kernel
    static const bool h3 = [] { const char* e = dlcs_knob("DLCS_MHSA_H3"); return !(e && e[0] == '0'); }();
    if (h3 && mhsa_hd_h3(head_dim))
        return dlcs_mhsa_fwd_h3_internal(a.qkv, a.out, a.lse, a.nseq, a.N, a.heads, (int)head_dim, scale,
                                         (hipStream_t)stream);
    return mhsa_dispatch(a, (int)head_dim, false, (hipStream_t)stream);
}

size_t dlcs_mhsa_bwd_workspace_bytes(int64_t nseq, int64_t N, int64_t heads) {
    return (size_t)nseq * N * heads * sizeof(float);
}

int dlcs_mhsa_bwd(int dtype, const void* qkv, const void* out, const void* dout, const float* lse, float* dqkv,
                  int64_t nseq, int64_t N, int64_t heads, int64_t head_dim, float scale, void* workspace,
                  size_t workspace_bytes, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(qkv && out && dout && lse && dqkv && nseq > 0 && N > 0 && heads > 0);
    if (dtype != DLCS_F32 || head_dim > 32 || head_dim % 4 || ((uintptr_t)qkv & 15) || ((uintptr_t)out & 15) ||
        ((uintptr_t)dout & 15) || ((uintptr_t)dqkv & 15))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    if (!workspace || workspace_bytes < dlcs_mhsa_bwd_workspace_bytes(nseq, N, heads)) return DLCS_ERR_WORKSPACE;
    MhsaArgs a{};
    a.qkv = (const float*)qkv; a.o = (const float*)out; a.dout = (const float*)dout; a.lse = (float*)lse;
    a.dsum = (float*)workspace; a.dqkv = dqkv;
    a.nseq = (int)nseq; a.N = (int)N; a.heads = (int)heads; a.scale = scale;
    // fp32 on fp16 matrix cores (mhsa_h3.inc) by default; DLCS_MHSA_H3_BWD=0 (or
    // DLCS_MHSA_H3=0) keeps the f32-MFMA kernels
    static const bool h3 = [] {
        const char* e = dlcs_knob("DLCS_MHSA_H3");
        const char* b = dlcs_knob("DLCS_MHSA_H3_BWD");
        return !(e && e[0] == '0') && !(b && b[0] == '0');
    }();
    if (h3 && mhsa_hd_h3(head_dim) && nseq * heads <= 0x7fffffffL) {
        const long tot = (long)a.nseq * a.N * a.heads;
        hipLaunchKernelGGL(mhsa_dsum_kernel, dim3(cdiv(tot, 256)), dim3(256), 0, (hipStream_t)stream, a, (int)head_dim);
        return dlcs_mhsa_bwd_h3_internal(a.qkv, a.dout, a.lse, a.dsum, a.dqkv, a.nseq, a.N, a.heads, (int)head_dim,
                                         scale, (hipStream_t)stream);
    }
    return mhsa_dispatch(a, (int)head_dim, true, (hipStream_t)stream);
}

int dlcs_conv3d_thin_im2col(const float* src, int64_t ld_src, int64_t C, float* dst, int64_t ld_dst, int sign,
                            int64_t B, int64_t D, int64_t H, int64_t W, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(src && dst && C > 0 && C <= 8 && ld_src >= C && ld_dst >= 27 * C && (sign == 1 || sign == -1));
    if (D % 4 || H % 4 || W % 4) return DLCS_ERR_UNSUPPORTED_SIZE;
    BlkGrid g{(int)B, (int)D, (int)H, (int)W, (int)(D / 4), (int)(H / 4), (int)(W / 4)};
    const long n = B * D * H * W * 28;
    hipLaunchKernelGGL(thin_im2col_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, src, (long)ld_src,
                       (int)C, dst, (long)ld_dst, sign, g);
    return dlcs_launch_status();
}

int dlcs_conv3d_thin_col2im(const float* P, int64_t ld_p, int64_t C, float* out, int64_t ld_out, const float* bias,
                            int sign, int accumulate, int64_t B, int64_t D, int64_t H, int64_t W,
                            dlcs_stream_t stream) {
    DLCS_CHECK_ARG(P && out && C > 0 && C <= 8 && ld_p >= 27 * C && ld_out >= C && (sign == 1 || sign == -1));
    if (D % 4 || H % 4 || W % 4) return DLCS_ERR_UNSUPPORTED_SIZE;
    BlkGrid g{(int)B, (int)D, (int)H, (int)W, (int)(D / 4), (int)(H / 4), (int)(W / 4)};
    const long n = B * D * H * W * ld_out;
    hipLaunchKernelGGL(thin_col2im_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, P, (long)ld_p,
                       (int)C, out, (long)ld_out, bias, sign, accumulate, g);
    return dlcs_launch_status();
}

int dlcs_dit_vec(int op, const float* a, const float* b, float* y, int64_t n, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(a && y && n > 0 && op >= 0 && op <= 3 && (op == 0 || op == 2 || b));
    hipLaunchKernelGGL(dit_vec_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, op, a, b, y, (long)n);
    return dlcs_launch_status();
}

int dlcs_timestep_embedding(const float* t, int64_t B, int64_t dim, float max_period, float* out,
                            dlcs_stream_t stream) {
    DLCS_CHECK_ARG(t && out && B > 0 && dim > 0 && max_period > 0.0f);
    hipLaunchKernelGGL(timestep_embedding_kernel, dim3(cdiv(B * dim, 256)), dim3(256), 0, (hipStream_t)stream, t,
                       (int)B, (int)dim, logf(max_period), out);
    return dlcs_launch_status();
}

int dlcs_gated_linear_grad(const float* W, const float* b, const float* G, const float* colsum, const float* gate,
                           float* dW, float* db, float* dgate, int64_t N, int64_t K, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(W && G && colsum && gate && dW && dgate && N > 0 && K > 0);
    hipLaunchKernelGGL(gated_linear_grad_kernel, dim3((unsigned)N), dim3(256), 0, (hipStream_t)stream, W, b, G,
                       colsum, gate, dW, db, dgate, (int)K);
    return dlcs_launch_status();
}

int dlcs_scale_rows(const float* W, const float* b, const float* gate, float* Wo, float* bo, int64_t N, int64_t K,
                    dlcs_stream_t stream) {
    DLCS_CHECK_ARG(W && gate && Wo && N > 0 && K > 0 && (!b || bo));
    hipLaunchKernelGGL(scale_rows_kernel, dim3(cdiv(std::max(N * K, N), 256)), dim3(256), 0, (hipStream_t)stream, W,
                       b, gate, Wo, bo, (int)N, (int)K);
    return dlcs_launch_status();
}

int dlcs_rows_add(float* dst, const int32_t* idx, const float* src, int64_t nrows, int64_t C, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(dst && src && nrows > 0 && C > 0);
    hipLaunchKernelGGL(rows_add_kernel, dim3(cdiv(nrows * C, 256)), dim3(256), 0, (hipStream_t)stream, dst, idx, src,
                       (long)nrows, (int)C);
    return dlcs_launch_status();
}

}  // extern "C"
