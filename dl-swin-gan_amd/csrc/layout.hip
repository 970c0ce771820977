// Layout / bookkeeping / normalisation kernels (gfx950).
//
// * dlcs_window_index   -- the integer window bookkeeping of vst:41-67, :229,
//   :243, :342-355 as three int32 tables built on the device: partition source
//   rows (cyclic shift + window_partition + zero pad), reverse destination
//   rows (window_reverse + roll back + crop) and the shift-mask region label
//   of every windowed row.  Bit-exact with the reference (tests/golden/windex).
// * dlcs_gather_rows    -- dst[r] = src[idx[r]] (0 where idx < 0): the data
//   movement of window_partition / window_reverse, with optional dtype cast.
// * dlcs_layernorm_fwd / _bwd -- nn.LayerNorm(C, eps) (vst:205, :211) with a
//   fused row gather (the windowed LN1 output) and fp32 statistics.
// * dlcs_colsum         -- bias gradients (column sums, fp32 atomics).
// * dlcs_swin_pre / _post (+ _bwd) -- s3d:394-418: complex <-> real channels,
//   circular time pad / crop, into / out of the patch-blocked channels-last
//   layout used by every conv / GEMM kernel:
//     act[b][t/4][y/4][x/4][(t%4)*16 + (y%4)*4 + x%4][c]
//   (a k4s4 patch is 64 contiguous rows, so PatchEmbed3D / PatchUnembed3D,
//   vst:455 / :503, are plain GEMMs on it).
#include "dlcs_common.h"

#include <algorithm>

namespace {

// ------------------------------------------------------------------ windows
// region label along one dim, exactly as the slices of vst:346-349 leave it
DLCS_DEV int region_label(int c, int n, int w, int s) {
    int lab = 0;                        // slice(-w): [0, n-w)
    if (s > 0) {
        if (c >= n - w && c < n - s) lab = 1;
        if (c >= n - s) lab = 2;
        if (c < n - w) lab = 0;
    } else {
        lab = 2;                        // slice(-0, None) covers the whole axis last
    }
    return lab;
}

__global__ void window_index_kernel(int B, int D, int H, int W, int wd, int wh, int ww,
                                    int sd, int sh, int sw, int32_t* part_src, int32_t* rev_dst,
                                    int32_t* labels) {
    const int Dp = (D + wd - 1) / wd * wd, Hp = (H + wh - 1) / wh * wh, Wp = (W + ww - 1) / ww * ww;
    const int nD = Dp / wd, nH = Hp / wh, nW = Wp / ww, N = wd * wh * ww;
    const long total = (long)B * nD * nH * nW * N;
    for (long r = blockIdx.x * (long)blockDim.x + threadIdx.x; r < total; r += (long)gridDim.x * blockDim.x) {
        const int n = (int)(r % N);
        long w = r / N;
        const int iW = (int)(w % nW); w /= nW;
        const int iH = (int)(w % nH); w /= nH;
        const int iD = (int)(w % nD);
        const int b = (int)(w / nD);
        const int td = n / (wh * ww), th = (n / ww) % wh, tw = n % ww;
        // coordinate in the rolled, padded array, and its source
        const int dr = iD * wd + td, hr = iH * wh + th, wr = iW * ww + tw;
        const int d = (dr + sd) % Dp, h = (hr + sh) % Hp, x = (wr + sw) % Wp;
        int32_t src = -1;
        if (d < D && h < H && x < W) src = (int32_t)((((long)b * D + d) * H + h) * W + x);
        if (part_src) part_src[r] = src;
        if (rev_dst && src >= 0) rev_dst[src] = (int32_t)r;
        if (labels) {
            // compute_mask labels the *rolled* padded lattice position (dr, hr, wr)
            const int ld = region_label(dr, Dp, wd, sd), lh = region_label(hr, Hp, wh, sh),
                      lw = region_label(wr, Wp, ww, sw);
            labels[r] = ld * 9 + lh * 3 + lw;
        }
    }
}

// ------------------------------------------------------------------ gathers
template <typename TI, typename TO>
__global__ void gather_rows_kernel(const TI* src, const int32_t* idx, TO* dst, long nrows, int C,
                                   long ld_src, long ld_dst) {
    const long total = nrows * C;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long r = i / C;
        const int c = (int)(i % C);
        const long s = idx ? (long)idx[r] : r;
        const float v = (s >= 0) ? to_f(src[s * ld_src + c]) : 0.0f;
        dst[r * ld_dst + c] = from_f<TO>(v);
    }
}

// ------------------------------------------------------------------ layernorm
// one wave per output row; C <= 64 * kLnMax
constexpr int kLnMax = 8;

template <typename TO>
__global__ void __launch_bounds__(256) layernorm_fwd_kernel(const float* x, const int32_t* src_map,
                                                            const float* gamma, const float* beta, float eps,
                                                            TO* out, float* mean_out, float* rstd_out,
                                                            long rows, int C) {
    const int lane = threadIdx.x & 63;
    const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const long s = src_map ? (long)src_map[r] : r;
    TO* o = out + r * C;
    if (s < 0) {                                   // zero pad row (vst:225 pads after norm1)
        for (int c = lane; c < C; c += 64) o[c] = from_f<TO>(0.0f);
        if (lane == 0) { mean_out[r] = 0.0f; rstd_out[r] = 0.0f; }
        return;
    }
    const float* xr = x + s * C;
    float v[kLnMax];
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < kLnMax; ++k) {
        const int c = lane + 64 * k;
        v[k] = (c < C) ? xr[c] : 0.0f;
        sum += v[k];
    }
    const float mean = wave_sum(sum) / (float)C;
    float sq = 0.0f;
#pragma unroll
    for (int k = 0; k < kLnMax; ++k) {
        const int c = lane + 64 * k;
        const float d = (c < C) ? v[k] - mean : 0.0f;
        sq += d * d;
    }
    const float var = wave_sum(sq) / (float)C;
    const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
    for (int k = 0; k < kLnMax; ++k) {
        const int c = lane + 64 * k;
        if (c < C) o[c] = from_f<TO>((v[k] - mean) * rstd * gamma[c] + beta[c]);
    }
    if (lane == 0) { mean_out[r] = mean; rstd_out[r] = rstd; }
}

// dx[src[r]] += rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma;
// dgamma += sum_r dy * xhat, dbeta += sum_r dy.  A wave owns kLnRows rows and
// issues all of their loads before the first reduction (one latency round per
// wave instead of one per row).  The column partials of a workgroup go to
// part[block][2][C] with plain stores (layernorm_bwd_reduce_kernel sums them):
// ~840 workgroups adding into the same 2 C floats through atomics serialised
// on a handful of L2 channels (44 us per call for 13,440 x 160).  Without a
// workspace the partials fall back to those atomics.
constexpr int kLnRows = 4;                      // rows per wave
constexpr int kLnBwdMax = 4;                    // C <= 256 on the batched path

template <int KM>
__global__ void __launch_bounds__(256) layernorm_bwd_kernel(const float* dy, const float* x,
                                                            const int32_t* src_map, const float* gamma,
                                                            const float* mean_in, const float* rstd_in,
                                                            const float* dx_in, float* dx, float* dgamma,
                                                            float* dbeta, float* part, long rows, int C) {
    __shared__ float sg[4][64 * KM];
    __shared__ float sb[4][64 * KM];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long rbase = (long)blockIdx.x * (4 * kLnRows) + wv * kLnRows;
    float gam[KM], pg[KM], pb[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
        const int c = lane + 64 * k;
        gam[k] = c < C ? gamma[c] : 0.0f;
        pg[k] = 0.0f;
        pb[k] = 0.0f;
    }
    long src[kLnRows];
    float mu[kLnRows], rs[kLnRows], d[kLnRows][KM], xv[kLnRows][KM];
#pragma unroll
    for (int j = 0; j < kLnRows; ++j) {
        const long r = rbase + j;
        src[j] = r < rows ? (src_map ? (long)src_map[r] : r) : -1;
    }
#pragma unroll
    for (int j = 0; j < kLnRows; ++j) {
        const long r = rbase + j;
        const bool ok = src[j] >= 0;
        mu[j] = ok ? mean_in[r] : 0.0f;
        rs[j] = ok ? rstd_in[r] : 0.0f;
#pragma unroll
        for (int k = 0; k < KM; ++k) {
            const int c = lane + 64 * k;
            const bool okc = ok && c < C;
            d[j][k] = okc ? dy[r * C + c] : 0.0f;
            xv[j][k] = okc ? x[src[j] * C + c] : 0.0f;
        }
    }
#pragma unroll
    for (int j = 0; j < kLnRows; ++j) {
        float xh[KM], g[KM];
        float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
        for (int k = 0; k < KM; ++k) {
            xh[k] = (xv[j][k] - mu[j]) * rs[j];
            g[k] = d[j][k] * gam[k];
            pg[k] += d[j][k] * xh[k];
            pb[k] += d[j][k];
            s1 += g[k];
            s2 += g[k] * xh[k];
        }
        const float m1 = wave_sum(s1) / (float)C, m2 = wave_sum(s2) / (float)C;
        if (src[j] < 0) continue;
        float* dxr = dx + src[j] * C;
        const float* dxi = dx_in ? dx_in + src[j] * C : dxr;
#pragma unroll
        for (int k = 0; k < KM; ++k) {
            const int c = lane + 64 * k;
            if (c < C) dxr[c] = dxi[c] + rs[j] * (g[k] - m1 - xh[k] * m2);
        }
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) { sg[wv][lane + 64 * k] = pg[k]; sb[wv][lane + 64 * k] = pb[k]; }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        const float a = sg[0][c] + sg[1][c] + sg[2][c] + sg[3][c];
        const float b = sb[0][c] + sb[1][c] + sb[2][c] + sb[3][c];
        if (part) {
            part[(long)blockIdx.x * 2 * C + c] = a;
            part[(long)blockIdx.x * 2 * C + C + c] = b;
        } else {
            if (dgamma) atomicAdd(dgamma + c, a);
            if (dbeta) atomicAdd(dbeta + c, b);
        }
    }
}

// dgamma[c] += sum_b part[b][0][c], dbeta[c] += sum_b part[b][1][c]: workgroup
// (64-column chunk of the 2 C columns, one of kLnRed partial-block ranges); 4
// waves x 4 independent sums per lane, one atomic per column and range
constexpr int kLnRed = 16;
__global__ void __launch_bounds__(256) layernorm_bwd_reduce_kernel(const float* part, int nblk, int C,
                                                                   float* dgamma, float* dbeta) {
    __shared__ float red[4][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int col = blockIdx.x * 64 + lane;          // 0 .. 2C
    const int b0 = (int)((long)nblk * blockIdx.y / kLnRed), b1 = (int)((long)nblk * (blockIdx.y + 1) / kLnRed);
    float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (col < 2 * C) {
        int b = b0 + wv;
        for (; b + 12 < b1; b += 16) {
#pragma unroll
            for (int u = 0; u < 4; ++u) s[u] += part[(long)(b + 4 * u) * 2 * C + col];
        }
        for (; b < b1; b += 4) s[0] += part[(long)b * 2 * C + col];
    }
    red[wv][lane] = (s[0] + s[1]) + (s[2] + s[3]);
    __syncthreads();
    if (wv == 0 && col < 2 * C) {
        const float t = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
        float* o = col < C ? dgamma : dbeta;
        if (o) atomicAdd(o + (col < C ? col : col - C), t);
    }
}

// generic fallback (C > 256): one row per wave iteration, fp32 atomics
__global__ void __launch_bounds__(256) layernorm_bwd_generic_kernel(const float* dy, const float* x,
                                                            const int32_t* src_map, const float* gamma,
                                                            const float* mean_in, const float* rstd_in,
                                                            const float* dx_in, float* dx, float* dgamma,
                                                            float* dbeta, long rows, int C, int rows_per_block) {
    __shared__ float sg[4][64 * kLnMax];
    __shared__ float sb[4][64 * kLnMax];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float pg[kLnMax], pb[kLnMax];
#pragma unroll
    for (int k = 0; k < kLnMax; ++k) { pg[k] = 0.0f; pb[k] = 0.0f; }
    const long r0 = (long)blockIdx.x * rows_per_block;
    for (long r = r0 + wv; r < min(rows, r0 + rows_per_block); r += 4) {
        const long s = src_map ? (long)src_map[r] : r;
        if (s < 0) continue;
        const float mean = mean_in[r], rstd = rstd_in[r];
        const float* dyr = dy + r * C;
        const float* xr = x + s * C;
        float xh[kLnMax], g[kLnMax];
        float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
        for (int k = 0; k < kLnMax; ++k) {
            const int c = lane + 64 * k;
            if (c < C) {
                const float d = dyr[c];
                xh[k] = (xr[c] - mean) * rstd;
                g[k] = d * gamma[c];
                pg[k] += d * xh[k];
                pb[k] += d;
            } else { xh[k] = 0.0f; g[k] = 0.0f; }
            s1 += g[k];
            s2 += g[k] * xh[k];
        }
        const float m1 = wave_sum(s1) / (float)C, m2 = wave_sum(s2) / (float)C;
        float* dxr = dx + s * C;
        const float* dxi = dx_in ? dx_in + s * C : dxr;
#pragma unroll
        for (int k = 0; k < kLnMax; ++k) {
            const int c = lane + 64 * k;
            if (c < C) dxr[c] = dxi[c] + rstd * (g[k] - m1 - xh[k] * m2);
        }
    }
#pragma unroll
    for (int k = 0; k < kLnMax; ++k) { sg[wv][lane + 64 * k] = pg[k]; sb[wv][lane + 64 * k] = pb[k]; }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        const float a = sg[0][c] + sg[1][c] + sg[2][c] + sg[3][c];
        const float b = sb[0][c] + sb[1][c] + sb[2][c] + sb[3][c];
        if (dgamma) atomicAdd(dgamma + c, a);
        if (dbeta) atomicAdd(dbeta + c, b);
    }
}

// ------------------------------------------------------------------ colsum
// out[c] += sum_r x[r, c].  Thread = (row group, 8-column chunk): 16-B (bf16) /
// 2 x 16-B (fp32) loads, rows strided by the number of row groups, 4 rows in
// flight; partial sums reduced over row groups in LDS, one atomic per column
// and workgroup.  Needs ld % 8 == 0 and a 16-B aligned base (else the scalar
// kernel below).
template <typename T>
__global__ void __launch_bounds__(256) colsum_vec_kernel(const T* x, long rows, int C, long ld, float* out,
                                                         long rows_per_block) {
    __shared__ float part[256 * 8];
    const int nch = (C + 7) >> 3;
    const int ngrp = 256 / nch;
    const int ch = threadIdx.x % nch, grp = threadIdx.x / nch;
    const long r0 = (long)blockIdx.x * rows_per_block;
    const long r1 = min(rows, r0 + rows_per_block);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (grp < ngrp) {
        long r = r0 + grp;
        for (; r + 3 * ngrp < r1; r += 4 * ngrp) {
            Frag8<T> f[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) f[u] = load8<T>(x + (r + u * ngrp) * ld + ch * 8);
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[e] += to_f(f[u].v[e]);
        }
        for (; r < r1; r += ngrp) {
            const Frag8<T> f = load8<T>(x + r * ld + ch * 8);
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] += to_f(f.v[e]);
        }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) part[threadIdx.x * 8 + e] = acc[e];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
        float s = 0.0f;
        for (int g = 0; g < ngrp; ++g) s += part[(g * nch + (c >> 3)) * 8 + (c & 7)];
        atomicAdd(out + c, s);
    }
}

template <typename T>
__global__ void __launch_bounds__(256) colsum_kernel(const T* x, long rows, int C, long ld, float* out,
                                                     int rows_per_block) {
    const long r0 = (long)blockIdx.x * rows_per_block;
    const long r1 = min(rows, r0 + rows_per_block);
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float s = 0.0f;
        for (long r = r0; r < r1; ++r) s += to_f(x[r * ld + c]);
        atomicAdd(out + c, s);
    }
}

// ------------------------------------------------------------------ swin pre / post
// blocked offset of voxel (b, t, y, x) in a [B, Tp, Y, X] grid (all multiples of 4)
DLCS_DEV long blocked_row(int b, int t, int y, int x, int Tp, int Y, int X) {
    const int nT = Tp >> 2, nY = Y >> 2, nX = X >> 2;
    const long patch = (((long)b * nT + (t >> 2)) * nY + (y >> 2)) * nX + (x >> 2);
    return patch * 64 + ((t & 3) << 4) + ((y & 3) << 2) + (x & 3);
}

// u[b, t', y, x, c] = (c < E ? Re : Im) x[b, c mod E, (t' - pad) mod T, y, x], c < 2E, zero for c >= 2E
template <typename T>
__global__ void swin_pre_kernel(const float2* x, T* u, int B, int E, int Tn, int Y, int X, int pad, int ldc) {
    const int Tp = Tn + 2 * pad;
    const long total = (long)B * Tp * Y * X;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int xx = (int)(i % X);
        long q = i / X;
        const int y = (int)(q % Y); q /= Y;
        const int tp = (int)(q % Tp);
        const int b = (int)(q / Tp);
        const int t = ((tp - pad) % Tn + Tn) % Tn;
        T* dst = u + blocked_row(b, tp, y, xx, Tp, Y, X) * ldc;
        for (int c = 0; c < ldc; ++c) {
            float v = 0.0f;
            if (c < 2 * E) {
                const int e = c % E;
                const float2 z = x[((((long)b * E + e) * Tn + t) * Y + y) * X + xx];
                v = (c < E) ? z.x : z.y;
            }
            dst[c] = from_f<T>(v);
        }
    }
}

// gx[b, e, t] = sum over t' = t + pad + k*T in [0, Tp) of g_u  (circular-pad adjoint)
template <typename T>
__global__ void swin_pre_bwd_kernel(const T* gu, float2* gx, int B, int E, int Tn, int Y, int X, int pad, int ldc) {
    const int Tp = Tn + 2 * pad;
    const long total = (long)B * E * Tn * Y * X;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int xx = (int)(i % X);
        long q = i / X;
        const int y = (int)(q % Y); q /= Y;
        const int t = (int)(q % Tn); q /= Tn;
        const int e = (int)(q % E);
        const int b = (int)(q / E);
        float re = 0.0f, im = 0.0f;
        for (int tp = (t + pad) % Tn; tp < Tp; tp += Tn) {
            const T* src = gu + blocked_row(b, tp, y, xx, Tp, Y, X) * ldc;
            re += to_f(src[e]);
            im += to_f(src[E + e]);
        }
        gx[i] = make_float2(re, im);
    }
}

// out[b, e, t] = complex(o[c = e], o[c = E + e]) at t' = t + pad   (s3d:410-416)
template <typename T>
__global__ void swin_post_kernel(const T* o, float2* out, int B, int E, int Tn, int Y, int X, int pad, int ldc) {
    const int Tp = Tn + 2 * pad;
    const long total = (long)B * E * Tn * Y * X;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int xx = (int)(i % X);
        long q = i / X;
        const int y = (int)(q % Y); q /= Y;
        const int t = (int)(q % Tn); q /= Tn;
        const int e = (int)(q % E);
        const int b = (int)(q / E);
        const T* src = o + blocked_row(b, t + pad, y, xx, Tp, Y, X) * ldc;
        out[i] = make_float2(to_f(src[e]), to_f(src[E + e]));
    }
}

// g_o = scatter of g_out into the cropped range (zero elsewhere, channels >= 2E zero)
template <typename T>
__global__ void swin_post_bwd_kernel(const float2* gout, T* go, int B, int E, int Tn, int Y, int X, int pad, int ldc) {
    const int Tp = Tn + 2 * pad;
    const long total = (long)B * Tp * Y * X;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int xx = (int)(i % X);
        long q = i / X;
        const int y = (int)(q % Y); q /= Y;
        const int tp = (int)(q % Tp);
        const int b = (int)(q / Tp);
        T* dst = go + blocked_row(b, tp, y, xx, Tp, Y, X) * ldc;
        const int t = tp - pad;
        for (int c = 0; c < ldc; ++c) {
            float v = 0.0f;
            if (t >= 0 && t < Tn && c < 2 * E) {
                const int e = c % E;
                const float2 z = gout[((((long)b * E + e) * Tn + t) * Y + y) * X + xx];
                v = (c < E) ? z.x : z.y;
            }
            dst[c] = from_f<T>(v);
        }
    }
}

// ------------------------------------------------------------------ elementwise
// y = a * x + b * y  (fp32 or T), n elements; y may alias nothing else
// batched fp32 -> bf16 casts: blockIdx.y = tensor, grid-stride over its elements
struct CastMultiArgs {
    const float* src[DLCS_CAST_MULTI_MAX];
    bf16* dst[DLCS_CAST_MULTI_MAX];
    int64_t n[DLCS_CAST_MULTI_MAX];
};
__global__ void __launch_bounds__(256) cast_multi_kernel(CastMultiArgs a) {
    const int t = blockIdx.y;
    const float* s = a.src[t];
    bf16* d = a.dst[t];
    const long n = a.n[t];
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        d[i] = (bf16)s[i];
}

template <typename TX, typename TY>
__global__ void axpby_kernel(const TX* x, TY* y, long n, float a, float b) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float yv = (b != 0.0f) ? to_f(y[i]) : 0.0f;
        y[i] = from_f<TY>(a * to_f(x[i]) + b * yv);
    }
}

// g[i] *= (a[i] > 0): the ReLU derivative taken from the stored post-ReLU
// activation, in place on the gradient (PatchGAN discriminator backward, where a
// GEMM dgrad feeds a ReLU'd conv input and no conv epilogue can apply it).
// 8 elements per lane per iteration: 16-B bf16 / 2x16-B fp32 vector accesses.
template <typename TG, typename TA>
__global__ void relu_grad_kernel(TG* g, const TA* a, long n) {
    const long nv = n / 8;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < nv; v += stride) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const long i = v * 8 + k;
            if (!(to_f(a[i]) > 0.0f)) g[i] = from_f<TG>(0.0f);
        }
    }
    for (long i = nv * 8 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride)
        if (!(to_f(a[i]) > 0.0f)) g[i] = from_f<TG>(0.0f);
}

// dst = src permuted: dst index (i_0..i_{n-1}) over dst shape reads src at
// sum_k i_k * src_stride_k (strides of src given per dst dim); optional accumulate
// NCDHW <-> patch-blocked channels-last rows (the layout the conv / patch GEMM
// kernels use, see the file header), for the standalone module API: the grid is
// padded to multiples of 4 with zeros (blocking) / cropped (unblocking).
//   row(b, t, y, x) = ((b nT + t/4) nY + y/4) nX + x/4) * 64 + (t%4) 16 + (y%4) 4 + x%4
template <typename TI, typename TO>
__global__ void to_blocked_kernel(const TI* src, TO* dst, int B, int C, int D, int H, int W, int ld) {
    const int nT = (D + 3) >> 2, nY = (H + 3) >> 2, nX = (W + 3) >> 2;
    const long rows = (long)B * nT * nY * nX * 64;
    const long total = rows * ld;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long row = i / ld;
        const int c = (int)(i - row * ld);
        const int ip = (int)(row & 63);
        long p = row >> 6;
        const int px = (int)(p % nX); p /= nX;
        const int py = (int)(p % nY); p /= nY;
        const int pt = (int)(p % nT);
        const int b = (int)(p / nT);
        const int t = pt * 4 + (ip >> 4), y = py * 4 + ((ip >> 2) & 3), x = px * 4 + (ip & 3);
        float v = 0.0f;
        if (c < C && t < D && y < H && x < W) v = to_f(src[(((long)b * C + c) * D + t) * (long)H * W + (long)y * W + x]);
        dst[i] = from_f<TO>(v);
    }
}

template <typename TI, typename TO>
__global__ void from_blocked_kernel(const TI* src, TO* dst, int B, int C, int D, int H, int W, int ld) {
    const int nT = (D + 3) >> 2, nY = (H + 3) >> 2, nX = (W + 3) >> 2;
    const long total = (long)B * C * D * H * W;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        long r = i;
        const int x = (int)(r % W); r /= W;
        const int y = (int)(r % H); r /= H;
        const int t = (int)(r % D); r /= D;
        const int c = (int)(r % C);
        const int b = (int)(r / C);
        const long row = ((((long)b * nT + (t >> 2)) * nY + (y >> 2)) * nX + (x >> 2)) * 64 + ((t & 3) << 4) +
                         ((y & 3) << 2) + (x & 3);
        dst[i] = from_f<TO>(to_f(src[row * ld + c]));
    }
}

struct PermArgs { long v[12]; };

template <typename TI, typename TO>
__global__ void permute_kernel_v(const TI* src, TO* dst, int nd, PermArgs pa, long total, int accumulate) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        long rem = i, off = 0;
        for (int k = nd - 1; k >= 0; --k) {
            const long dk = pa.v[k];
            off += (rem % dk) * pa.v[6 + k];
            rem /= dk;
        }
        float v = to_f(src[off]);
        if (accumulate) v += to_f(dst[i]);
        dst[i] = from_f<TO>(v);
    }
}

// out[r, c] = bias[c % period]  (split-K GEMM outputs start from their bias)
__global__ void fill_bias_kernel(float* out, const float* bias, long rows, int C, int period) {
    const long total = rows * C;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x)
        out[i] = bias ? bias[(i % C) % period] : 0.0f;
}

static unsigned grid_for(long n) {
    long g = (n + 255) / 256;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    return (unsigned)g;
}

}  // namespace

extern "C" {

int dlcs_window_index(int64_t B, int64_t D, int64_t H, int64_t W, int64_t wd, int64_t wh, int64_t ww,
                      int64_t sd, int64_t sh, int64_t sw, int32_t* part_src, int32_t* rev_dst,
                      int32_t* labels, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(B > 0 && D > 0 && H > 0 && W > 0 && wd > 0 && wh > 0 && ww > 0);
    DLCS_CHECK_ARG(sd >= 0 && sd < wd && sh >= 0 && sh < wh && sw >= 0 && sw < ww);
    const long Dp = (D + wd - 1) / wd * wd, Hp = (H + wh - 1) / wh * wh, Wp = (W + ww - 1) / ww * ww;
    const long total = B * Dp * Hp * Wp;
    hipLaunchKernelGGL(window_index_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                       (int)B, (int)D, (int)H, (int)W, (int)wd, (int)wh, (int)ww, (int)sd, (int)sh, (int)sw,
                       part_src, rev_dst, labels);
    return dlcs_launch_status();
}

int dlcs_gather_rows(int src_dtype, int dst_dtype, const void* src, const int32_t* idx, void* dst,
                     int64_t nrows, int64_t C, int64_t ld_src, int64_t ld_dst, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(src && dst && nrows >= 0 && C > 0);
    if (nrows == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    dim3 g(grid_for(nrows * C)), b(256);
    if (src_dtype == DLCS_F32 && dst_dtype == DLCS_F32)
        hipLaunchKernelGGL((gather_rows_kernel<float, float>), g, b, 0, st, (const float*)src, idx, (float*)dst, nrows, (int)C, ld_src, ld_dst);
    else if (src_dtype == DLCS_F32 && dst_dtype == DLCS_BF16)
        hipLaunchKernelGGL((gather_rows_kernel<float, bf16>), g, b, 0, st, (const float*)src, idx, (bf16*)dst, nrows, (int)C, ld_src, ld_dst);
    else if (src_dtype == DLCS_BF16 && dst_dtype == DLCS_F32)
        hipLaunchKernelGGL((gather_rows_kernel<bf16, float>), g, b, 0, st, (const bf16*)src, idx, (float*)dst, nrows, (int)C, ld_src, ld_dst);
    else
        hipLaunchKernelGGL((gather_rows_kernel<bf16, bf16>), g, b, 0, st, (const bf16*)src, idx, (bf16*)dst, nrows, (int)C, ld_src, ld_dst);
    return dlcs_launch_status();
}

int dlcs_layernorm_fwd(int out_dtype, const float* x, const int32_t* src_map, const float* gamma,
                       const float* beta, float eps, void* out, float* mean, float* rstd,
                       int64_t rows, int64_t C, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(x && gamma && beta && out && mean && rstd && rows > 0 && C > 0 && C <= 64 * kLnMax);
    dim3 g(cdiv(rows, 4)), b(256);
    hipStream_t st = (hipStream_t)stream;
    if (out_dtype == DLCS_F32)
        hipLaunchKernelGGL(layernorm_fwd_kernel<float>, g, b, 0, st, x, src_map, gamma, beta, eps, (float*)out, mean, rstd, rows, (int)C);
    else
        hipLaunchKernelGGL(layernorm_fwd_kernel<bf16>, g, b, 0, st, x, src_map, gamma, beta, eps, (bf16*)out, mean, rstd, rows, (int)C);
    return dlcs_launch_status();
}

static inline long ln_bwd_blocks(long rows) { return (rows + 4 * kLnRows - 1) / (4 * kLnRows); }

size_t dlcs_layernorm_bwd_workspace_bytes(int64_t rows, int64_t C) {
    return (size_t)ln_bwd_blocks(rows) * 2 * (size_t)C * sizeof(float);
}

int dlcs_layernorm_bwd(const float* dy, const float* x, const int32_t* src_map, const float* gamma,
                       const float* mean, const float* rstd, const float* dx_in, float* dx, float* dgamma, float* dbeta,
                       int64_t rows, int64_t C, void* workspace, size_t workspace_bytes, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(dy && x && gamma && mean && rstd && dx && rows > 0 && C > 0 && C <= 64 * kLnMax);
    hipStream_t st = (hipStream_t)stream;
    if (C > 64 * kLnBwdMax) {
        const int rpb = 16;
        hipLaunchKernelGGL(layernorm_bwd_generic_kernel, dim3(cdiv(rows, rpb)), dim3(256), 0, st,
                           dy, x, src_map, gamma, mean, rstd, dx_in, dx, dgamma, dbeta, rows, (int)C, rpb);
        return dlcs_launch_status();
    }
    const long nblk = ln_bwd_blocks(rows);
    float* part = nullptr;
    if (workspace && (dgamma || dbeta)) {
        if (workspace_bytes < dlcs_layernorm_bwd_workspace_bytes(rows, C)) return DLCS_ERR_WORKSPACE;
        part = reinterpret_cast<float*>(workspace);
    }
    const int km = (int)((C + 63) / 64);
#define DLCS_LN_BWD(KM_)                                                                                   \
    hipLaunchKernelGGL(layernorm_bwd_kernel<KM_>, dim3((unsigned)nblk), dim3(256), 0, st, dy, x, src_map, gamma, \
                       mean, rstd, dx_in, dx, dgamma, dbeta, part, rows, (int)C)
    if (km <= 1) DLCS_LN_BWD(1);
    else if (km == 2) DLCS_LN_BWD(2);
    else if (km == 3) DLCS_LN_BWD(3);
    else DLCS_LN_BWD(4);
#undef DLCS_LN_BWD
    if (part)
        hipLaunchKernelGGL(layernorm_bwd_reduce_kernel, dim3(cdiv(2 * C, 64), kLnRed), dim3(256), 0, st, part, (int)nblk,
                           (int)C, dgamma, dbeta);
    return dlcs_launch_status();
}

int dlcs_colsum(int dtype, const void* x, int64_t rows, int64_t C, int64_t ld, float* out, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(x && out && rows > 0 && C > 0 && ld >= C);
    hipStream_t st = (hipStream_t)stream;
    if (ld % 8 == 0 && ((uintptr_t)x & 15) == 0 && C <= 2048) {
        // ~2048 workgroups, >= 64 rows each
        long rpb = std::max<long>(64, (rows + 2047) / 2048);
        const unsigned nb = (unsigned)((rows + rpb - 1) / rpb);
        if (dtype == DLCS_F32)
            hipLaunchKernelGGL(colsum_vec_kernel<float>, dim3(nb), dim3(256), 0, st, (const float*)x, rows, (int)C, ld, out, rpb);
        else
            hipLaunchKernelGGL(colsum_vec_kernel<bf16>, dim3(nb), dim3(256), 0, st, (const bf16*)x, rows, (int)C, ld, out, rpb);
        return dlcs_launch_status();
    }
    const int rpb = 128;
    dim3 g(cdiv(rows, rpb)), b(256);
    if (dtype == DLCS_F32)
        hipLaunchKernelGGL(colsum_kernel<float>, g, b, 0, st, (const float*)x, rows, (int)C, ld, out, rpb);
    else
        hipLaunchKernelGGL(colsum_kernel<bf16>, g, b, 0, st, (const bf16*)x, rows, (int)C, ld, out, rpb);
    return dlcs_launch_status();
}

#define DLCS_PREPOST_CHECK() \
    DLCS_CHECK_ARG(B > 0 && E > 0 && Tn > 0 && (Tn + 2 * pad) % 4 == 0 && Y % 4 == 0 && X % 4 == 0 && ldc >= 2 * E)

int dlcs_swin_pre(int dtype, const void* x, void* u, int64_t B, int64_t E, int64_t Tn, int64_t Y, int64_t X,
                  int64_t pad, int64_t ldc, dlcs_stream_t stream) {
    DLCS_PREPOST_CHECK();
    const long n = B * (Tn + 2 * pad) * Y * X;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == DLCS_F32)
        hipLaunchKernelGGL(swin_pre_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, (const float2*)x, (float*)u, (int)B, (int)E, (int)Tn, (int)Y, (int)X, (int)pad, (int)ldc);
    else
        hipLaunchKernelGGL(swin_pre_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, (const float2*)x, (bf16*)u, (int)B, (int)E, (int)Tn, (int)Y, (int)X, (int)pad, (int)ldc);
    return dlcs_launch_status();
}

int dlcs_swin_pre_bwd(int dtype, const void* gu, void* gx, int64_t B, int64_t E, int64_t Tn, int64_t Y, int64_t X,
                      int64_t pad, int64_t ldc, dlcs_stream_t stream) {
    DLCS_PREPOST_CHECK();
    const long n = B * E * Tn * Y * X;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == DLCS_F32)
        hipLaunchKernelGGL(swin_pre_bwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, (const float*)gu, (float2*)gx, (int)B, (int)E, (int)Tn, (int)Y, (int)X, (int)pad, (int)ldc);
    else
        hipLaunchKernelGGL(swin_pre_bwd_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, (const bf16*)gu, (float2*)gx, (int)B, (int)E, (int)Tn, (int)Y, (int)X, (int)pad, (int)ldc);
    return dlcs_launch_status();
}

int dlcs_swin_post(int dtype, const void* o, void* out, int64_t B, int64_t E, int64_t Tn, int64_t Y, int64_t X,
                   int64_t pad, int64_t ldc, dlcs_stream_t stream) {
    DLCS_PREPOST_CHECK();
    const long n = B * E * Tn * Y * X;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == DLCS_F32)
        hipLaunchKernelGGL(swin_post_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, (const float*)o, (float2*)out, (int)B, (int)E, (int)Tn, (int)Y, (int)X, (int)pad, (int)ldc);
    else
        hipLaunchKernelGGL(swin_post_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, (const bf16*)o, (float2*)out, (int)B, (int)E, (int)Tn, (int)Y, (int)X, (int)pad, (int)ldc);
    return dlcs_launch_status();
}

int dlcs_swin_post_bwd(int dtype, const void* gout, void* go, int64_t B, int64_t E, int64_t Tn, int64_t Y, int64_t X,
                       int64_t pad, int64_t ldc, dlcs_stream_t stream) {
    DLCS_PREPOST_CHECK();
    const long n = B * (Tn + 2 * pad) * Y * X;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == DLCS_F32)
        hipLaunchKernelGGL(swin_post_bwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, (const float2*)gout, (float*)go, (int)B, (int)E, (int)Tn, (int)Y, (int)X, (int)pad, (int)ldc);
    else
        hipLaunchKernelGGL(swin_post_bwd_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, (const float2*)gout, (bf16*)go, (int)B, (int)E, (int)Tn, (int)Y, (int)X, (int)pad, (int)ldc);
    return dlcs_launch_status();
}

int dlcs_cast_multi_bf16(int64_t count, const float* const* src, void* const* dst, const int64_t* n,
                         dlcs_stream_t stream) {
    DLCS_CHECK_ARG(count >= 0 && count <= DLCS_CAST_MULTI_MAX && (count == 0 || (src && dst && n)));
    if (count == 0) return 0;
    CastMultiArgs a{};
    int64_t nmax = 0;
    for (int64_t i = 0; i < count; ++i) {
        DLCS_CHECK_ARG(n[i] >= 0 && (n[i] == 0 || (src[i] && dst[i])));
        a.src[i] = src[i];
        a.dst[i] = reinterpret_cast<bf16*>(dst[i]);
        a.n[i] = n[i];
        nmax = std::max(nmax, n[i]);
    }
    if (nmax == 0) return 0;
    const unsigned gx = (unsigned)std::min<int64_t>(1024, (nmax + 1023) / 1024);
    hipLaunchKernelGGL(cast_multi_kernel, dim3(gx, (unsigned)count), dim3(256), 0, (hipStream_t)stream, a);
    return dlcs_launch_status();
}

int dlcs_axpby(int x_dtype, int y_dtype, const void* x, void* y, int64_t n, float a, float b, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(x && y && n >= 0);
    if (n == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    dim3 g(grid_for(n)), bl(256);
    if (x_dtype == DLCS_F32 && y_dtype == DLCS_F32)
        hipLaunchKernelGGL((axpby_kernel<float, float>), g, bl, 0, st, (const float*)x, (float*)y, n, a, b);
    else if (x_dtype == DLCS_F32 && y_dtype == DLCS_BF16)
        hipLaunchKernelGGL((axpby_kernel<float, bf16>), g, bl, 0, st, (const float*)x, (bf16*)y, n, a, b);
    else if (x_dtype == DLCS_BF16 && y_dtype == DLCS_F32)
        hipLaunchKernelGGL((axpby_kernel<bf16, float>), g, bl, 0, st, (const bf16*)x, (float*)y, n, a, b);
    else
        hipLaunchKernelGGL((axpby_kernel<bf16, bf16>), g, bl, 0, st, (const bf16*)x, (bf16*)y, n, a, b);
    return dlcs_launch_status();
}

int dlcs_relu_grad(int g_dtype, void* g, int a_dtype, const void* a, int64_t n, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(g && a && n >= 0);
    if (n == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    dim3 gr(grid_for((n + 7) / 8)), bl(256);
    if (g_dtype == DLCS_F32 && a_dtype == DLCS_F32)
        hipLaunchKernelGGL((relu_grad_kernel<float, float>), gr, bl, 0, st, (float*)g, (const float*)a, n);
    else if (g_dtype == DLCS_F32 && a_dtype == DLCS_BF16)
        hipLaunchKernelGGL((relu_grad_kernel<float, bf16>), gr, bl, 0, st, (float*)g, (const bf16*)a, n);
    else if (g_dtype == DLCS_BF16 && a_dtype == DLCS_F32)
        hipLaunchKernelGGL((relu_grad_kernel<bf16, float>), gr, bl, 0, st, (bf16*)g, (const float*)a, n);
    else
        hipLaunchKernelGGL((relu_grad_kernel<bf16, bf16>), gr, bl, 0, st, (bf16*)g, (const bf16*)a, n);
    return dlcs_launch_status();
}

int dlcs_permute(int src_dtype, int dst_dtype, const void* src, void* dst, int64_t ndim,
                 const int64_t* dst_shape, const int64_t* src_strides, int accumulate, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(src && dst && ndim >= 1 && ndim <= 6 && dst_shape && src_strides);
    PermArgs pa{};
    long total = 1;
    for (int k = 0; k < ndim; ++k) { pa.v[k] = dst_shape[k]; pa.v[6 + k] = src_strides[k]; total *= dst_shape[k]; }
    if (total == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    dim3 g(grid_for(total)), b(256);
    if (src_dtype == DLCS_F32 && dst_dtype == DLCS_F32)
        hipLaunchKernelGGL((permute_kernel_v<float, float>), g, b, 0, st, (const float*)src, (float*)dst, (int)ndim, pa, total, accumulate);
    else if (src_dtype == DLCS_F32 && dst_dtype == DLCS_BF16)
        hipLaunchKernelGGL((permute_kernel_v<float, bf16>), g, b, 0, st, (const float*)src, (bf16*)dst, (int)ndim, pa, total, accumulate);
    else if (src_dtype == DLCS_BF16 && dst_dtype == DLCS_F32)
        hipLaunchKernelGGL((permute_kernel_v<bf16, float>), g, b, 0, st, (const bf16*)src, (float*)dst, (int)ndim, pa, total, accumulate);
    else
        hipLaunchKernelGGL((permute_kernel_v<bf16, bf16>), g, b, 0, st, (const bf16*)src, (bf16*)dst, (int)ndim, pa, total, accumulate);
    return dlcs_launch_status();
}

int dlcs_block_layout(int src_dtype, int dst_dtype, const void* src, void* dst, int64_t B, int64_t C, int64_t D,
                      int64_t H, int64_t W, int64_t ld, int inverse, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(src && dst && B > 0 && C > 0 && D > 0 && H > 0 && W > 0 && ld >= C);
    const long n = inverse ? B * C * D * H * W : B * ((D + 3) / 4) * ((H + 3) / 4) * ((W + 3) / 4) * 64 * ld;
    hipStream_t st = (hipStream_t)stream;
    dim3 g(grid_for(n)), b(256);
#define DLCS_BL(TI, TO)                                                                                      \
    do {                                                                                                     \
        if (inverse) hipLaunchKernelGGL((from_blocked_kernel<TI, TO>), g, b, 0, st, (const TI*)src, (TO*)dst, \
                                        (int)B, (int)C, (int)D, (int)H, (int)W, (int)ld);                    \
        else hipLaunchKernelGGL((to_blocked_kernel<TI, TO>), g, b, 0, st, (const TI*)src, (TO*)dst, (int)B,   \
                                (int)C, (int)D, (int)H, (int)W, (int)ld);                                    \
    } while (0)
    if (src_dtype == DLCS_F32 && dst_dtype == DLCS_F32) DLCS_BL(float, float);
    else if (src_dtype == DLCS_F32 && dst_dtype == DLCS_BF16) DLCS_BL(float, bf16);
    else if (src_dtype == DLCS_BF16 && dst_dtype == DLCS_F32) DLCS_BL(bf16, float);
    else DLCS_BL(bf16, bf16);
#undef DLCS_BL
    return dlcs_launch_status();
}

int dlcs_fill_bias(float* out, const float* bias, int64_t rows, int64_t C, int64_t period, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(out && rows > 0 && C > 0 && period > 0);
    hipLaunchKernelGGL(fill_bias_kernel, dim3(grid_for(rows * C)), dim3(256), 0, (hipStream_t)stream, out, bias, rows, (int)C, (int)period);
    return dlcs_launch_status();
}

}  // extern "C"
