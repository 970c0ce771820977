// Generic MFMA GEMM with fused epilogues (gfx950).
//
//   C[m, n] (+)= epi( sum_k A(m, k) * B(n, k) )
//   A(m, k) = a_trans ? A[k*lda + m] : A[m*lda + k]
//   B(n, k) = b_trans ? B[k*ldb + n] : B[n*ldb + k]      (b_trans = 0: nn.Linear weight layout)
//   epi(v) = alpha * act(v + bias[n]) + res_scale * residual[row(m), n] + res2_scale * residual2[row(m), n],
//   row(m) = row_map ? row_map[m] : m
//   act: 0 none, 1 GELU(erf) (vst:29; pre-activation also written to aux when given), 4 GELU(tanh) (dit:322),
//        2 GELU backward: v * gelu'(aux[m, n]), 3 ReLU (the next ConvBlock's pre-activation)
//        5 GELU(tanh) backward, 6 ReLU backward: v * (aux > 0), 7 ReLU after the residuals
//   alpha: DropPath scale (1/keep, vst:266-271) on the residual branch
//   accumulate: C += (fp32 C uses atomic adds, which also implements split-K)
//
// Serves every nn.Linear of the Swin block (qkv / proj / fc1 / fc2; vst:131,
// :133, :27-29) forward and backward, the k4s4 patch embed / unembed
// (vst:455, :503) as plain GEMMs on the patch-blocked activation layout, and
// their weight gradients (split-K over tokens).
//
// Tiling: WM x WN waves, each TM x TN tiles of 32x32 (v_mfma_f32_32x32x16_bf16,
// or 8 x v_mfma_f32_32x32x2_f32 for the fp32 build), BK = 32, register-staged
// global loads of the next K tile issued before the MFMAs of the current one.
#include "dlcs_common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace {

constexpr int BK = 32;

struct GemmArgs {
    const void* A; const void* B; void* C;
    const float* bias; const void* aux; void* aux_out; const void* res; const void* res2; const int32_t* row_map;
    float alpha, res_scale, res2_scale;
    long M, N, K, lda, ldb, ldc, ldaux, ldr, ldr2;
    int a_trans, b_trans, act, c_f32, r_f32, r2_f32, accumulate;
    long kchunk;   // K range per blockIdx.z
    float* part;   // deterministic split-K: raw partial of K range z at part + z M ldc (f32 kernel only)
};

template <typename T> struct Pad;
template <> struct Pad<bf16> { static constexpr int v = 8; };
template <> struct Pad<float> { static constexpr int v = 4; };

// load 8 consecutive-in-memory elements starting at p (n_valid of them valid)
template <typename T>
DLCS_DEV Frag8<T> load_chunk(const T* p, int n_valid, bool aligned) {
    if (n_valid >= 8 && aligned) return load8<T>(p);
    Frag8<T> f = zero8<T>();
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if (i < n_valid) f.v[i] = p[i];
    return f;
}

// Stage one operand tile [ROWS][BK] of X(row, k) into registers.
// trans = 0: X[row*ld + k] (k contiguous); trans = 1: X[k*ld + row] (row contiguous).
template <typename T, int ROWS, int NTHR>
struct TileLoader {
    static constexpr int CHUNKS = ROWS * BK / 8;
    static constexpr int PER = (CHUNKS + NTHR - 1) / NTHR;
    Frag8<T> r[PER];

    DLCS_DEV void load(const T* X, long ld, int trans, long row0, long nrows, long k0, long kend) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int c = threadIdx.x + i * NTHR;
            r[i] = zero8<T>();
            if (c >= CHUNKS) continue;
            if (!trans) {
                const int row = c / (BK / 8), kc = (c % (BK / 8)) * 8;
                const long gr = row0 + row, gk = k0 + kc;
                if (gr < nrows && gk < kend) {
                    const T* p = X + gr * ld + gk;
                    const bool al = ((reinterpret_cast<uintptr_t>(p) & 15) == 0);
                    r[i] = load_chunk<T>(p, (int)min<long>(8, kend - gk), al);
                }
            } else {
                const int krow = c / (ROWS / 8), rc = (c % (ROWS / 8)) * 8;
                const long gk = k0 + krow, gr = row0 + rc;
                if (gk < kend && gr < nrows) {
                    const T* p = X + gk * ld + gr;
                    const bool al = ((reinterpret_cast<uintptr_t>(p) & 15) == 0);
                    r[i] = load_chunk<T>(p, (int)min<long>(8, nrows - gr), al);
                }
            }
        }
    }

    DLCS_DEV void store(T* S, int trans) const {
        constexpr int LD = BK + Pad<T>::v;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int c = threadIdx.x + i * NTHR;
            if (c >= CHUNKS) continue;
            if (!trans) {
                const int row = c / (BK / 8), kc = (c % (BK / 8)) * 8;
                *reinterpret_cast<decltype(r[i].v)*>(S + row * LD + kc) = r[i].v;
            } else {
                const int krow = c / (ROWS / 8), rc = (c % (ROWS / 8)) * 8;
#pragma unroll
                for (int j = 0; j < 8; ++j) S[(rc + j) * LD + krow] = r[i].v[j];
            }
        }
    }
};

template <typename T>
DLCS_DEV float load_as_f(const void* p, long idx, int is_f32) {
    return is_f32 ? reinterpret_cast<const float*>(p)[idx] : to_f(reinterpret_cast<const T*>(p)[idx]);
}

template <typename T, int WM, int WN, int TM, int TN>
__global__ void __launch_bounds__(WM * WN * 64) gemm_kernel(GemmArgs g) {
    constexpr int NTHR = WM * WN * 64;
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    constexpr int LD = BK + Pad<T>::v;
    __shared__ __attribute__((aligned(16))) T As[BM * LD];
    __shared__ __attribute__((aligned(16))) T Bs[BN * LD];

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const long m0 = (long)blockIdx.x * BM, n0 = (long)blockIdx.y * BN;
    const long kbeg = (long)blockIdx.z * g.kchunk;
    const long kend = min(g.K, kbeg + g.kchunk);
    const T* A = reinterpret_cast<const T*>(g.A);
    const T* B = reinterpret_cast<const T*>(g.B);

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16)0.0f;

    TileLoader<T, BM, NTHR> la;
    TileLoader<T, BN, NTHR> lb;
    if (kbeg < kend) {
        la.load(A, g.lda, g.a_trans, m0, g.M, kbeg, kend);
        lb.load(B, g.ldb, g.b_trans, n0, g.N, kbeg, kend);
    }
    for (long k0 = kbeg; k0 < kend; k0 += BK) {
        __syncthreads();
        la.store(As, g.a_trans);
        lb.store(Bs, g.b_trans);
        __syncthreads();
        if (k0 + BK < kend) {
            la.load(A, g.lda, g.a_trans, m0, g.M, k0 + BK, kend);
            lb.load(B, g.ldb, g.b_trans, n0, g.N, k0 + BK, kend);
        }
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
            const int kof = kk * 16 + 8 * (lane >> 5);
            Frag8<T> af[TM], bfr[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = load8<T>(As + (wm * TM * 32 + i * 32 + (lane & 31)) * LD + kof);
#pragma unroll
            for (int j = 0; j < TN; ++j) bfr[j] = load8<T>(Bs + (wn * TN * 32 + j * 32 + (lane & 31)) * LD + kof);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) mfma32(acc[i][j], af[i], bfr[j]);
        }
    }

    // epilogue
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const long n = n0 + wn * TN * 32 + j * 32 + (lane & 31);
            if (n >= g.N) continue;
            const float bias = g.bias ? g.bias[n] : 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const long m = m0 + wm * TM * 32 + i * 32 + acc_row(r, lane);
                if (m >= g.M) continue;
                long orow = m;
                if (g.row_map) {
                    orow = g.row_map[m];
                    if (orow < 0) continue;
                }
                float v = acc[i][j][r] + bias;
                if (act_is_fwd(g.act)) {
                    if (g.aux_out && g.act != 3) reinterpret_cast<T*>(g.aux_out)[m * g.ldaux + n] = from_f<T>(v);
                    v = act_fwd(g.act, v);
                } else if (act_is_grad(g.act)) {
                    v *= act_grad_scale(g.act, to_f(reinterpret_cast<const T*>(g.aux)[m * g.ldaux + n]));
                }
                v *= g.alpha;
                if (g.res) v += g.res_scale * load_as_f<T>(g.res, orow * g.ldr + n, g.r_f32);
                if (g.res2) v += g.res2_scale * load_as_f<T>(g.res2, orow * g.ldr2 + n, g.r2_f32);
                if (g.act == 7) v = fmaxf(v, 0.0f);
                const long ci = orow * g.ldc + n;
                if (g.c_f32) {
                    float* C = reinterpret_cast<float*>(g.C);
                    if (g.accumulate) atomicAdd(C + ci, v);
                    else C[ci] = v;
                } else {
                    T* C = reinterpret_cast<T*>(g.C);
                    if (g.accumulate) v += to_f(C[ci]);
                    C[ci] = from_f<T>(v);
                }
            }
        }
    }
}

// ---------------------------------------------------------------- v2 (bf16)
// 256 threads = 2 x 2 waves, wave tile (BM/2) x (BN/2) of 16x16x32 MFMA tiles,
// BK = 64 per LDS stage (single buffer, next stage register-prefetched).
// Operands are staged in their memory layout with 16-B copies: a k-contiguous
// operand as [rows][BK + 8] read by ds_read_b128; a row-contiguous ("trans")
// operand as [BK][rows (+ pad)] read k-contiguous by ds_read_b64_tr_b16,
// its 16-column tiles XOR-swizzled by bit 3 of k so the two 16-lane groups of
// a read (k rows 8 apart) hit disjoint banks.  Epilogue through LDS in two
// halves (64-row slabs of fp32): bias, act, alpha, residual, row_map and the
// output as 16-B accesses per 8 columns.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;

constexpr int BK2 = 64;

DLCS_DEV bf16x8_t tr_read_b16(const bf16* p0, const bf16* p1) {
    const v4s_t r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(const_cast<bf16*>(p0)));
    const v4s_t r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(const_cast<bf16*>(p1)));
    typedef short v8s __attribute__((ext_vector_type(8)));
    const v8s both = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3]};
    return __builtin_bit_cast(bf16x8_t, both);
}

template <int ROWS, int TRANS>
struct Stage2 {
    // LDS image geometry
    // trans rows: (LD / 2) % 64 in {16, 48} dwords so 4 consecutive k rows start
    // on distinct 16-bank groups (160 -> 160, 64 -> 96, 128 -> 160)
    static constexpr int LD = TRANS ? (((ROWS / 2) % 32 == 16) ? ROWS : ROWS + 32) : BK2 + 8;
    static constexpr int SIZE = TRANS ? BK2 * LD : ROWS * LD;      // bf16
    static constexpr int CHUNKS = ROWS * BK2 / 8;
    static constexpr int PER = (CHUNKS + 255) / 256;
    bf16x8_t r[PER];

    DLCS_DEV void load(const bf16* X, long ld, long row0, long nrows, long k0, long kend) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int c = threadIdx.x + i * 256;
            r[i] = (bf16x8_t)(bf16)0.0f;
            if (c >= CHUNKS) continue;
            long gr, gk;
            if (!TRANS) { gr = row0 + c / (BK2 / 8); gk = k0 + (c % (BK2 / 8)) * 8; }
            else { gk = k0 + c / (ROWS / 8); gr = row0 + (c % (ROWS / 8)) * 8; }
            if (gr < nrows && gk < kend)
                r[i] = *reinterpret_cast<const bf16x8_t*>(X + (TRANS ? gk * ld + gr : gr * ld + gk));
        }
    }
    DLCS_DEV void store(bf16* S) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int c = threadIdx.x + i * 256;
            if (c >= CHUNKS) continue;
            if (!TRANS) {
                *reinterpret_cast<bf16x8_t*>(S + (c / (BK2 / 8)) * LD + (c % (BK2 / 8)) * 8) = r[i];
            } else {
                const int kr = c / (ROWS / 8), col = ((c % (ROWS / 8)) * 8) ^ (((kr >> 3) & 1) << 4);
                *reinterpret_cast<bf16x8_t*>(S + kr * LD + col) = r[i];
            }
        }
    }
    // fragment of 16 rows starting at tile row t0, k-step ks (32 k), lane layout of
    // the 16x16x32 operand: row t0 + (lane & 15), k = 32 ks + 8 (lane >> 4) + j
    DLCS_DEV bf16x8_t frag(const bf16* S, int t0, int ks, int lane) const {
        if (!TRANS) {
            return *reinterpret_cast<const bf16x8_t*>(S + (t0 + (lane & 15)) * LD + 32 * ks + 8 * (lane >> 4));
        } else {
            const int gq = lane >> 4, q = (lane >> 2) & 3, p4 = (lane & 3) * 4;
            const bf16* p0 = S + (32 * ks + 8 * gq + q) * LD + ((t0 ^ ((gq & 1) << 4)) + p4);
            return tr_read_b16(p0, p0 + 4 * LD);
        }
    }
};

template <int BM, int BN, int AT, int BT>
__global__ void __launch_bounds__(256) gemm_v2_kernel(GemmArgs g) {
    using SA = Stage2<BM, AT>;
    using SB = Stage2<BN, BT>;
    constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
    constexpr int OPS = SA::SIZE + SB::SIZE;                       // bf16
    constexpr int EPI = WM * (BN + 4) * 2;                         // fp32 slab, in bf16 units
    __shared__ __attribute__((aligned(16))) bf16 smem[OPS > EPI ? OPS : EPI];
    bf16* As = smem;
    bf16* Bs = smem + SA::SIZE;

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const long m0 = (long)blockIdx.x * BM, n0 = (long)blockIdx.y * BN;
    const long kbeg = (long)blockIdx.z * g.kchunk;
    const long kend = min(g.K, kbeg + g.kchunk);
    const bf16* A = reinterpret_cast<const bf16*>(g.A);
    const bf16* B = reinterpret_cast<const bf16*>(g.B);

    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4_t)0.0f;

    SA la;
    SB lb;
    if (kbeg < kend) {
        la.load(A, g.lda, m0, g.M, kbeg, kend);
        lb.load(B, g.ldb, n0, g.N, kbeg, kend);
    }
    for (long k0 = kbeg; k0 < kend; k0 += BK2) {
        __syncthreads();
        la.store(As);
        lb.store(Bs);
        __syncthreads();
        if (k0 + BK2 < kend) {
            la.load(A, g.lda, m0, g.M, k0 + BK2, kend);
            lb.load(B, g.ldb, n0, g.N, k0 + BK2, kend);
        }
#pragma unroll
        for (int ks = 0; ks < BK2 / 32; ++ks) {
            bf16x8_t af[TM];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = la.frag(As, wm * WM + 16 * i, ks, lane);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const bf16x8_t bfr = lb.frag(Bs, wn * WN + 16 * j, ks, lane);
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
            }
        }
    }

    // ---- epilogue: two 64-row (WM) slabs through LDS
    float* E = reinterpret_cast<float*>(smem);
    constexpr int EL = BN + 4;
    constexpr int NCH = BN / 8;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        __syncthreads();
        if (wm == h) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        E[(16 * i + (lane >> 4) * 4 + r) * EL + wn * WN + 16 * j + (lane & 15)] = acc[i][j][r];
        }
        __syncthreads();
        if (g.c_f32 && g.accumulate && gridDim.z > 1) {
            // split-K partial sums: fp32 atomics, one column per lane so a wave
            // adds 256 contiguous bytes (full atomic rate); plain epilogue terms
            // (bias, act, residual) are not allowed with split-K
            for (int c = threadIdx.x; c < WM * BN; c += 256) {
                const int rl = c / BN, cc = c % BN;
                const long m = m0 + h * WM + rl, n = n0 + cc;
                if (m >= g.M || n >= g.N) continue;
                const long orow = g.row_map ? (long)g.row_map[m] : m;
                if (orow < 0) continue;
                atomicAdd(reinterpret_cast<float*>(g.C) + orow * g.ldc + n, g.alpha * E[rl * EL + cc]);
            }
            continue;
        }
        for (int c = threadIdx.x; c < WM * NCH; c += 256) {
            const int rl = c / NCH, cc = (c % NCH) * 8;
            const long m = m0 + h * WM + rl, n = n0 + cc;
            if (m >= g.M || n >= g.N) continue;
            long orow = m;
            if (g.row_map) {
                orow = g.row_map[m];
                if (orow < 0) continue;
            }
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = E[rl * EL + cc + e] + (g.bias ? g.bias[n + e] : 0.0f);
            if (act_is_fwd(g.act)) {
                if (g.aux_out && g.act != 3) {
                    bf16x8_t o;
#pragma unroll
                    for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
                    *reinterpret_cast<bf16x8_t*>(reinterpret_cast<bf16*>(g.aux_out) + m * g.ldaux + n) = o;
                }
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = act_fwd(g.act, v[e]);
            } else if (act_is_grad(g.act)) {
                const bf16x8_t ax = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const bf16*>(g.aux) + m * g.ldaux + n);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] *= act_grad_scale(g.act, (float)ax[e]);
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] *= g.alpha;
            auto add_res = [&](const void* R, long ldr, int rf32, float sc) {
                if (rf32) {
                    const float* rp = reinterpret_cast<const float*>(R) + orow * ldr + n;
                    const f32x4_t r0 = *reinterpret_cast<const f32x4_t*>(rp), r1 = *reinterpret_cast<const f32x4_t*>(rp + 4);
#pragma unroll
                    for (int e = 0; e < 4; ++e) { v[e] += sc * r0[e]; v[4 + e] += sc * r1[e]; }
                } else {
                    const bf16x8_t rr = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const bf16*>(R) + orow * ldr + n);
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += sc * (float)rr[e];
                }
            };
            if (g.res) add_res(g.res, g.ldr, g.r_f32, g.res_scale);
            if (g.res2) add_res(g.res2, g.ldr2, g.r2_f32, g.res2_scale);
            if (g.act == 7) {
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.0f);
            }
            const long ci = orow * g.ldc + n;
            if (g.c_f32) {
                float* C = reinterpret_cast<float*>(g.C) + ci;
                f32x4_t o0, o1;
#pragma unroll
                for (int e = 0; e < 4; ++e) { o0[e] = v[e]; o1[e] = v[4 + e]; }
                if (g.accumulate) {          // sole writer of the element (no split-K): plain RMW
                    o0 += *reinterpret_cast<const f32x4_t*>(C);
                    o1 += *reinterpret_cast<const f32x4_t*>(C + 4);
                }
                *reinterpret_cast<f32x4_t*>(C) = o0;
                *reinterpret_cast<f32x4_t*>(C + 4) = o1;
            } else {
                bf16* C = reinterpret_cast<bf16*>(g.C) + ci;
                if (g.accumulate) {
                    const bf16x8_t pv = *reinterpret_cast<const bf16x8_t*>(C);
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += (float)pv[e];
                }
                bf16x8_t o;
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
                *reinterpret_cast<bf16x8_t*>(C) = o;
            }
        }
    }
}

// ---------------------------------------------------------------- v3 (bf16, N % 160 == 0, K % 160 == 0)
// The fwd / dgrad GEMMs of the model all have N and K in {160, 480, 640, 10240}
// and M = tokens: K is one to four 160-deep stages, so v2's 64-deep stages made
// every tile a chain of 3-10 dependent load -> barrier -> MFMA rounds plus an
// epilogue whose bias / residual / aux loads were issued one chunk at a time.
// v3: tile 64 (m) x 160 (n), 4 waves of 32 x 80, one 160-deep stage per
// round trip ([64][168] A image + [160][168] or [160 k][160 n] B image, 75 KB:
// two workgroups per CU).  A workgroup owns one 160-column slice and a run of
// m-tiles; with K == 160 the weight slice is staged ONCE and stays resident
// while the A tiles stream through (the wide unembed / embed-dgrad GEMMs,
// N = 10240, then read their weights 16 x instead of 210 x).  The next stage is
// register-prefetched during the MFMAs; the epilogue is specialised per fused
// term (EPI flags) and issues all of its global loads (residuals, aux, the
// accumulated output, the row map) before the LDS round trip; the bias lives in
// LDS.  No split-K: the K = 10240 embed / unembed-dgrad GEMMs loop 64 stages.
constexpr int kG3M = 64, kG3N = 160, kG3K = 160;
constexpr int kG3LD = kG3K + 8;                 // k-contiguous image row (bf16)
constexpr int kG3EL = kG3N + 4;                 // epilogue slab row (fp32)
enum {
    kG3Bias = 1, kG3Gelu = 2, kG3GeluGrad = 4, kG3Relu = 8, kG3ResF32 = 16, kG3ResBf = 32, kG3Res2Bf = 64,
    kG3RowMap = 128, kG3OutF32 = 256, kG3Acc = 512, kG3Atomic = 1024
};

template <int BT, int EPI, int MULTI>
__global__ void __launch_bounds__(256, 2) gemm_v3_kernel(GemmArgs g, int nslices, int mgroups, int nsplit) {
    constexpr int A_SZ = kG3M * kG3LD;
    constexpr int B_SZ = BT ? kG3K * kG3N : kG3N * kG3LD;
    static_assert(32 * kG3EL * 2 <= A_SZ, "epilogue slab must fit the A image");
    __shared__ __attribute__((aligned(16))) bf16 smem3[A_SZ + B_SZ];
    __shared__ float bias_s[kG3N];
    bf16* As = smem3;
    bf16* Bs = smem3 + A_SZ;
    float* E = reinterpret_cast<float*>(smem3);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int split = blockIdx.x / (nslices * mgroups);
    const int slice = blockIdx.x % nslices, grp = (blockIdx.x / nslices) % mgroups;
    const long n0 = (long)slice * kG3N;
    const int mtiles = (int)((g.M + kG3M - 1) / kG3M);
    const int t0 = (int)((long)grp * mtiles / mgroups), t1 = (int)((long)(grp + 1) * mtiles / mgroups);
    // K stages of this workgroup: [ks0, ks0 + nks) (split-K only with kG3Atomic)
    const int nks_all = (int)(g.K / kG3K);
    const int ks0 = (int)((long)nks_all * split / nsplit);
    const int nks = (int)((long)nks_all * (split + 1) / nsplit) - ks0;
    const int total = (t1 - t0) * nks;
    const bf16* A = reinterpret_cast<const bf16*>(g.A);
    const bf16* B = reinterpret_cast<const bf16*>(g.B);

    if constexpr ((EPI & kG3Bias) != 0) {
        if (tid < kG3N) bias_s[tid] = g.bias[n0 + tid];
    }

    // register staging: A 1280 chunks (5 / thread), B 3200 (12.5 / thread)
    constexpr int APER = kG3M * (kG3K / 8) / 256, BCH = kG3N * (kG3K / 8), BPER = (BCH + 255) / 256;
    bf16x8_t ra[APER], rb[BPER];
    auto load_a = [&](int mt, int ks) {
#pragma unroll
        for (int i = 0; i < APER; ++i) {
            const int c = tid + 256 * i, r = c / 20, kc = c % 20;
            const long m = min((long)mt * kG3M + r, g.M - 1);      // tail rows: duplicates, never stored
            ra[i] = *reinterpret_cast<const bf16x8_t*>(A + m * g.lda + (long)(ks0 + ks) * kG3K + kc * 8);
        }
    };
    auto load_b = [&](int ks) {
#pragma unroll
        for (int i = 0; i < BPER; ++i) {
            const int c = tid + 256 * i;
            if (c < BCH) {
                const int r = c / 20, kc = c % 20;
                rb[i] = BT ? *reinterpret_cast<const bf16x8_t*>(B + ((long)(ks0 + ks) * kG3K + r) * g.ldb + n0 + kc * 8)
                           : *reinterpret_cast<const bf16x8_t*>(B + (n0 + r) * g.ldb + (long)(ks0 + ks) * kG3K + kc * 8);
            }
        }
    };
    auto store_a = [&]() {
#pragma unroll
        for (int i = 0; i < APER; ++i) {
            const int c = tid + 256 * i;
            *reinterpret_cast<bf16x8_t*>(As + (c / 20) * kG3LD + (c % 20) * 8) = ra[i];
        }
    };
    auto store_b = [&]() {
#pragma unroll
        for (int i = 0; i < BPER; ++i) {
            const int c = tid + 256 * i;
            if (c < BCH) {
                const int r = c / 20, cc = (c % 20) * 8;
                if (BT) *reinterpret_cast<bf16x8_t*>(Bs + r * kG3N + (cc ^ (((r >> 3) & 1) << 4))) = rb[i];
                else *reinterpret_cast<bf16x8_t*>(Bs + r * kG3LD + cc) = rb[i];
            }
        }
    };

    f32x4_t acc[2][5];
    // ---- epilogue: two 32-row slabs through the A image's LDS
    auto epilogue = [&](int mt) {
        const long m0 = (long)mt * kG3M;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            // this thread's 8-column chunks of the slab: c = tid + 256 i (640 chunks)
            constexpr int EIT = 3;
            long orow[EIT];
            bool ok[EIT];
            bf16x8_t rbf[EIT], r2bf[EIT], axv[EIT], pvb[EIT];
            f32x4_t rf0[EIT], rf1[EIT], pv0[EIT], pv1[EIT];
#pragma unroll
            for (int i = 0; i < EIT; ++i) {
                const int c = tid + 256 * i;
                const int rl = c / 20, cc = (c % 20) * 8;
                const long m = m0 + h * 32 + rl, n = n0 + cc;
                ok[i] = c < 640 && m < g.M;
                orow[i] = m;
                if constexpr ((EPI & kG3RowMap) != 0) {
                    if (ok[i]) orow[i] = g.row_map[m];
                    ok[i] = ok[i] && orow[i] >= 0;
                }
                if (!ok[i]) continue;
                if constexpr ((EPI & kG3ResF32) != 0) {
                    const float* rp = reinterpret_cast<const float*>(g.res) + orow[i] * g.ldr + n;
                    rf0[i] = *reinterpret_cast<const f32x4_t*>(rp);
                    rf1[i] = *reinterpret_cast<const f32x4_t*>(rp + 4);
                }
                if constexpr ((EPI & kG3ResBf) != 0)
                    rbf[i] = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const bf16*>(g.res) + orow[i] * g.ldr + n);
                if constexpr ((EPI & kG3Res2Bf) != 0)
                    r2bf[i] = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const bf16*>(g.res2) + orow[i] * g.ldr2 + n);
                if constexpr ((EPI & kG3GeluGrad) != 0)
                    axv[i] = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const bf16*>(g.aux) + m * g.ldaux + n);
                if constexpr ((EPI & kG3Acc) != 0 && (EPI & kG3Atomic) == 0) {
                    if constexpr ((EPI & kG3OutF32) != 0) {
                        const float* cp = reinterpret_cast<const float*>(g.C) + orow[i] * g.ldc + n;
                        pv0[i] = *reinterpret_cast<const f32x4_t*>(cp);
                        pv1[i] = *reinterpret_cast<const f32x4_t*>(cp + 4);
                    } else {
                        pvb[i] = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const bf16*>(g.C) + orow[i] * g.ldc + n);
                    }
                }
            }
            __syncthreads();                      // MFMA reads of As (h = 0) / slab reads (h = 1) done
            if (wm == h) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 5; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            E[(16 * i + (lane >> 4) * 4 + r) * kG3EL + wn * 80 + 16 * j + (lane & 15)] = acc[i][j][r];
            }
            __syncthreads();
            if constexpr ((EPI & kG3Atomic) != 0) {
                // split-K partial sums: lane-contiguous fp32 atomics (64 consecutive
                // floats of one row per wave instruction, the full-rate shape; the
                // 8-floats-per-lane chunk shape below runs several times slower)
                for (int j = tid; j < 32 * kG3N; j += 256) {
                    const int rl = j / kG3N, cc = j % kG3N;
                    const long m = m0 + h * 32 + rl;
                    if (m < g.M) atomicAdd(reinterpret_cast<float*>(g.C) + m * g.ldc + n0 + cc, g.alpha * E[rl * kG3EL + cc]);
                }
                continue;
            }
#pragma unroll
            for (int i = 0; i < EIT; ++i) {
                if (!ok[i]) continue;
                const int c = tid + 256 * i;
                const int rl = c / 20, cc = (c % 20) * 8;
                const long m = m0 + h * 32 + rl, n = n0 + cc;
                const f32x4_t e0 = *reinterpret_cast<const f32x4_t*>(E + rl * kG3EL + cc);
                const f32x4_t e1 = *reinterpret_cast<const f32x4_t*>(E + rl * kG3EL + cc + 4);
                float v[8];
#pragma unroll
                for (int e = 0; e < 4; ++e) { v[e] = e0[e]; v[4 + e] = e1[e]; }
                if constexpr ((EPI & kG3Bias) != 0) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += bias_s[cc + e];
                }
                if constexpr ((EPI & kG3Gelu) != 0) {
                    if (g.aux_out) {
                        bf16x8_t o;
#pragma unroll
                        for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
                        *reinterpret_cast<bf16x8_t*>(reinterpret_cast<bf16*>(g.aux_out) + m * g.ldaux + n) = o;
                    }
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
                }
                if constexpr ((EPI & kG3GeluGrad) != 0) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] *= gelu_erf_grad((float)axv[i][e]);
                }
                if constexpr ((EPI & kG3Relu) != 0) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.0f);
                }
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] *= g.alpha;
                if constexpr ((EPI & kG3ResF32) != 0) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) { v[e] += g.res_scale * rf0[i][e]; v[4 + e] += g.res_scale * rf1[i][e]; }
                }
                if constexpr ((EPI & kG3ResBf) != 0) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += g.res_scale * (float)rbf[i][e];
                }
                if constexpr ((EPI & kG3Res2Bf) != 0) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += g.res2_scale * (float)r2bf[i][e];
                }
                const long ci = orow[i] * g.ldc + n;
                if constexpr ((EPI & kG3OutF32) != 0) {
                    f32x4_t o0, o1;
#pragma unroll
                    for (int e = 0; e < 4; ++e) { o0[e] = v[e]; o1[e] = v[4 + e]; }
                    float* C = reinterpret_cast<float*>(g.C) + ci;
                    if constexpr ((EPI & kG3Atomic) != 0) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) { atomicAdd(C + e, o0[e]); atomicAdd(C + 4 + e, o1[e]); }
                    } else {
                        if constexpr ((EPI & kG3Acc) != 0) { o0 += pv0[i]; o1 += pv1[i]; }
                        *reinterpret_cast<f32x4_t*>(C) = o0;
                        *reinterpret_cast<f32x4_t*>(C + 4) = o1;
                    }
                } else {
                    bf16x8_t o;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        float x = v[e];
                        if constexpr ((EPI & kG3Acc) != 0) x += (float)pvb[i][e];
                        o[e] = (bf16)x;
                    }
                    *reinterpret_cast<bf16x8_t*>(reinterpret_cast<bf16*>(g.C) + ci) = o;
                }
            }
        }
    };

    if (total <= 0) return;
    if (!MULTI) {                                 // K == 160: the weight slice is staged once
        load_b(0);
        store_b();
    }
    load_a(t0, 0);
    if (MULTI) load_b(0);
    for (int it = 0; it < total; ++it) {
        const int mt = MULTI ? t0 + it / nks : t0 + it, ks = MULTI ? it % nks : 0;
        __syncthreads();                          // previous round's MFMAs / epilogue are done with LDS
        store_a();
        if (MULTI) store_b();
        __syncthreads();
        if (it + 1 < total) {
            if (MULTI) {
                load_a(t0 + (it + 1) / nks, (it + 1) % nks);
                load_b((it + 1) % nks);
            } else {
                load_a(t0 + it + 1, 0);
            }
        }
        if (ks == 0) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 5; ++j) acc[i][j] = (f32x4_t)0.0f;
        }
#pragma unroll
        for (int kk = 0; kk < kG3K / 32; ++kk) {
            bf16x8_t af[2];
#pragma unroll
            for (int i = 0; i < 2; ++i)
                af[i] = *reinterpret_cast<const bf16x8_t*>(As + (wm * 32 + 16 * i + (lane & 15)) * kG3LD + 32 * kk +
                                                           8 * (lane >> 4));
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const int t = wn * 80 + 16 * j;
                bf16x8_t bfr;
                if (BT) {
                    const int gq = lane >> 4, q = (lane >> 2) & 3, p4 = (lane & 3) * 4;
                    const bf16* p0 = Bs + (32 * kk + 8 * gq + q) * kG3N + ((t ^ ((gq & 1) << 4)) + p4);
                    bfr = tr_read_b16(p0, p0 + 4 * kG3N);
                } else {
                    bfr = *reinterpret_cast<const bf16x8_t*>(Bs + (t + (lane & 15)) * kG3LD + 32 * kk + 8 * (lane >> 4));
                }
#pragma unroll
                for (int i = 0; i < 2; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
            }
        }
        if (!MULTI) epilogue(mt);
    }
    if (MULTI) epilogue(t0);
}

static bool g3_disabled() {
    static const bool off = dlcs_knob("DLCS_GEMM_V2") != nullptr;
    return off;
}

// epilogue flags of a call, or -1 when v3 has no specialisation for it
static int g3_epi(const GemmArgs& g) {
    int e = 0;
    if (g.bias) e |= kG3Bias;
    if (g.act == 1) e |= kG3Gelu;
    else if (g.act == 2) e |= kG3GeluGrad;
    else if (g.act == 3) e |= kG3Relu;
    else if (g.act != 0) return -1;                      // acts 4-7 (DiT): v2 / generic
    if (g.res) e |= g.r_f32 ? kG3ResF32 : kG3ResBf;
    if (g.res2) {
        if (g.r2_f32) return -1;
        e |= kG3Res2Bf;
    }
    if (g.row_map) e |= kG3RowMap;
    if (g.c_f32) e |= kG3OutF32;
    if (g.accumulate) e |= kG3Acc;
    return e;
}

// the combinations the Swin / patch GEMMs use (engine.py); others go to v2
#define DLCS_G3_CASES(X)                                                                 \
    X(0, kG3Bias, 0)                                       /* qkv fwd */                  \
    X(0, kG3Bias | kG3ResF32 | kG3RowMap | kG3OutF32, 0)   /* proj fwd */                 \
    X(0, kG3Bias | kG3Gelu, 0)                             /* fc1 fwd */                  \
    X(0, kG3Bias | kG3ResF32 | kG3OutF32, 1)               /* fc2 fwd (K = 640) */        \
    X(0, kG3OutF32 | kG3Acc, 1)                            /* patch embed fwd (K = 10240) */ \
    X(0, kG3OutF32 | kG3Acc | kG3Atomic, 1)                /* (split-K variant) */        \
    X(0, kG3Bias | kG3Relu, 0)                             /* patch unembed fwd */        \
    X(1, kG3GeluGrad, 0)                                   /* fc1 dgrad (x gelu') */      \
    X(1, kG3OutF32, 1)                                     /* fc2 / qkv dgrad (K = 640 / 480) */ \
    X(1, 0, 0)                                             /* proj dgrad */               \
    X(1, kG3OutF32 | kG3Acc, 1)                            /* unembed dgrad (K = 10240) */ \
    X(1, kG3OutF32 | kG3Acc | kG3Atomic, 1)                /* (split-K variant) */        \
    X(1, kG3ResBf | kG3Res2Bf, 0)                          /* embed dgrad + skips */

static bool launch_v3(const GemmArgs& g, hipStream_t st) {
    if (g.a_trans || g.N % kG3N || g.K % kG3K) return false;
    int epi = g3_epi(g);
    if (epi < 0) return false;
    const int nslices = (int)(g.N / kG3N);
    const int mtiles = (int)((g.M + kG3M - 1) / kG3M);
    // K == 160: the weight slice stays resident, so give each workgroup a run
    // of m-tiles (~1024 workgroups); deeper K restages B per tile anyway
    int mgroups = mtiles;
    if (g.K == kG3K && (long)nslices * mtiles > 1024) mgroups = std::max(1, std::min(mtiles, 1024 / nslices));
    // deep K into fp32 (embed fwd / unembed dgrad, K = 10240): one workgroup per
    // m-tile would leave 210 workgroups looping 64 stages (~170 us); split K in
    // DLCS_GEMM_SPLIT (default 2: 160 -> 116 us; 4 and 8 splits measured slower)
    // ranges summed by lane-contiguous fp32 atomics
    int nsplit = 1;
    if (epi == (kG3OutF32 | kG3Acc) && g.K >= 16 * kG3K && (long)nslices * mgroups < 512) {
        static const int ns = [] { const char* e = dlcs_knob("DLCS_GEMM_SPLIT"); return e ? std::atoi(e) : 2; }();
        if (ns > 1) {
            nsplit = ns;
            epi |= kG3Atomic;
        }
    }
    const dim3 grid((unsigned)(nslices * mgroups * nsplit));
    const int key = (g.b_trans << 16) | ((g.K > kG3K) << 17) | epi;
    switch (key) {
#define DLCS_G3_LAUNCH(BT_, E_, MULTI_)                                                                        \
    case ((BT_) << 16) | ((MULTI_) << 17) | (E_):                                                            \
        hipLaunchKernelGGL((gemm_v3_kernel<BT_, E_, MULTI_>), grid, dim3(256), 0, st, g, nslices, mgroups, nsplit); \
        return true;
        DLCS_G3_CASES(DLCS_G3_LAUNCH)
#undef DLCS_G3_LAUNCH
        default:
            return false;
    }
}

template <int BM, int BN>
void launch_v2(const GemmArgs& g, int splitk, hipStream_t st) {
    dim3 grid(cdiv(g.M, BM), cdiv(g.N, BN), splitk);
    if (!g.a_trans && !g.b_trans) hipLaunchKernelGGL((gemm_v2_kernel<BM, BN, 0, 0>), grid, dim3(256), 0, st, g);
    else if (!g.a_trans && g.b_trans) hipLaunchKernelGGL((gemm_v2_kernel<BM, BN, 0, 1>), grid, dim3(256), 0, st, g);
    else if (g.a_trans && !g.b_trans) hipLaunchKernelGGL((gemm_v2_kernel<BM, BN, 1, 0>), grid, dim3(256), 0, st, g);
    else hipLaunchKernelGGL((gemm_v2_kernel<BM, BN, 1, 1>), grid, dim3(256), 0, st, g);
}

template <typename T, int WM, int WN, int TM, int TN>
void launch(const GemmArgs& g, int splitk, hipStream_t st) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    dim3 grid(cdiv(g.M, BM), cdiv(g.N, BN), splitk);
    hipLaunchKernelGGL((gemm_kernel<T, WM, WN, TM, TN>), grid, dim3(WM * WN * 64), 0, st, g);
}

#include "gemm_f32.inc"

template <typename T>
int gemm_dispatch(GemmArgs g, int splitk, hipStream_t st) {
    // split-K: round each K range to a multiple of BK
    if (splitk < 1) splitk = 1;
    long kc = (g.K + splitk - 1) / splitk;
    kc = ((kc + BK - 1) / BK) * BK;
    if (kc < BK) kc = BK;
    splitk = (int)((g.K + kc - 1) / kc);
    if (splitk < 1) splitk = 1;
    g.kchunk = kc;
    if (splitk > 1 && !(g.c_f32 && g.accumulate)) return DLCS_ERR_INVALID_ARG;
    if constexpr (std::is_same<T, bf16>::value) {
        auto al = [](const void* p) { return p == nullptr || ((uintptr_t)p & 15) == 0; };
        const bool vec = g.K % 8 == 0 && g.lda % 8 == 0 && g.ldb % 8 == 0 && g.N % 8 == 0 && g.ldc % 8 == 0 &&
                         (!g.a_trans || g.M % 8 == 0) && (!g.b_trans || g.N % 8 == 0) &&
                         (!g.res || g.ldr % 8 == 0) && (!g.res2 || g.ldr2 % 8 == 0) &&
                         (!(g.aux || g.aux_out) || g.ldaux % 8 == 0) &&
                         al(g.A) && al(g.B) && al(g.C) && al(g.res) && al(g.res2) && al(g.aux) && al(g.aux_out);
        if (vec) {
            if (!g3_disabled() && (splitk == 1 || (g.c_f32 && g.accumulate)) && launch_v3(g, st))
                return dlcs_launch_status();
            const int BN = (g.N % 160 == 0 && g.N <= 640) ? 160 : (g.N >= 128 ? 128 : 64);
            const long tiles128 = cdiv(g.M, 128) * cdiv(g.N, BN);
            const int BM = (tiles128 * splitk >= 512 || g.M > 4096 && BN != 160) ? 128 : 64;
            // more K splits when the output has few tiles (allowed: fp32 atomic accumulate)
            if (g.c_f32 && g.accumulate && splitk > 1 && !g.bias && !g.res && !g.res2 && g.act == 0) {
                // the caller allows split-K: pick it from the tile count (~512
                // workgroups, >= 256 k per split) -- atomics cost M*N*splitk*4 B at ~1.3 TB/s
                const long tiles = cdiv(g.M, BM) * cdiv(g.N, BN);
                long sk = (512 + tiles - 1) / tiles;
                sk = std::min<long>(sk, std::max<long>(1, g.K / 256));
                splitk = (int)std::max<long>(1, sk);
                long kc2 = (g.K + splitk - 1) / splitk;
                kc2 = ((kc2 + BK2 - 1) / BK2) * BK2;
                splitk = (int)((g.K + kc2 - 1) / kc2);
                g.kchunk = kc2;
            } else {
                g.kchunk = ((g.kchunk + BK2 - 1) / BK2) * BK2;
                splitk = (int)((g.K + g.kchunk - 1) / g.kchunk);
            }
            if (BM == 128 && BN == 160) launch_v2<128, 160>(g, splitk, st);
            else if (BM == 64 && BN == 160) launch_v2<64, 160>(g, splitk, st);
            else if (BM == 128 && BN == 128) launch_v2<128, 128>(g, splitk, st);
            else if (BM == 64 && BN == 128) launch_v2<64, 128>(g, splitk, st);
            else if (BM == 128) launch_v2<128, 64>(g, splitk, st);
            else launch_v2<64, 64>(g, splitk, st);
            return dlcs_launch_status();
        }
    }
    if constexpr (std::is_same<T, float>::value) {
        static const bool off = [] { const char* e = dlcs_knob("DLCS_GEMM_F32_GENERIC"); return e && e[0] == '1'; }();
        if (!off && gemm_f32_fast(g, splitk, st)) return dlcs_launch_status();
    }
    if (g.N % 160 == 0 && g.N <= 640) launch<T, 4, 1, 1, 5>(g, splitk, st);      // 128 x 160
    else if (g.M <= 64 || g.N <= 64) launch<T, 2, 2, 1, 1>(g, splitk, st);       // 64 x 64
    else launch<T, 2, 2, 2, 2>(g, splitk, st);                                     // 128 x 128
    return dlcs_launch_status();
}

// ---------------------------------------------------------------- grouped weight gradients (bf16)
// dW_g[m, n] += sum_t A_g[t, m] B_g[t, n] and db_g[m] += sum_t A_g[t, m] for up to
// four (A_g, B_g) pairs of one backward phase in ONE launch -- the four nn.Linear
// weight gradients of a Swin block (vst:27-29, :131, :133) or the k4s4 patch
// embed / unembed (vst:455, :503).  The reduction over T = 13,440 tokens is split
// into S token ranges; each workgroup writes its fp32 160 x 160 partial tile with
// plain 16-B stores and a second kernel sums the S partials (split-K through fp32
// atomics would move S x |dW| x 4 B at the chip's ~1.3 TB/s atomic rate, 5-15 x
// the operand bytes here).  The bias gradient rides on the A operand: waves of
// the first column half also multiply their A fragments by an all-ones B
// fragment, which leaves the row sums in every column of an extra 16 x 16 tile.
// Tile: 160 (m) x 160 (n), 10 waves = 5 m-slabs of 32 x 2 n-halves of 80,
// v_mfma_f32_16x16x32_bf16; both operands are token-major, staged per 64-token
// step as [64][160] images by global->LDS DMA (saddr form, XOR swizzle of the
// 16-column tiles by bit 3 of the token applied on the source side) into a
// 2-slot ring, read k-contiguous with ds_read_b64_tr_b16.
constexpr int kDwT = 160;                       // tile edge
constexpr int kDwBK = 64;                       // tokens per step
constexpr int kDwImg = kDwBK * kDwT;            // bf16 per operand image (20 KB)
constexpr int kDwMaxG = 4;

struct DwGroup {
    const bf16* A; const bf16* B;
    long lda, ldb;
    int M, N, tiles_n, tile0;
    float* part;                                // [S][M][N] fp32 partials
    float* bpart;                               // [S][M] bias partials, or null
};
struct DwArgs {
    DwGroup g[kDwMaxG];
    int ng, S, steps_total, total_tiles;
};

// the same DMA as conv3d.hip's glds16_s: uniform 64-bit base in SGPRs + per-lane
// 32-bit byte offset; m0 saved and restored (the compiler may keep a value in it)
DLCS_DEV void dw_glds16(const void* sbase, unsigned voff, unsigned lds_addr) {
    unsigned saved;
    const unsigned long long sb = (unsigned long long)(uintptr_t)sbase;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)sb);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(sb >> 32));
    const unsigned long long sbu = ((unsigned long long)hi << 32) | lo;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 4\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(saved) : "v"(voff), "s"(sbu), "s"(__builtin_amdgcn_readfirstlane(lds_addr)) : "memory");
}

__global__ void __launch_bounds__(640) gemm_dw_grouped_kernel(DwArgs a) {
    __shared__ __attribute__((aligned(16))) bf16 smem_dw[2 * 2 * kDwImg];     // 2 slots x (A, B) = 80 KB
    const int tile = blockIdx.x % a.total_tiles, split = blockIdx.x / a.total_tiles;
    int gi = 0;
#pragma unroll
    for (int i = 1; i < kDwMaxG; ++i)
        if (i < a.ng && tile >= a.g[i].tile0) gi = i;
    const DwGroup& G = a.g[gi];
    const int lt = tile - G.tile0;
    const int m0 = (lt / G.tiles_n) * kDwT, n0 = (lt % G.tiles_n) * kDwT;
    const int s0 = (int)((long)a.steps_total * split / a.S), s1 = (int)((long)a.steps_total * (split + 1) / a.S);
    const int nsteps = s1 - s0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave % 5, wn = wave / 5;

    // DMA pieces of a step: 40 x 1 KB, piece wave + 10 k (k < 4); pieces 0-19 fill
    // the A image, 20-39 the B image.  LDS chunk p of an image = token row p / 20,
    // 16-B slot p % 20 holding logical 8-column chunk slot ^ 2 (bit 3 of the row).
    unsigned voff[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int pi = k * 10 + wave;
        const int p = (pi % 20) * 64 + lane;
        const int kr = p / 20, c = p % 20;
        const int lc = c ^ (((kr >> 3) & 1) << 1);
        const long ld = pi < 20 ? G.lda : G.ldb;
        voff[k] = (unsigned)((kr * ld + lc * 8) * 2);
    }
    const unsigned base_lds = (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)smem_dw);
    auto issue = [&](int step, int slot) {
        const long t0 = (long)(s0 + step) * kDwBK;
        const bf16* srcA = G.A + t0 * G.lda + m0;
        const bf16* srcB = G.B + t0 * G.ldb + n0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int pi = k * 10 + wave;
            const unsigned dst = base_lds + (unsigned)((slot * 2 * kDwImg) * 2) + (unsigned)(pi * 1024);
            dw_glds16(pi < 20 ? (const void*)srcA : (const void*)srcB, voff[k], dst);
        }
    };

    f32x4_t acc[2][5], accb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        accb[i] = (f32x4_t)0.0f;
#pragma unroll
        for (int j = 0; j < 5; ++j) acc[i][j] = (f32x4_t)0.0f;
    }
    bf16x8_t ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.0f;
    using Img = Stage2<kDwT, 1>;
    static_assert(Img::LD == kDwT, "lane-linear DMA image needs unpadded rows");
    Img im;

    if (nsteps > 0) issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int st = 0; st < nsteps; ++st) {
        const int slot = st & 1;
        if (st + 1 < nsteps) issue(st + 1, slot ^ 1);
        const bf16* As = smem_dw + slot * 2 * kDwImg;
        const bf16* Bs = As + kDwImg;
#pragma unroll
        for (int ks = 0; ks < kDwBK / 32; ++ks) {
            bf16x8_t af[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) af[i] = im.frag(As, wm * 32 + 16 * i, ks, lane);
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const bf16x8_t bfr = im.frag(Bs, wn * 80 + 16 * j, ks, lane);
#pragma unroll
                for (int i = 0; i < 2; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
            }
            if (wn == 0) {
#pragma unroll
                for (int i = 0; i < 2; ++i) accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], ones, accb[i], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    // partials [S][M][N] in dW's own layout: C/D rows m (4 per lane) x col n;
    // each store instruction writes 4 rows x 64 contiguous bytes
    float* part = G.part + (long)split * G.M * G.N;
    const int mq = (lane >> 4) * 4, nl = lane & 15;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int m = m0 + wm * 32 + 16 * i + mq, n = n0 + wn * 80 + 16 * j + nl;
#pragma unroll
            for (int r = 0; r < 4; ++r) part[(long)(m + r) * G.N + n] = acc[i][j][r];
        }
    if (G.bpart && wn == 0 && n0 == 0 && nl == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
            *reinterpret_cast<f32x4_t*>(G.bpart + (long)split * G.M + m0 + wm * 32 + 16 * i + mq) = accb[i];
    }
}

#ifdef DLCS_DIAG_BUILD
// (DIAG build) the f32-MFMA and bf16 3-plane (x6) grouped weight gradients, superseded
// by gemm_dw_h3.inc
// fp32 build of the grouped weight gradients: the same tiles, splits, partial
// slabs and reduce kernel; a step is 32 tokens (the [32][160] fp32 images are
// the bf16 [64][160] images' 20 KB, so the 40-piece DMA is unchanged), the
// operands are read as single floats (v_mfma_f32_16x16x4_f32: lane (m, q) takes
// k = 4 q + e in the e-th of four MFMAs) and the 16-column blocks of token row
// k sit XOR-swizzled by bit 2 of k, so the two k rows a 32-lane half reads land
// on opposite 16-bank halves (ds_read_b32 banks are mod 32).
constexpr int kDwBKf = 32;

__global__ void __launch_bounds__(640) gemm_dw_grouped_f32_kernel(DwArgs a) {
    __shared__ __attribute__((aligned(16))) float smem_dwf[2 * 2 * kDwBKf * kDwT];   // 2 slots x (A, B) = 80 KB
    const int tile = blockIdx.x % a.total_tiles, split = blockIdx.x / a.total_tiles;
    int gi = 0;
#pragma unroll
    for (int i = 1; i < kDwMaxG; ++i)
        if (i < a.ng && tile >= a.g[i].tile0) gi = i;
    const DwGroup& G = a.g[gi];
    const float* GA = reinterpret_cast<const float*>(G.A);
    const float* GB = reinterpret_cast<const float*>(G.B);
    const int lt = tile - G.tile0;
    const int m0 = (lt / G.tiles_n) * kDwT, n0 = (lt % G.tiles_n) * kDwT;
    const int steps = a.steps_total * (kDwBK / kDwBKf);
    const int s0 = (int)((long)steps * split / a.S), s1 = (int)((long)steps * (split + 1) / a.S);
    const int nsteps = s1 - s0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave % 5, wn = wave / 5;
    constexpr int IMG = kDwBKf * kDwT;            // floats per image

    // DMA pieces of a step: 40 x 1 KB (0-19 the A image, 20-39 B); LDS chunk p of
    // an image = token row p / 40, 16-B slot p % 40 holding logical chunk slot ^ 4 (bit 2 of the row)
    unsigned voff[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int pi = k * 10 + wave;
        const int p = (pi % 20) * 64 + lane;
        const int kr = p / 40, c = p % 40;
        const int lc = c ^ (((kr >> 2) & 1) << 2);
        const long ld = pi < 20 ? G.lda : G.ldb;
        voff[k] = (unsigned)((kr * ld + lc * 4) * 4);
    }
    const unsigned base_lds = (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)smem_dwf);
    auto issue = [&](int step, int slot) {
        const long t0 = (long)(s0 + step) * kDwBKf;
        const float* srcA = GA + t0 * G.lda + m0;
        const float* srcB = GB + t0 * G.ldb + n0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int pi = k * 10 + wave;
            const unsigned dst = base_lds + (unsigned)((slot * 2 * IMG) * 4) + (unsigned)(pi * 1024);
            dw_glds16(pi < 20 ? (const void*)srcA : (const void*)srcB, voff[k], dst);
        }
    };

    f32x4_t acc[2][5], accb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        accb[i] = (f32x4_t)0.0f;
#pragma unroll
        for (int j = 0; j < 5; ++j) acc[i][j] = (f32x4_t)0.0f;
    }
    const int q = lane >> 4, ml = lane & 15;
    // physical float of (token row k, column c): row k * 160 + (c ^ 16 (k >> 2 & 1))
    auto col = [&](int c, int k) { return c ^ (((k >> 2) & 1) << 4); };

    if (nsteps > 0) issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int st = 0; st < nsteps; ++st) {
        const int slot = st & 1;
        if (st + 1 < nsteps) issue(st + 1, slot ^ 1);
        const float* As = smem_dwf + slot * 2 * IMG;
        const float* Bs = As + IMG;
#pragma unroll
        for (int kb = 0; kb < kDwBKf; kb += 16) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = kb + 4 * q + e;                    // this lane's token row in the MFMA
                float af[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) af[i] = As[k * kDwT + col(wm * 32 + 16 * i + ml, k)];
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const float bv = Bs[k * kDwT + col(wn * 80 + 16 * j + ml, k)];
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bv, acc[i][j], 0, 0, 0);
                }
                if (wn == 0) {
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        accb[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], 1.0f, accb[i], 0, 0, 0);
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    float* part = G.part + (long)split * G.M * G.N;
    const int mq = q * 4;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int m = m0 + wm * 32 + 16 * i + mq, n = n0 + wn * 80 + 16 * j + ml;
#pragma unroll
            for (int r = 0; r < 4; ++r) part[(long)(m + r) * G.N + n] = acc[i][j][r];
        }
    if (G.bpart && wn == 0 && n0 == 0 && ml == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
            *reinterpret_cast<f32x4_t*>(G.bpart + (long)split * G.M + m0 + wm * 32 + 16 * i + mq) = accb[i];
    }
}

// fp32 grouped weight gradients on bf16 matrix cores (x6): every fp32 operand
// element is split x = h + m + l into three bf16 planes (h = bf16(x), m =
// bf16(x - h), l = bf16(x - h - m); both differences exact in fp32) and dW takes
// the six plane products >= 2^-16 of the leading term (l h, h l, m m, m h, h m,
// h h), exact in the fp32 accumulator -- fp32 accuracy (the dropped m l, l m,
// l l are below 2^-24 of |a b|) with no scale at all, since bf16 keeps fp32's
// exponent range (gradients of any magnitude split losslessly; the f16 2-plane
// split of the convs needs a per-tensor scale for that).  Same tiles, token
// splits, partial slabs and reduce kernel as the bf16 / fp32 builds; a step is
// 32 tokens (one K = 32 v_mfma_f32_16x16x32_bf16).  Thread t converts column
// t % 160, tokens 8 (t / 160) .. + 7 of both operands: eight coalesced fp32
// row loads held in registers one step ahead, split, and stored k-contiguous
// into [plane][160 columns][32 tokens] images (16-B token groups XOR-swizzled
// by bits 2-3 of the column: conflict-free stores and fragment reads).
constexpr int kDwX6K = 32;                       // tokens per step
constexpr int kDwX6Img = 3 * kDwT * kDwX6K;      // bf16 per operand image [3][160][32] (30 KB)

__global__ void __launch_bounds__(640) gemm_dw_grouped_x6_kernel(DwArgs a) {
    __shared__ __attribute__((aligned(16))) bf16 smem_dwx6[2 * kDwX6Img];    // A, B images: 60 KB
    const int tile = blockIdx.x % a.total_tiles, split = blockIdx.x / a.total_tiles;
    int gi = 0;
#pragma unroll
    for (int i = 1; i < kDwMaxG; ++i)
        if (i < a.ng && tile >= a.g[i].tile0) gi = i;
    const DwGroup& G = a.g[gi];
    const int lt = tile - G.tile0;
    const int m0 = (lt / G.tiles_n) * kDwT, n0 = (lt % G.tiles_n) * kDwT;
    const int steps = a.steps_total * (kDwBK / kDwX6K);
    const int s0 = (int)((long)steps * split / a.S), s1 = (int)((long)steps * (split + 1) / a.S);
    const int nsteps = s1 - s0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave % 5, wn = wave / 5;
    // converter role
    const int cc = threadIdx.x % kDwT, kg = threadIdx.x / kDwT;
    // edge tiles (M or N not a multiple of 160): columns past the edge load from the
    // last column (an unconditional load) and are zeroed when split (not right after
    // the load: a select there would wait for the prefetch)
    const bool aok = m0 + cc < G.M, bok = n0 + cc < G.N;
    const float* GA = reinterpret_cast<const float*>(G.A) + min(m0 + cc, G.M - 1);
    const float* GB = reinterpret_cast<const float*>(G.B) + min(n0 + cc, G.N - 1);
    float ra[8], rb[8];
    auto load = [&](int step) {
        const long t0 = (long)(s0 + step) * kDwX6K + 8 * kg;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            ra[e] = GA[(t0 + e) * G.lda];
            rb[e] = GB[(t0 + e) * G.ldb];
        }
    };
    const int cslot = (cc * kDwX6K + ((kg ^ ((cc >> 2) & 3)) << 3));
    auto convert = [&](const float (&r)[8], bf16* img, bool ok) {
        bf16x8_t h, m, l;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float x = ok ? r[e] : 0.0f;
            const bf16 hv = (bf16)x;
            const float r1 = x - (float)hv;
            const bf16 mv = (bf16)r1;
            const float r2 = r1 - (float)mv;
            h[e] = hv; m[e] = mv; l[e] = (bf16)r2;
        }
        *reinterpret_cast<bf16x8_t*>(img + cslot) = h;
        *reinterpret_cast<bf16x8_t*>(img + kDwT * kDwX6K + cslot) = m;
        *reinterpret_cast<bf16x8_t*>(img + 2 * kDwT * kDwX6K + cslot) = l;
    };
    // fragment of column c, plane p: tokens 8 (lane >> 4) .. + 7
    const int kq = lane >> 4, ml = lane & 15;
    auto frag = [&](const bf16* img, int c, int p) {
        return *reinterpret_cast<const bf16x8_t*>(img + p * kDwT * kDwX6K + c * kDwX6K + ((kq ^ ((c >> 2) & 3)) << 3));
    };

    f32x4_t acc[2][5], accb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        accb[i] = (f32x4_t)0.0f;
#pragma unroll
        for (int j = 0; j < 5; ++j) acc[i][j] = (f32x4_t)0.0f;
    }
    bf16x8_t ones;                                   // the bias gradient rides on an all-ones B fragment
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.0f;
    bf16* As = smem_dwx6;
    bf16* Bs = smem_dwx6 + kDwX6Img;
    if (nsteps > 0) load(0);
    for (int st = 0; st < nsteps; ++st) {
        __syncthreads();                             // the previous step's fragment reads are done
        convert(ra, As, aok);
        convert(rb, Bs, bok);
        __syncthreads();
        if (st + 1 < nsteps) load(st + 1);           // in flight during this step's products
        bf16x8_t af[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int p = 0; p < 3; ++p) af[i][p] = frag(As, wm * 32 + 16 * i + ml, p);
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            bf16x8_t bfr[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) bfr[p] = frag(Bs, wn * 80 + 16 * j + ml, p);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                // the step's six products into a fresh tile, added to the running sum by the
                // VALU (the matrix core's accumulate drifts in a long running sum:
                // tools/mfma_round.py, conv3d_f16x3.inc FOLD)
                f32x4_t c = (f32x4_t)0.0f;
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][2], bfr[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bfr[2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][1], bfr[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][1], bfr[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bfr[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bfr[0], c, 0, 0, 0);
                acc[i][j] += c;
            }
        }
        if (wn == 0) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                f32x4_t c = (f32x4_t)0.0f;
#pragma unroll
                for (int p = 2; p >= 0; --p) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][p], ones, c, 0, 0, 0);
                accb[i] += c;
            }
        }
    }
    float* part = G.part + (long)split * G.M * G.N;
    const int mq = kq * 4;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int m = m0 + wm * 32 + 16 * i + mq, n = n0 + wn * 80 + 16 * j + ml;
            if (m < G.M && n < G.N) {                    // M % 16 == 0: the row quad is whole
#pragma unroll
                for (int r = 0; r < 4; ++r) part[(long)(m + r) * G.N + n] = acc[i][j][r];
            }
        }
    if (G.bpart && wn == 0 && n0 == 0 && ml == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
            if (m0 + wm * 32 + 16 * i + mq < G.M)
                *reinterpret_cast<f32x4_t*>(G.bpart + (long)split * G.M + m0 + wm * 32 + 16 * i + mq) = accb[i];
    }
}
#endif  // DLCS_DIAG_BUILD

#include "gemm_dw_h3.inc"

// DLCS_DW_F32=1: the fp32 grouped weight gradients on the f32 MFMA; DLCS_DW_X6=1: on
// the bf16 3-plane split (A/B timing, DLCS_DIAG=1)
static bool dw_f32_mfma() {
    static const bool v = [] { const char* e = dlcs_knob("DLCS_DW_F32"); return e && e[0] == '1'; }();
    return v;
}
static bool dw_x6() {
    static const bool v = [] { const char* e = dlcs_knob("DLCS_DW_X6"); return e && e[0] == '1'; }();
    return v;
}

struct DwOut {
    float* dW[kDwMaxG]; float* db[kDwMaxG];
    const float* part[kDwMaxG]; const float* bpart[kDwMaxG];
    int M[kDwMaxG], N[kDwMaxG], bper[kDwMaxG];
    int S;
};

// dW[m][n] += sum_s part[s][m][n]; db[c] += sum_s sum_{m = c mod period} bpart[s][m].
// Workgroup = 64 float4 quads (or 64 bias columns) x 4 waves: wave p sums the
// partials s = p, p + 4, ... with every load in flight (two accumulators), then
// the four wave sums combine through LDS in a fixed order -- run-to-run
// deterministic, and one memory round trip instead of a chain of S / 4 (a
// Swin block's four Linears have S ~ 21 token ranges; the unembed bias folds
// 4 x 64 terms per column).  16-B loads and read-modify-write of dW.
__global__ void __launch_bounds__(256) gemm_dw_reduce_kernel(DwOut o) {
    __shared__ f32x4_t red[4][64];
    const int g = blockIdx.y;
    const int M = o.M[g], N = o.N[g];
    const long nq = (long)M * N / 4;
    const int l = threadIdx.x & 63, p = threadIdx.x >> 6;
    const long sstr = (long)M * N;
    for (long q0 = blockIdx.x * 64L; q0 < nq; q0 += (long)gridDim.x * 64) {
        const long q = q0 + l;
        f32x4_t s0 = (f32x4_t)0.0f, s1 = (f32x4_t)0.0f;
        if (q < nq) {
            const float* pp = o.part[g] + q * 4;
            int k = p;
            for (; k + 4 < o.S; k += 8) {
                s0 += *reinterpret_cast<const f32x4_t*>(pp + k * sstr);
                s1 += *reinterpret_cast<const f32x4_t*>(pp + (k + 4) * sstr);
            }
            if (k < o.S) s0 += *reinterpret_cast<const f32x4_t*>(pp + k * sstr);
        }
        red[p][l] = s0 + s1;
        __syncthreads();
        if (p == 0 && q < nq) {
            const f32x4_t t = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
            float* d = o.dW[g] + q * 4;
            if (((uintptr_t)o.dW[g] & 15) == 0) {
                *reinterpret_cast<f32x4_t*>(d) += t;
            } else {                                // dW may be a view at any float offset of a gradient bucket
#pragma unroll
                for (int e = 0; e < 4; ++e) d[e] += t[e];
            }
        }
        __syncthreads();
    }
    if (o.db[g]) {
        const int P = o.bper[g], per = M / P, nterm = o.S * per;
        float* redf = reinterpret_cast<float*>(red);
        for (int c0 = blockIdx.x * 64; c0 < P; c0 += gridDim.x * 64) {
            const int c = c0 + l;
            float b0 = 0.0f, b1 = 0.0f;
            if (c < P) {
                // term t = (s, r): bpart[s][c + r P]; wave p takes t = p, p + 4, ...
                int t = p;
                for (; t + 4 < nterm; t += 8) {
                    b0 += o.bpart[g][(long)(t / per) * M + c + (long)(t % per) * P];
                    b1 += o.bpart[g][(long)((t + 4) / per) * M + c + (long)((t + 4) % per) * P];
                }
                if (t < nterm) b0 += o.bpart[g][(long)(t / per) * M + c + (long)(t % per) * P];
            }
            redf[p * 64 + l] = b0 + b1;
            __syncthreads();
            if (p == 0 && c < P) o.db[g][c] += (redf[l] + redf[64 + l]) + (redf[128 + l] + redf[192 + l]);
            __syncthreads();
        }
    }
}

static void dw_reduce_launch(const DwOut& o, int ngroups, long maxq, long maxp, hipStream_t st) {
    const long blocks = std::max<long>(cdiv(maxq, 64), cdiv(maxp, 64));
    hipLaunchKernelGGL(gemm_dw_reduce_kernel, dim3((unsigned)std::min<long>(2048, blocks), (unsigned)ngroups), dim3(256), 0,
                       st, o);
}

#ifdef DLCS_DIAG_BUILD
#include "gemm_nt_x6.inc"                                // superseded bf16 3-plane NT GEMM (DIAG build)
#endif

}  // namespace

extern "C" int dlcs_gemm(int dtype, int64_t M, int64_t N, int64_t K,
                         const void* A, int64_t lda, int a_trans,
                         const void* B, int64_t ldb, int b_trans,
                         void* C, int64_t ldc, int c_dtype,
                         const float* bias, int act, const void* aux, void* aux_out, int64_t ldaux, float alpha,
                         const void* residual, int64_t ldr, int r_dtype, float res_scale,
                         const void* residual2, int64_t ldr2, int r2_dtype, float res2_scale,
                         const int32_t* row_map, int accumulate, int splitk,
                         dlcs_stream_t stream) {
    DLCS_CHECK_ARG(A && B && C && M > 0 && N > 0 && K > 0);
    DLCS_CHECK_ARG(dtype == DLCS_F32 || dtype == DLCS_BF16);
    DLCS_CHECK_ARG(act >= 0 && act <= 7 && ((act != 2 && act != 5 && act != 6) || aux));
    GemmArgs g{};
    g.A = A; g.B = B; g.C = C; g.bias = bias; g.aux = aux; g.aux_out = aux_out; g.res = residual; g.res2 = residual2;
    g.row_map = row_map;
    g.alpha = alpha; g.res_scale = res_scale; g.res2_scale = res2_scale;
    g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldaux = ldaux; g.ldr = ldr; g.ldr2 = ldr2;
    g.a_trans = a_trans; g.b_trans = b_trans; g.act = act;
    g.c_f32 = (c_dtype == DLCS_F32); g.r_f32 = (r_dtype == DLCS_F32); g.r2_f32 = (r2_dtype == DLCS_F32);
    g.accumulate = accumulate;
    hipStream_t st = (hipStream_t)stream;
    return dtype == DLCS_F32 ? gemm_dispatch<float>(g, splitk, st) : gemm_dispatch<bf16>(g, splitk, st);
}

static int dw_splits(int total_tiles, int steps_total) {
    // ~DLCS_DW_WG workgroups (default 256: one per CU), at least 4 token steps per range
    static const int target = [] { const char* e = dlcs_knob("DLCS_DW_WG"); return e && atoi(e) > 0 ? atoi(e) : 256; }();
    int S = (target + total_tiles / 2) / total_tiles;
    S = std::max(1, std::min(S, steps_total / 4));
    return std::max(1, S);
}

extern "C" size_t dlcs_gemm_dw_workspace_bytes(int ngroups, const int64_t* M, const int64_t* N, int64_t T) {
    if (ngroups < 1 || ngroups > kDwMaxG || T % kDwBK) return 0;
    int tiles = 0;
    for (int g = 0; g < ngroups; ++g) tiles += (int)(cdiv(M[g], kDwT) * cdiv(N[g], kDwT));
    const int S = dw_splits(tiles, (int)(T / kDwBK));
    size_t b = 0;
    for (int g = 0; g < ngroups; ++g) b += (size_t)S * (size_t)(M[g] * N[g] + M[g]) * sizeof(float);
    return b;
}

static int dw_grouped_impl(int f32, int ngroups, const void* const* A, const int64_t* lda, const void* const* B,
                           const int64_t* ldb, const int64_t* M, const int64_t* N, float* const* dW,
                           float* const* db, const int64_t* db_period, int64_t T, void* workspace,
                           size_t workspace_bytes, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(ngroups >= 1 && ngroups <= kDwMaxG && A && B && lda && ldb && M && N && dW && T > 0);
    if (T % kDwBK) return DLCS_ERR_UNSUPPORTED_SIZE;
    if (!workspace || workspace_bytes < dlcs_gemm_dw_workspace_bytes(ngroups, M, N, T)) return DLCS_ERR_WORKSPACE;
    DwArgs a{};
    DwOut o{};
    a.ng = ngroups;
    int tiles = 0;
    for (int g = 0; g < ngroups; ++g) {
        DLCS_CHECK_ARG(A[g] && B[g] && dW[g] && M[g] > 0 && N[g] > 0);
        // the fp32 h3 / x6 kernels take edge tiles (M, N multiples of 16); the others whole 160 tiles
        const bool edge_ok = f32 && !dw_f32_mfma();
        if ((edge_ok ? (M[g] % 16 || N[g] % 16) : (M[g] % kDwT || N[g] % kDwT)) || lda[g] % 8 || ldb[g] % 8 ||
            lda[g] < M[g] || ldb[g] < N[g] ||
            ((uintptr_t)A[g] & 15) || ((uintptr_t)B[g] & 15) || (long)kDwBK * lda[g] * 4 > (1L << 31) ||
            (long)kDwBK * ldb[g] * 4 > (1L << 31))
            return DLCS_ERR_UNSUPPORTED_SIZE;
        const int P = (db && db[g]) ? (int)(db_period && db_period[g] > 0 ? db_period[g] : M[g]) : 0;
        if (P && M[g] % P) return DLCS_ERR_INVALID_ARG;
        tiles += (int)(cdiv(M[g], kDwT) * cdiv(N[g], kDwT));
    }
    a.total_tiles = tiles;
    a.steps_total = (int)(T / kDwBK);
    a.S = dw_splits(tiles, a.steps_total);
    o.S = a.S;
    char* ws = reinterpret_cast<char*>(workspace);
    int t0 = 0;
    for (int g = 0; g < ngroups; ++g) {
        DwGroup& G = a.g[g];
        G.A = reinterpret_cast<const bf16*>(A[g]); G.B = reinterpret_cast<const bf16*>(B[g]);
        G.lda = lda[g]; G.ldb = ldb[g]; G.M = (int)M[g]; G.N = (int)N[g];
        G.tiles_n = (int)cdiv(G.N, kDwT); G.tile0 = t0;
        t0 += (int)cdiv(G.M, kDwT) * G.tiles_n;
        G.part = reinterpret_cast<float*>(ws);
        ws += (size_t)a.S * G.M * G.N * sizeof(float);
        const bool hasb = db && db[g];
        G.bpart = hasb ? reinterpret_cast<float*>(ws) : nullptr;
        ws += (size_t)a.S * G.M * sizeof(float);
        o.dW[g] = dW[g]; o.db[g] = hasb ? db[g] : nullptr;
        o.part[g] = G.part; o.bpart[g] = G.bpart;
        o.M[g] = G.M; o.N[g] = G.N;
        o.bper[g] = hasb ? (int)(db_period && db_period[g] > 0 ? db_period[g] : M[g]) : 0;
    }
    hipStream_t st = (hipStream_t)stream;
#ifdef DLCS_DIAG_BUILD
    if (f32 && dw_f32_mfma()) hipLaunchKernelGGL(gemm_dw_grouped_f32_kernel, dim3((unsigned)(tiles * a.S)), dim3(640), 0, st, a);
    else if (f32 && dw_x6()) hipLaunchKernelGGL(gemm_dw_grouped_x6_kernel, dim3((unsigned)(tiles * a.S)), dim3(640), 0, st, a);
    else
#endif
    if (f32) hipLaunchKernelGGL(gemm_dw_grouped_h3_kernel, dim3((unsigned)(tiles * a.S)), dim3(640), 0, st, a);
    else hipLaunchKernelGGL(gemm_dw_grouped_kernel, dim3((unsigned)(tiles * a.S)), dim3(640), 0, st, a);
    long maxq = 0, maxp = 0;
    for (int g = 0; g < ngroups; ++g) {
        maxq = std::max<long>(maxq, (long)M[g] * N[g] / 4);
        maxp = std::max<long>(maxp, o.bper[g]);
    }
    dw_reduce_launch(o, ngroups, maxq, maxp, st);
    return dlcs_launch_status();
}

// C[m, n] += sum_k A[m, k] B[n, k] (fp32, both K-contiguous), split over K into
// S <= 4 ranges whose raw partials land in `workspace` and are summed by
// gemm_dw_reduce_kernel in a fixed order: split-K occupancy with a run-to-run
// deterministic result (the patch embed forward, vst:472: 13440 x 160 x 10240
// -- 210 row tiles alone leave most CUs idle).
extern "C" size_t dlcs_gemm_f32_splitk_det_workspace_bytes(int64_t M, int64_t N) {
    return (size_t)4 * (size_t)M * (size_t)N * sizeof(float);
}

extern "C" int dlcs_gemm_f32_splitk_det(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int64_t N,
                                        int64_t K, float* C, void* workspace, size_t workspace_bytes,
                                        dlcs_stream_t stream) {
    DLCS_CHECK_ARG(A && B && C && M > 0 && N > 0 && K > 0);
    if (!workspace || workspace_bytes < dlcs_gemm_f32_splitk_det_workspace_bytes(M, N)) return DLCS_ERR_WORKSPACE;
    auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (!al(A) || !al(B) || !al(C) || !al(workspace) || lda % 4 || ldb % 4 || K % 4 || N % 160 || M * N % 4)
        return DLCS_ERR_UNSUPPORTED_SIZE;
    GemmArgs g{};
    g.A = A; g.B = B; g.C = C; g.alpha = 1.0f; g.res_scale = 1.0f; g.res2_scale = 1.0f;
    g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = N;
    g.c_f32 = 1; g.r_f32 = 1; g.r2_f32 = 1;
    g.part = reinterpret_cast<float*>(workspace);
    long kc = (K + 3) / 4;
    kc = ((kc + kGfBK - 1) / kGfBK) * kGfBK;
    g.kchunk = kc;
    const int S = (int)((K + kc - 1) / kc);
    hipStream_t st = (hipStream_t)stream;
    gemm_f32_launch_bm<64>(g, S, st);
    DwOut o{};
    o.dW[0] = C; o.part[0] = g.part; o.M[0] = (int)M; o.N[0] = (int)N; o.S = S;
    dw_reduce_launch(o, 1, M * N / 4, 0, st);
    return dlcs_launch_status();
}

#ifdef DLCS_DIAG_BUILD
// C[m, n] += sum_k A[m, k] B[n, k] (fp32, both K-contiguous) on bf16 matrix
// cores with the 3-plane split (gemm_nt_x6.inc): B's planes, then S <= 4 raw
// K-range partial slabs, live in `workspace`; the slabs are summed in a fixed
// order (run-to-run deterministic).  N % 160 == 0, K % 32 == 0, 16-B aligned
// operands with lda, ldb % 4 == 0; any M.
static size_t nt_x6_bplanes_bytes(int64_t N, int64_t K) { return ((size_t)3 * N * K * sizeof(bf16) + 255) & ~(size_t)255; }

static int nt_x6_splits(long tiles, long steps) {
    static const int env = [] { const char* e = dlcs_knob("DLCS_NT_X6_S"); return e ? atoi(e) : 0; }();
    int S = env > 0 ? env : (int)(256 / tiles);          // one workgroup per CU (156 KB of LDS), one round
    S = std::max(1, std::min<int>(S, 4));
    while (S > 1 && steps / S < 8) --S;
    return S;
}

extern "C" size_t dlcs_gemm_nt_x6_workspace_bytes(int64_t M, int64_t N, int64_t K) {
    if (M <= 0 || N <= 0 || K <= 0) return 0;
    return nt_x6_bplanes_bytes(N, K) + (size_t)4 * (size_t)M * (size_t)N * sizeof(float);
}

extern "C" int dlcs_gemm_nt_x6(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int64_t N, int64_t K,
                               float* C, void* workspace, size_t workspace_bytes, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(A && B && C && M > 0 && N > 0 && K > 0);
    if (!workspace || workspace_bytes < dlcs_gemm_nt_x6_workspace_bytes(M, N, K)) return DLCS_ERR_WORKSPACE;
    auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (!al(A) || !al(B) || !al(C) || !al(workspace) || lda % 4 || ldb % 4 || lda < K || ldb < K || K % kNtK ||
        N % kNtN || M > (1L << 30) || N * K > (1L << 30))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    hipStream_t st = (hipStream_t)stream;
    bf16* bp = reinterpret_cast<bf16*>(workspace);
    const long nq = N * K / 4;
    hipLaunchKernelGGL(split3_rows_kernel, dim3((unsigned)std::min<long>(1024, cdiv(nq, 256))), dim3(256), 0, st, B, (long)N,
                       (int)K, (long)ldb, bp);
    NtX6Args g{};
    g.a = A; g.lda = lda; g.bp = bp;
    g.part = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + nt_x6_bplanes_bytes(N, K));
    g.M = (int)M; g.N = (int)N; g.K = (int)K;
    g.mtiles = (int)cdiv(M, kNtM);
    const long ntiles = N / kNtN;
    g.S = nt_x6_splits((long)g.mtiles * ntiles, K / kNtK);
    (void)hipFuncSetAttribute((const void*)gemm_nt_x6_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kNtSmem);
    hipLaunchKernelGGL(gemm_nt_x6_kernel, dim3((unsigned)(g.mtiles * g.S), (unsigned)ntiles), dim3(512), kNtSmem, st, g);
    DwOut o{};
    o.dW[0] = C; o.part[0] = g.part; o.M[0] = (int)M; o.N[0] = (int)N; o.S = g.S;
    dw_reduce_launch(o, 1, M * N / 4, 0, st);
    return dlcs_launch_status();
}
#endif  // DLCS_DIAG_BUILD

extern "C" int dlcs_gemm_dw_grouped(int ngroups, const void* const* A, const int64_t* lda, const void* const* B,
                                    const int64_t* ldb, const int64_t* M, const int64_t* N, float* const* dW,
                                    float* const* db, const int64_t* db_period, int64_t T, void* workspace,
                                    size_t workspace_bytes, dlcs_stream_t stream) {
    return dw_grouped_impl(0, ngroups, A, lda, B, ldb, M, N, dW, db, db_period, T, workspace, workspace_bytes, stream);
}

extern "C" int dlcs_gemm_dw_grouped_f32(int ngroups, const void* const* A, const int64_t* lda, const void* const* B,
                                        const int64_t* ldb, const int64_t* M, const int64_t* N, float* const* dW,
                                        float* const* db, const int64_t* db_period, int64_t T, void* workspace,
                                        size_t workspace_bytes, dlcs_stream_t stream) {
    return dw_grouped_impl(1, ngroups, A, lda, B, ldb, M, N, dW, db, db_period, T, workspace, workspace_bytes, stream);
}
