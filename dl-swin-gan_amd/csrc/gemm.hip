// Generic MFMA GEMM with fused epilogues (gfx950).
//
//   C[m, n] (+)= epi( sum_k A(m, k) * B(n, k) )
//   A(m, k) = a_trans ? A[k*lda + m] : A[m*lda + k]
//   B(n, k) = b_trans ? B[k*ldb + n] : B[n*ldb + k]      (b_trans = 0: nn.Linear weight layout)
//   epi(v) = alpha * act(v + bias[n]) + residual[row(m), n],  row(m) = row_map ? row_map[m] : m
//   act: 0 none, 1 GELU(erf) (vst:29; pre-activation also written to aux when given),
//        2 GELU backward: v * gelu'(aux[m, n]), 3 ReLU (the next ConvBlock's pre-activation)
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

namespace {

constexpr int BK = 32;

struct GemmArgs {
    const void* A; const void* B; void* C;
    const float* bias; const void* aux; void* aux_out; const void* res; const int32_t* row_map;
    float alpha;
    long M, N, K, lda, ldb, ldc, ldaux, ldr;
    int a_trans, b_trans, act, c_f32, r_f32, accumulate;
    long kchunk;   // K range per blockIdx.z
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
                if (g.act == 1) {
                    if (g.aux_out) reinterpret_cast<T*>(g.aux_out)[m * g.ldaux + n] = from_f<T>(v);
                    v = gelu_erf(v);
                } else if (g.act == 2) {
                    v *= gelu_erf_grad(to_f(reinterpret_cast<const T*>(g.aux)[m * g.ldaux + n]));
                } else if (g.act == 3) {
                    v = fmaxf(v, 0.0f);
                }
                v *= g.alpha;
                if (g.res) v += load_as_f<T>(g.res, orow * g.ldr + n, g.r_f32);
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

template <typename T, int WM, int WN, int TM, int TN>
void launch(const GemmArgs& g, int splitk, hipStream_t st) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    dim3 grid(cdiv(g.M, BM), cdiv(g.N, BN), splitk);
    hipLaunchKernelGGL((gemm_kernel<T, WM, WN, TM, TN>), grid, dim3(WM * WN * 64), 0, st, g);
}

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
    if (g.N % 160 == 0 && g.N <= 640) launch<T, 4, 1, 1, 5>(g, splitk, st);      // 128 x 160
    else if (g.M <= 64 || g.N <= 64) launch<T, 2, 2, 1, 1>(g, splitk, st);       // 64 x 64
    else launch<T, 2, 2, 2, 2>(g, splitk, st);                                     // 128 x 128
    return dlcs_launch_status();
}

}  // namespace

extern "C" int dlcs_gemm(int dtype, int64_t M, int64_t N, int64_t K,
                         const void* A, int64_t lda, int a_trans,
                         const void* B, int64_t ldb, int b_trans,
                         void* C, int64_t ldc, int c_dtype,
                         const float* bias, int act, const void* aux, void* aux_out, int64_t ldaux, float alpha,
                         const void* residual, int64_t ldr, int r_dtype,
                         const int32_t* row_map, int accumulate, int splitk,
                         dlcs_stream_t stream) {
    DLCS_CHECK_ARG(A && B && C && M > 0 && N > 0 && K > 0);
    DLCS_CHECK_ARG(dtype == DLCS_F32 || dtype == DLCS_BF16);
    DLCS_CHECK_ARG(act >= 0 && act <= 3 && (act != 2 || aux));
    GemmArgs g{};
    g.A = A; g.B = B; g.C = C; g.bias = bias; g.aux = aux; g.aux_out = aux_out; g.res = residual; g.row_map = row_map;
    g.alpha = alpha;
    g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldaux = ldaux; g.ldr = ldr;
    g.a_trans = a_trans; g.b_trans = b_trans; g.act = act;
    g.c_f32 = (c_dtype == DLCS_F32); g.r_f32 = (r_dtype == DLCS_F32); g.accumulate = accumulate;
    hipStream_t st = (hipStream_t)stream;
    return dtype == DLCS_F32 ? gemm_dispatch<float>(g, splitk, st) : gemm_dispatch<bf16>(g, splitk, st);
}
