// SENSE forward / adjoint (coil-map multiply, orthonormal uncentered 2D FFT,
// k-space mask) on gfx950.  Replaces tr:49-110 (SenseModel) and tr:12-46 (FFT).
//
// Layout (torch complex64 = interleaved float2, all contiguous):
//   x    [B,E,T,Y,X]     maps [B,E,C,Y,X]     k-space [B,C,T,Y,X]
//   weights f32 [B,Wc,T,Y,X], Wc in {1, C} (broadcast over coils when 1)
//
// The 2D FFT is split into an X-pass ("rows", X contiguous) and a Y-pass
// ("cols", strided by X); each pass runs a mixed-radix (2,3,4,5) Stockham
// autosort FFT on a batch of lines staged in LDS, twiddles from a per-block
// double-precision table.  The coil combine (forward) and the conj-map coil
// reduction + PGD data-consistency epilogue (adjoint) are fused into the row
// pass, the mask and the 1/sqrt(YX) scale into the column pass, so each op is
// two launches and one k-space-sized intermediate (which stays in the 256 MiB
// Infinity Cache between the two launches at the BASELINE size).
#include "dlcs_common.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace {

constexpr int kThreads = 256;
constexpr int kPoints = 4096;            // complex points staged per column block
constexpr int kMaxPts = kPoints / kThreads;
constexpr int kRowPoints = 2048;         // complex points staged per row block
constexpr int kRowPts = kRowPoints / kThreads;
constexpr int kMaxE = 2;                 // max ESPIRiT maps in the fused row pass

struct FftPlan {
    int n, npass;
    int radix[12];
};

static bool make_plan(int n, FftPlan& p) {
    if (n < 1 || n > 1024) return false;
    p.n = n;
    p.npass = 0;
    int m = n;
    const int rs[4] = {4, 2, 3, 5};
    for (int r : rs) {
        while (m % r == 0) { p.radix[p.npass++] = r; m /= r; }
    }
    return m == 1 && p.npass <= 12;
}

DLCS_DEV float2 cmul(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
DLCS_DEV float2 cmulc(float2 a, float2 b) { return make_float2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y); } // a * conj(b)
DLCS_DEV float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
DLCS_DEV float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }

// twiddle table: tw[m] = exp(-2 pi i m / n), m in [0, n), double precision.
DLCS_DEV void build_twiddles(float2* tw, int n) {
    for (int m = threadIdx.x; m < n; m += blockDim.x) {
        double s, c;
        sincospi(-2.0 * (double)m / (double)n, &s, &c);
        tw[m] = make_float2((float)c, (float)s);
    }
}

// in-register R-point DFT; inverse uses conjugate roots.
template <int R>
DLCS_DEV void dft(float2 (&a)[R], bool inv) {
    if constexpr (R == 2) {
        float2 t0 = cadd(a[0], a[1]), t1 = csub(a[0], a[1]);
        a[0] = t0; a[1] = t1;
    } else if constexpr (R == 4) {
        float2 s02 = cadd(a[0], a[2]), d02 = csub(a[0], a[2]);
        float2 s13 = cadd(a[1], a[3]), d13 = csub(a[1], a[3]);
        // forward: multiply d13 by -i ; inverse: by +i
        float2 jd13 = inv ? make_float2(-d13.y, d13.x) : make_float2(d13.y, -d13.x);
        a[0] = cadd(s02, s13);
        a[2] = csub(s02, s13);
        a[1] = cadd(d02, jd13);
        a[3] = csub(d02, jd13);
    } else if constexpr (R == 3) {
        const float c1 = -0.5f, s1 = inv ? 0.86602540378443865f : -0.86602540378443865f;
        float2 t = cadd(a[1], a[2]);
        float2 d = csub(a[1], a[2]);
        float2 b0 = cadd(a[0], t);
        float2 m = make_float2(a[0].x + c1 * t.x, a[0].y + c1 * t.y);
        // s1 * i * d
        float2 r = make_float2(-s1 * d.y, s1 * d.x);
        a[0] = b0;
        a[1] = cadd(m, r);
        a[2] = csub(m, r);
    } else if constexpr (R == 5) {
        const float c1 = 0.30901699437494742f, c2 = -0.80901699437494742f;
        const float s1v = 0.95105651629515357f, s2v = 0.58778525229247313f;
        const float s1 = inv ? s1v : -s1v, s2 = inv ? s2v : -s2v;
        float2 t1 = cadd(a[1], a[4]), d1 = csub(a[1], a[4]);
        float2 t2 = cadd(a[2], a[3]), d2 = csub(a[2], a[3]);
        float2 b0 = make_float2(a[0].x + t1.x + t2.x, a[0].y + t1.y + t2.y);
        float2 m1 = make_float2(a[0].x + c1 * t1.x + c2 * t2.x, a[0].y + c1 * t1.y + c2 * t2.y);
        float2 m2 = make_float2(a[0].x + c2 * t1.x + c1 * t2.x, a[0].y + c2 * t1.y + c1 * t2.y);
        // i * (s1 d1 + s2 d2) and i * (s2 d1 - s1 d2)
        float2 n1 = make_float2(s1 * d1.x + s2 * d2.x, s1 * d1.y + s2 * d2.y);
        float2 n2 = make_float2(s2 * d1.x - s1 * d2.x, s2 * d1.y - s1 * d2.y);
        float2 r1 = make_float2(-n1.y, n1.x), r2 = make_float2(-n2.y, n2.x);
        a[0] = b0;
        a[1] = cadd(m1, r1);
        a[4] = csub(m1, r1);
        a[2] = cadd(m2, r2);
        a[3] = csub(m2, r2);
    }
}

// One Stockham pass of radix R over `nbatch` length-n lines in LDS.
// element i of line b lives at buf[i*si + b*sb].  ifast: butterfly index
// varies fastest across threads (use when si == 1), else the line index does.
template <int R, int MAXPTS>
DLCS_DEV void stockham_pass(float2* buf, int si, int sb, int nbatch, int n, int p,
                            const float2* tw, bool inv, bool ifast) {
    constexpr int kIt = MAXPTS / R + ((MAXPTS % R) ? 1 : 0);
    const int nbf = n / R;
    const int total = nbf * nbatch;
    const int tstride = n / (p * R);
    float2 v[kIt][R];
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
        const int bf = threadIdx.x + it * kThreads;
        if (bf < total) {
            const int b = ifast ? bf / nbf : bf % nbatch;
            const int i = ifast ? bf % nbf : bf / nbatch;
            const int k = i % p;
#pragma unroll
            for (int t = 0; t < R; ++t) {
                float2 a = buf[(i + t * nbf) * si + b * sb];
                if (t > 0) {
                    const float2 w = tw[(t * k * tstride) % n];
                    a = inv ? cmulc(a, w) : cmul(a, w);
                }
                v[it][t] = a;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
        const int bf = threadIdx.x + it * kThreads;
        if (bf < total) {
            const int b = ifast ? bf / nbf : bf % nbatch;
            const int i = ifast ? bf % nbf : bf / nbatch;
            const int k = i % p;
            dft<R>(v[it], inv);
            const int j = (i - k) * R + k;
#pragma unroll
            for (int s = 0; s < R; ++s) buf[(j + s * p) * si + b * sb] = v[it][s];
        }
    }
    __syncthreads();
}

template <int MAXPTS>
DLCS_DEV void fft_lds(float2* buf, int si, int sb, int nbatch, const FftPlan& plan,
                      const float2* tw, bool inv) {
    const bool ifast = (si == 1);
    int p = 1;
    for (int q = 0; q < plan.npass; ++q) {
        const int r = plan.radix[q];
        switch (r) {
            case 2: stockham_pass<2, MAXPTS>(buf, si, sb, nbatch, plan.n, p, tw, inv, ifast); break;
            case 3: stockham_pass<3, MAXPTS>(buf, si, sb, nbatch, plan.n, p, tw, inv, ifast); break;
            case 4: stockham_pass<4, MAXPTS>(buf, si, sb, nbatch, plan.n, p, tw, inv, ifast); break;
            default: stockham_pass<5, MAXPTS>(buf, si, sb, nbatch, plan.n, p, tw, inv, ifast); break;
        }
        p *= r;
    }
}

// ---------------------------------------------------------------------------
// Row pass (FFT along X over `rows` consecutive lines of one (b, t) frame).
// MODE 0: plain (in = planes)                       out = F_x(in)
// MODE 1: SENSE forward: in = x, coil images sum_e S_e x_e, loop over coils
// MODE 2: SENSE adjoint: in = tmp (after the Y pass), acc_e += conj(S_e) F_x^-1
// ---------------------------------------------------------------------------
struct RowArgs {
    const float2* in;      // MODE0: [P,Y,X]; MODE1: x [B,E,T,Y,X]; MODE2: tmp [B,C,T,Y,X]
    const float2* maps;    // [B,E,C,Y,X]
    float2* out;           // MODE0: [P,Y,X]; MODE1: tmp [B,C,T,Y,X]; MODE2: x [B,E,T,Y,X]
    const float2* base;    // MODE2 epilogue (may be null)
    const float2* sub;     // MODE2 epilogue (may be null)
    float step, scale;
    float bscale;          // MODE2 epilogue: out = bscale * base + step * (v - sub)
    int B, E, C, T, Y, X, rows;
    int inverse;
    FftPlan plan;
    int dbg_nofft;         // timing experiments only (DLCS_SENSE_NOFFT=1): skip the FFT
};

template <int MODE>
__global__ void __launch_bounds__(kThreads) sense_rows_kernel(RowArgs a) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    float2* tw = smem;                      // [X]
    float2* buf = smem + a.X;               // [rows * X]
    const int X = a.X, Y = a.Y;
    const int y0 = blockIdx.x * a.rows;
    const int nrow = min(a.rows, Y - y0);
    const int npts = nrow * X;
    const int frame = blockIdx.y;           // MODE0: plane; else b*T + t
    build_twiddles(tw, X);
    const bool inv = (MODE == 2) ? true : (MODE == 1 ? false : a.inverse != 0);

    if constexpr (MODE == 0) {
        const float2* src = a.in + ((size_t)frame * Y + y0) * X;
        for (int i = threadIdx.x; i < npts; i += kThreads) buf[i] = src[i];
        __syncthreads();
        fft_lds<kRowPts>(buf, 1, X, nrow, a.plan, tw, inv);
        float2* dst = a.out + ((size_t)frame * Y + y0) * X;
        for (int i = threadIdx.x; i < npts; i += kThreads)
            dst[i] = make_float2(buf[i].x * a.scale, buf[i].y * a.scale);
    } else if constexpr (MODE == 1) {
        const int b = frame / a.T, t = frame % a.T;
        float2 xv[kMaxE][kRowPts];
#pragma unroll
        for (int e = 0; e < kMaxE; ++e) {
            if (e < a.E) {
                const float2* src = a.in + ((((size_t)b * a.E + e) * a.T + t) * Y + y0) * X;
#pragma unroll
                for (int k = 0; k < kRowPts; ++k) {
                    const int i = threadIdx.x + k * kThreads;
                    if (i < npts) xv[e][k] = src[i];
                }
            }
        }
        for (int c = 0; c < a.C; ++c) {
#pragma unroll
            for (int k = 0; k < kRowPts; ++k) {
                const int i = threadIdx.x + k * kThreads;
                if (i < npts) {
                    float2 acc = make_float2(0.f, 0.f);
#pragma unroll
                    for (int e = 0; e < kMaxE; ++e) {
                        if (e < a.E) {
                            const float2 s = a.maps[(((size_t)b * a.E + e) * a.C + c) * Y * X + (size_t)y0 * X + i];
                            acc = cadd(acc, cmul(s, xv[e][k]));
                        }
                    }
                    buf[i] = acc;
                }
            }
            __syncthreads();
            fft_lds<kRowPts>(buf, 1, X, nrow, a.plan, tw, false);
            float2* dst = a.out + ((((size_t)b * a.C + c) * a.T + t) * Y + y0) * X;
            for (int i = threadIdx.x; i < npts; i += kThreads) dst[i] = buf[i];
            __syncthreads();
        }
    } else {
        const int b = frame / a.T, t = frame % a.T;
        float2 acc[kMaxE][kRowPts];
#pragma unroll
        for (int e = 0; e < kMaxE; ++e)
#pragma unroll
            for (int k = 0; k < kRowPts; ++k) acc[e][k] = make_float2(0.f, 0.f);
        for (int c = 0; c < a.C; ++c) {
            const float2* src = a.in + ((((size_t)b * a.C + c) * a.T + t) * Y + y0) * X;
            for (int i = threadIdx.x; i < npts; i += kThreads) buf[i] = src[i];
            __syncthreads();
            fft_lds<kRowPts>(buf, 1, X, nrow, a.plan, tw, true);
#pragma unroll
            for (int k = 0; k < kRowPts; ++k) {
                const int i = threadIdx.x + k * kThreads;
                if (i < npts) {
                    const float2 v = buf[i];
#pragma unroll
                    for (int e = 0; e < kMaxE; ++e) {
                        if (e < a.E) {
                            const float2 s = a.maps[(((size_t)b * a.E + e) * a.C + c) * Y * X + (size_t)y0 * X + i];
                            acc[e][k] = cadd(acc[e][k], cmulc(v, s));
                        }
                    }
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int e = 0; e < kMaxE; ++e) {
            if (e < a.E) {
                const size_t off = ((((size_t)b * a.E + e) * a.T + t) * Y + y0) * X;
#pragma unroll
                for (int k = 0; k < kRowPts; ++k) {
                    const int i = threadIdx.x + k * kThreads;
                    if (i < npts) {
                        float2 v = make_float2(acc[e][k].x * a.scale, acc[e][k].y * a.scale);
                        if (a.base) {
                            float2 s = a.sub ? a.sub[off + i] : make_float2(0.f, 0.f);
                            float2 bb = a.base[off + i];
                            v = make_float2(a.bscale * bb.x + a.step * (v.x - s.x), a.bscale * bb.y + a.step * (v.y - s.y));
                        }
                        a.out[off + i] = v;
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Column pass (FFT along Y over `cols` consecutive columns of one plane).
// pre-multiply by weights (adjoint) or post-multiply (forward), times scale.
// ---------------------------------------------------------------------------
struct ColArgs {
    const float2* in;
    float2* out;
    const float* weights;   // [B,Wc,T,Y,X] or null
    int wc;                 // 1 or C
    int B, C, T, Y, X, cols;
    int inverse;
    int weights_pre;        // 1: multiply before the FFT (adjoint), 0: after (forward)
    int normal;             // fast path only: FFT, weights^2, IFFT in one pass (dlcs_sense_normal)
    float scale;
    FftPlan plan;
};

__global__ void __launch_bounds__(kThreads) sense_cols_kernel(ColArgs a) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    float2* tw = smem;
    float2* buf = smem + a.Y;
    const int X = a.X, Y = a.Y;
    const int x0 = blockIdx.x * a.cols;
    const int ncol = min(a.cols, X - x0);
    const int plane = blockIdx.y;           // (b*C + c)*T + t   (or generic plane)
    const int npts = ncol * Y;
    build_twiddles(tw, Y);
    const float* wrow = nullptr;
    if (a.weights) {
        const int t = plane % a.T;
        const int c = (plane / a.T) % a.C;
        const int b = plane / (a.T * a.C);
        const int cw = (a.wc == 1) ? 0 : c;
        wrow = a.weights + (((size_t)b * a.wc + cw) * a.T + t) * Y * X;
    }
    const float2* src = a.in + (size_t)plane * Y * X;
    for (int i = threadIdx.x; i < npts; i += kThreads) {
        const int y = i / ncol, j = i % ncol;
        float2 v = src[(size_t)y * X + x0 + j];
        if (wrow && a.weights_pre) {
            const float w = wrow[(size_t)y * X + x0 + j];
            v = make_float2(v.x * w, v.y * w);
        }
        buf[y * ncol + j] = v;
    }
    __syncthreads();
    fft_lds<kMaxPts>(buf, ncol, 1, ncol, a.plan, tw, a.inverse != 0);
    float2* dst = a.out + (size_t)plane * Y * X;
    for (int i = threadIdx.x; i < npts; i += kThreads) {
        const int y = i / ncol, j = i % ncol;
        float2 v = buf[y * ncol + j];
        float s = a.scale;
        if (wrow && !a.weights_pre) s *= wrow[(size_t)y * X + x0 + j];
        dst[(size_t)y * X + x0 + j] = make_float2(v.x * s, v.y * s);
    }
}

static int sense_nofft() {
    static const int v = [] { const char* s = dlcs_knob("DLCS_SENSE_NOFFT"); return s && s[0] == '1' ? 1 : 0; }();
    return v;
}
#include "sense_fast.inc"
#include "sense_rows.inc"

static int rows_per_block(int X, int Y) { int r = kRowPoints / X; if (r < 1) r = 1; return r > Y ? Y : r; }
static int cols_per_block(int X, int Y) { int c = kPoints / Y; if (c > 16) c = 16; if (c < 1) c = 1; return c > X ? X : c; }

}  // namespace

namespace {

// ---------------------------------------------------------------------------
// Conjugate gradient on the SENSE normal operator (alg:11-73, urs:151-158):
// every scalar of the recurrence stays on the device.  Per iteration:
//   Ap = (A^H A + lamda) p                       dlcs_sense_normal (3 launches)
//   pAp partials      <- sum conj(p) Ap          cg_dot_kernel
//   alpha = rs / pAp; x += alpha p; r -= alpha Ap; |r|^2 partials   cg_update_kernel
//   beta = rs' / rs;  p = beta p + r             cg_direction_kernel
// Reductions: per-block fp64 partials, re-reduced by every block of the next
// launch (<= kCgBlocks partials), so no grid-wide sync and no host round trip.
// rs is double-buffered by iteration parity: block 0 of cg_direction writes
// the next slot while every block reads the current one.
// ---------------------------------------------------------------------------
constexpr int kCgBlocks = 512, kCgThreads = 256;

struct CgScalars {
    double2 pap[kCgBlocks];      // partials of sum conj(p) Ap
    double rr[kCgBlocks];        // partials of sum |r|^2
    double rs[2];                // rsold, double-buffered by iteration parity
};

DLCS_DEV double block_sum_d(double v, double* sh) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    double t = 0.0;
    for (int i = 0; i < nw; ++i) t += sh[i];
    return t;
}

// sum of the first n partials, every thread gets it
DLCS_DEV double sum_partials(const double* p, int n, double* sh) {
    double v = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) v += p[i];
    return block_sum_d(v, sh);
}

__global__ void __launch_bounds__(kCgThreads) cg_dot_kernel(const float2* p, const float2* ap, long n, CgScalars* sc) {
    __shared__ double sh[kCgThreads / 64];
    double re = 0.0, im = 0.0;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float2 a = p[i], b = ap[i];
        re += (double)a.x * b.x + (double)a.y * b.y;       // conj(a) b
        im += (double)a.x * b.y - (double)a.y * b.x;
    }
    re = block_sum_d(re, sh);
    im = block_sum_d(im, sh);
    if (threadIdx.x == 0) sc->pap[blockIdx.x] = make_double2(re, im);
}

// |r|^2 partials of r (the first residual)
__global__ void __launch_bounds__(kCgThreads) cg_norm_kernel(const float2* r, long n, CgScalars* sc) {
    __shared__ double sh[kCgThreads / 64];
    double v = 0.0;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float2 a = r[i];
        v += (double)a.x * a.x + (double)a.y * a.y;
    }
    v = block_sum_d(v, sh);
    if (threadIdx.x == 0) sc->rr[blockIdx.x] = v;
}

__global__ void __launch_bounds__(kCgThreads) cg_init_rs_kernel(CgScalars* sc, int nblk) {
    __shared__ double sh[kCgThreads / 64];
    const double v = sum_partials(sc->rr, nblk, sh);
    if (threadIdx.x == 0) sc->rs[0] = v;
}

__global__ void __launch_bounds__(kCgThreads) cg_update_kernel(float2* x, float2* r, const float2* p, const float2* ap,
                                                               long n, CgScalars* sc, int nblk, int slot) {
    __shared__ double sh[kCgThreads / 64];
    __shared__ double2 pap_sh;
    double pre = 0.0, pim = 0.0;
    for (int i = threadIdx.x; i < nblk; i += blockDim.x) { pre += sc->pap[i].x; pim += sc->pap[i].y; }
    pre = block_sum_d(pre, sh);
    pim = block_sum_d(pim, sh);
    if (threadIdx.x == 0) pap_sh = make_double2(pre, pim);
    __syncthreads();
    // alpha = rs / pAp in complex64 arithmetic, as the reference's torch scalars
    const float rs = (float)sc->rs[slot];
    const float ar = (float)pap_sh.x, ai = (float)pap_sh.y;
    const float den = ar * ar + ai * ai;
    const float2 alpha = make_float2(rs * ar / den, -rs * ai / den);
    double v = 0.0;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float2 pv = p[i], av = ap[i];
        float2 xv = x[i], rv = r[i];
        xv = cadd(xv, cmul(alpha, pv));
        rv = csub(rv, cmul(alpha, av));
        x[i] = xv;
        r[i] = rv;
        v += (double)rv.x * rv.x + (double)rv.y * rv.y;
    }
    v = block_sum_d(v, sh);
    if (threadIdx.x == 0) sc->rr[blockIdx.x] = v;
}

__global__ void __launch_bounds__(kCgThreads) cg_direction_kernel(float2* p, const float2* r, long n, CgScalars* sc,
                                                                  int nblk, int slot) {
    __shared__ double sh[kCgThreads / 64];
    const double rsnew = sum_partials(sc->rr, nblk, sh);
    const float beta = (float)rsnew / (float)sc->rs[slot];
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float2 pv = p[i], rv = r[i];
        p[i] = make_float2(beta * pv.x + rv.x, beta * pv.y + rv.y);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) sc->rs[slot ^ 1] = rsnew;
}

}  // namespace

extern "C" {

int dlcs_version(void) { return DLCS_VERSION; }

const char* dlcs_status_string(int s) {
    switch (s) {
        case DLCS_OK: return "ok";
        case DLCS_ERR_INVALID_ARG: return "invalid argument";
        case DLCS_ERR_UNSUPPORTED_SIZE: return "unsupported size";
        case DLCS_ERR_WORKSPACE: return "workspace too small";
        default: return hipGetErrorString((hipError_t)s);
    }
}

size_t dlcs_sense_workspace_bytes(int64_t B, int64_t C, int64_t T, int64_t Y, int64_t X) {
    return (size_t)(B * C * T * Y * X) * sizeof(float2);
}

int dlcs_fft2(const void* in, void* out, int64_t nplanes, int64_t Y, int64_t X, int inverse,
              void* workspace, size_t workspace_bytes, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(in && out && nplanes > 0);
    FftPlan px, py;
    if (!make_plan((int)X, px) || !make_plan((int)Y, py) || X > kRowPoints || Y > kPoints) return DLCS_ERR_UNSUPPORTED_SIZE;
    if (workspace_bytes < (size_t)(nplanes * Y * X) * sizeof(float2) || !workspace) return DLCS_ERR_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    const float scale = 1.0f / sqrtf((float)(Y * X));
    RowArgs ra{};
    ra.in = (const float2*)in; ra.out = (float2*)workspace; ra.scale = 1.0f;
    ra.Y = (int)Y; ra.X = (int)X; ra.rows = rows_per_block((int)X, (int)Y); ra.inverse = inverse; ra.plan = px;
    ra.B = 1; ra.E = 1; ra.C = 1; ra.T = 1;
    bool done = false;
    if (rows_fast_ok(Y, X, 1)) {
        const dim3 g(cdiv(Y, kFLW * kFRowWaves), (unsigned)nplanes);
        done = inverse ? rows_fast<0, true>((int)X, ra, g, kFRowWaves * 64, st)
                       : rows_fast<0, false>((int)X, ra, g, kFRowWaves * 64, st);
    }
    if (!done) {
        dim3 g1(cdiv(Y, ra.rows), (unsigned)nplanes);
        size_t sh1 = (size_t)(X + ra.rows * X) * sizeof(float2);
        hipLaunchKernelGGL(sense_rows_kernel<0>, g1, dim3(kThreads), sh1, st, ra);
    }
    ColArgs ca{};
    ca.in = (const float2*)workspace; ca.out = (float2*)out; ca.weights = nullptr; ca.wc = 1;
    ca.B = 1; ca.C = 1; ca.T = (int)nplanes; ca.Y = (int)Y; ca.X = (int)X;
    ca.cols = cols_per_block((int)X, (int)Y); ca.inverse = inverse; ca.weights_pre = 0; ca.scale = scale; ca.plan = py;
    done = false;
    if (cols_fast_ok(Y, X)) {
        const dim3 g((unsigned)(X / kFColW), (unsigned)nplanes);
        done = inverse ? cols_fast<true>((int)Y, ca, g, st) : cols_fast<false>((int)Y, ca, g, st);
    }
    if (!done) {
        dim3 g2(cdiv(X, ca.cols), (unsigned)nplanes);
        size_t sh2 = (size_t)(Y + ca.cols * Y) * sizeof(float2);
        hipLaunchKernelGGL(sense_cols_kernel, g2, dim3(kThreads), sh2, st, ca);
    }
    return dlcs_launch_status();
}

int dlcs_sense_fwd(const void* x, const void* maps, const float* weights, int64_t weights_coils,
                   void* y, int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                   void* workspace, size_t workspace_bytes, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(x && maps && y && B > 0 && E > 0 && C > 0 && T > 0);
    if (E > kMaxE) return DLCS_ERR_UNSUPPORTED_SIZE;
    DLCS_CHECK_ARG(!weights || weights_coils == 1 || weights_coils == C);
    FftPlan px, py;
    if (!make_plan((int)X, px) || !make_plan((int)Y, py) || X > kRowPoints || Y > kPoints) return DLCS_ERR_UNSUPPORTED_SIZE;
    if (!workspace || workspace_bytes < dlcs_sense_workspace_bytes(B, C, T, Y, X)) return DLCS_ERR_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    RowArgs ra{};
    ra.in = (const float2*)x; ra.maps = (const float2*)maps; ra.out = (float2*)workspace;
    ra.scale = 1.0f; ra.B = (int)B; ra.E = (int)E; ra.C = (int)C; ra.T = (int)T; ra.Y = (int)Y; ra.X = (int)X;
    ra.rows = rows_per_block((int)X, (int)Y); ra.plan = px;
    ra.dbg_nofft = sense_nofft();
    bool done = false;
    if (rows_fast_ok(Y, X, E)) {
        const int nw = (int)std::min<int64_t>(C, kFRowWaves);
        done = rows_fast<1, false>((int)X, ra, dim3(cdiv(Y, kFLW), (unsigned)(B * T)), nw * 64, st);
    }
    if (!done) {
        dim3 g1(cdiv(Y, ra.rows), (unsigned)(B * T));
        size_t sh1 = (size_t)(X + ra.rows * X) * sizeof(float2);
        hipLaunchKernelGGL(sense_rows_kernel<1>, g1, dim3(kThreads), sh1, st, ra);
    }
    ColArgs ca{};
    ca.in = (const float2*)workspace; ca.out = (float2*)y; ca.weights = weights; ca.wc = (int)(weights ? weights_coils : 1);
    ca.B = (int)B; ca.C = (int)C; ca.T = (int)T; ca.Y = (int)Y; ca.X = (int)X;
    ca.cols = cols_per_block((int)X, (int)Y); ca.inverse = 0; ca.weights_pre = 0;
    ca.scale = 1.0f / sqrtf((float)(Y * X)); ca.plan = py;
    done = false;
    if (cols_fast_ok(Y, X)) done = cols_fast<false>((int)Y, ca, dim3((unsigned)(X / kFColW), (unsigned)(B * C * T)), st);
    if (!done) {
        dim3 g2(cdiv(X, ca.cols), (unsigned)(B * C * T));
        size_t sh2 = (size_t)(Y + ca.cols * Y) * sizeof(float2);
        hipLaunchKernelGGL(sense_cols_kernel, g2, dim3(kThreads), sh2, st, ca);
    }
    return dlcs_launch_status();
}

int dlcs_sense_adj(const void* y, const void* maps, const float* weights, int64_t weights_coils,
                   void* out, const void* base, const void* sub, float step,
                   int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                   void* workspace, size_t workspace_bytes, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(y && maps && out && B > 0 && E > 0 && C > 0 && T > 0);
    if (E > kMaxE) return DLCS_ERR_UNSUPPORTED_SIZE;
    DLCS_CHECK_ARG(!weights || weights_coils == 1 || weights_coils == C);
    FftPlan px, py;
    if (!make_plan((int)X, px) || !make_plan((int)Y, py) || X > kRowPoints || Y > kPoints) return DLCS_ERR_UNSUPPORTED_SIZE;
    if (!workspace || workspace_bytes < dlcs_sense_workspace_bytes(B, C, T, Y, X)) return DLCS_ERR_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    ColArgs ca{};
    ca.in = (const float2*)y; ca.out = (float2*)workspace; ca.weights = weights; ca.wc = (int)(weights ? weights_coils : 1);
    ca.B = (int)B; ca.C = (int)C; ca.T = (int)T; ca.Y = (int)Y; ca.X = (int)X;
    ca.cols = cols_per_block((int)X, (int)Y); ca.inverse = 1; ca.weights_pre = 1; ca.scale = 1.0f; ca.plan = py;
    bool done = false;
    if (cols_fast_ok(Y, X)) done = cols_fast<true>((int)Y, ca, dim3((unsigned)(X / kFColW), (unsigned)(B * C * T)), st);
    if (!done) {
        dim3 g1(cdiv(X, ca.cols), (unsigned)(B * C * T));
        size_t sh1 = (size_t)(Y + ca.cols * Y) * sizeof(float2);
        hipLaunchKernelGGL(sense_cols_kernel, g1, dim3(kThreads), sh1, st, ca);
    }
    RowArgs ra{};
    ra.in = (const float2*)workspace; ra.maps = (const float2*)maps; ra.out = (float2*)out;
    ra.base = (const float2*)base; ra.sub = (const float2*)sub; ra.step = step; ra.bscale = 1.0f;
    ra.scale = 1.0f / sqrtf((float)(Y * X));
    ra.B = (int)B; ra.E = (int)E; ra.C = (int)C; ra.T = (int)T; ra.Y = (int)Y; ra.X = (int)X;
    ra.rows = rows_per_block((int)X, (int)Y); ra.plan = px;
    ra.dbg_nofft = sense_nofft();
    done = false;
    if (rows_fast_ok(Y, X, E)) {
        const int nw = (int)std::min<int64_t>(C, kFRowWaves);
        done = rows_fast<2, true>((int)X, ra, dim3(cdiv(Y, kFLW), (unsigned)(B * T)), nw * 64, st);
    }
    if (!done) {
        dim3 g2(cdiv(Y, ra.rows), (unsigned)(B * T));
        size_t sh2 = (size_t)(X + ra.rows * X) * sizeof(float2);
        hipLaunchKernelGGL(sense_rows_kernel<2>, g2, dim3(kThreads), sh2, st, ra);
    }
    return dlcs_launch_status();
}

/* out = base_scale * x + step * (A^H A x - sub): the PGD data-consistency step
 * (base_scale 1, step s, sub A^H y; urs:109) or the HQS normal operator
 * (base_scale lamda, step 1, sub NULL; urs:151).  Three launches: the forward
 * row pass, ONE column pass (FFT_Y, weights^2, IFFT_Y: the k-space of a plane
 * never leaves LDS) and the adjoint row pass with the epilogue. */
int dlcs_sense_normal(const void* x, const void* maps, const float* weights, int64_t weights_coils,
                      void* out, const void* sub, float base_scale, float step,
                      int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                      void* workspace, size_t workspace_bytes, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(x && maps && out && B > 0 && E > 0 && C > 0 && T > 0 && out != x);
    if (E > kMaxE) return DLCS_ERR_UNSUPPORTED_SIZE;
    DLCS_CHECK_ARG(!weights || weights_coils == 1 || weights_coils == C);
    FftPlan px, py;
    if (!make_plan((int)X, px) || !make_plan((int)Y, py) || X > kRowPoints || Y > kPoints) return DLCS_ERR_UNSUPPORTED_SIZE;
    if (!workspace || workspace_bytes < dlcs_sense_workspace_bytes(B, C, T, Y, X)) return DLCS_ERR_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    float2* k = (float2*)workspace;
    // forward row pass: coil combine + FFT_X -> k
    RowArgs ra{};
    ra.in = (const float2*)x; ra.maps = (const float2*)maps; ra.out = k;
    ra.scale = 1.0f; ra.B = (int)B; ra.E = (int)E; ra.C = (int)C; ra.T = (int)T; ra.Y = (int)Y; ra.X = (int)X;
    ra.rows = rows_per_block((int)X, (int)Y); ra.plan = px;
    ra.dbg_nofft = sense_nofft();
    bool done = false;
    if (rows_fast_ok(Y, X, E)) {
        const int nw = (int)std::min<int64_t>(C, kFRowWaves);
        done = rows_fast<1, false>((int)X, ra, dim3(cdiv(Y, kFLW), (unsigned)(B * T)), nw * 64, st);
    }
    if (!done) {
        dim3 g1(cdiv(Y, ra.rows), (unsigned)(B * T));
        size_t sh1 = (size_t)(X + ra.rows * X) * sizeof(float2);
        hipLaunchKernelGGL(sense_rows_kernel<1>, g1, dim3(kThreads), sh1, st, ra);
    }
    // column passes, in place on k
    ColArgs ca{};
    ca.in = k; ca.out = k; ca.weights = weights; ca.wc = (int)(weights ? weights_coils : 1);
    ca.B = (int)B; ca.C = (int)C; ca.T = (int)T; ca.Y = (int)Y; ca.X = (int)X;
    ca.cols = cols_per_block((int)X, (int)Y); ca.plan = py;
    if (cols_fast_ok(Y, X)) {
        ca.normal = 1; ca.inverse = 0; ca.weights_pre = 0; ca.scale = 1.0f / sqrtf((float)(Y * X));
        cols_fast<false>((int)Y, ca, dim3((unsigned)(X / kFColW), (unsigned)(B * C * T)), st);
    } else {
        dim3 g2(cdiv(X, ca.cols), (unsigned)(B * C * T));
        size_t sh2 = (size_t)(Y + ca.cols * Y) * sizeof(float2);
        ca.inverse = 0; ca.weights_pre = 0; ca.scale = 1.0f / sqrtf((float)(Y * X));
        hipLaunchKernelGGL(sense_cols_kernel, g2, dim3(kThreads), sh2, st, ca);
        ca.inverse = 1; ca.weights_pre = 1; ca.scale = 1.0f;
        hipLaunchKernelGGL(sense_cols_kernel, g2, dim3(kThreads), sh2, st, ca);
    }
    // adjoint row pass: IFFT_X, conj-map coil sum, epilogue
    RowArgs rb = ra;
    rb.in = k; rb.out = (float2*)out;
    rb.base = (const float2*)x; rb.sub = (const float2*)sub; rb.step = step; rb.bscale = base_scale;
    rb.scale = 1.0f / sqrtf((float)(Y * X));
    done = false;
    if (rows_fast_ok(Y, X, E)) {
        const int nw = (int)std::min<int64_t>(C, kFRowWaves);
        done = rows_fast<2, true>((int)X, rb, dim3(cdiv(Y, kFLW), (unsigned)(B * T)), nw * 64, st);
    }
    if (!done) {
        dim3 g2(cdiv(Y, rb.rows), (unsigned)(B * T));
        size_t sh2 = (size_t)(X + rb.rows * X) * sizeof(float2);
        hipLaunchKernelGGL(sense_rows_kernel<2>, g2, dim3(kThreads), sh2, st, rb);
    }
    return dlcs_launch_status();
}

size_t dlcs_sense_cg_workspace_bytes(int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X) {
    const size_t n = (size_t)(B * E * T * Y * X);
    return dlcs_sense_workspace_bytes(B, C, T, Y, X) + 3 * n * sizeof(float2) + ((sizeof(CgScalars) + 255) & ~(size_t)255);
}

/* Row-sparse normal operator (sense_rows.inc): the row table of a weights
 * tensor, built once per mask, and the three-launch operator on it. */
size_t dlcs_sense_rowtab_bytes(int64_t B, int64_t weights_coils, int64_t T, int64_t Y) {
    return (size_t)(kRtHdr + B * weights_coils * T * (1 + Y)) * sizeof(int);
}

int dlcs_sense_rowtab(const float* weights, int64_t weights_coils, int64_t B, int64_t T, int64_t Y, int64_t X,
                      void* table, size_t table_bytes, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(weights && table && B > 0 && T > 0 && Y > 0 && X > 0 && weights_coils > 0);
    if (Y > 1024) return DLCS_ERR_UNSUPPORTED_SIZE;
    if (table_bytes < dlcs_sense_rowtab_bytes(B, weights_coils, T, Y)) return DLCS_ERR_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(table, 0, kRtHdr * sizeof(int), st) != hipSuccess) return dlcs_launch_status();
    const int planes = (int)(B * weights_coils * T);
    hipLaunchKernelGGL(rowtab_kernel, dim3((unsigned)planes), dim3(256), 0, st, weights, (int)Y, (int)X, planes, (int*)table);
    return dlcs_launch_status();
}

size_t dlcs_sense_rows_workspace_bytes(int64_t B, int64_t C, int64_t T, int64_t jcap, int64_t X) {
    return (size_t)(B * C * T * std::max<int64_t>(jcap, 1) * X) * sizeof(float2);
}

int dlcs_sense_normal_rows(const void* x, const void* maps, const float* weights, int64_t weights_coils,
                           const void* table, int64_t jcap, void* out, const void* sub, float base_scale, float step,
                           int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                           void* workspace, size_t workspace_bytes, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(x && maps && weights && table && out && B > 0 && E > 0 && C > 0 && T > 0 && out != x);
    DLCS_CHECK_ARG(weights_coils == 1 || weights_coils == C);
    DLCS_CHECK_ARG(jcap >= 0 && jcap <= Y);
    if (E > kMaxE || !fast_len(Y) || !fast_len(X) || X % kFColW) return DLCS_ERR_UNSUPPORTED_SIZE;
    if (!workspace || workspace_bytes < dlcs_sense_rows_workspace_bytes(B, C, T, jcap, X)) return DLCS_ERR_WORKSPACE;
    NrmArgs na{};
    na.x = (const float2*)x; na.maps = (const float2*)maps; na.weights = weights; na.wc = (int)weights_coils;
    const int* tab = (const int*)table;
    na.cnt = tab + kRtHdr; na.rows = tab + kRtHdr + B * weights_coils * T;
    na.k = (float2*)workspace; na.out = (float2*)out; na.sub = (const float2*)sub;
    na.bscale = base_scale; na.step = step; na.scale = 1.0f / (float)(Y * X);
    na.B = (int)B; na.E = (int)E; na.C = (int)C; na.T = (int)T; na.Y = (int)Y; na.X = (int)X;
    na.jcap = (int)std::max<int64_t>(jcap, 1);
    if (!nrm_launch(na, sub != nullptr, (hipStream_t)stream)) return DLCS_ERR_UNSUPPORTED_SIZE;
    return dlcs_launch_status();
}

int dlcs_sense_adj_rows(const void* y, const void* maps, const float* weights, int64_t weights_coils,
                        const void* table, int64_t jcap, void* out, const void* base, const void* sub, float step,
                        int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                        void* workspace, size_t workspace_bytes, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(y && maps && weights && table && out && B > 0 && E > 0 && C > 0 && T > 0);
    DLCS_CHECK_ARG(weights_coils == 1 || weights_coils == C);
    DLCS_CHECK_ARG(jcap >= 0 && jcap <= Y && out != base && out != sub);
    if (E > kMaxE || !fast_len(Y) || !fast_len(X) || X % kFColW) return DLCS_ERR_UNSUPPORTED_SIZE;
    if (!workspace || workspace_bytes < dlcs_sense_rows_workspace_bytes(B, C, T, jcap, X)) return DLCS_ERR_WORKSPACE;
    NrmArgs na{};
    na.x = (const float2*)base; na.maps = (const float2*)maps; na.weights = weights; na.wc = (int)weights_coils;
    const int* tab = (const int*)table;
    na.cnt = tab + kRtHdr; na.rows = tab + kRtHdr + B * weights_coils * T;
    na.k = (float2*)workspace; na.out = (float2*)out; na.sub = (const float2*)sub;
    na.bscale = base ? 1.0f : 0.0f; na.step = step; na.scale = 1.0f / sqrtf((float)(Y * X));
    na.B = (int)B; na.E = (int)E; na.C = (int)C; na.T = (int)T; na.Y = (int)Y; na.X = (int)X;
    na.jcap = (int)std::max<int64_t>(jcap, 1);
    if (!nrm_adj_rows(na, (const float2*)y, sub != nullptr, (hipStream_t)stream)) return DLCS_ERR_UNSUPPORTED_SIZE;
    return dlcs_launch_status();
}

/* x <- num_iter conjugate-gradient steps on (A^H A + lamda I) x = b from x
 * (alg:50-73 with model_normal of urs:151); in place on x, no host sync.
 * table != NULL: the normal operator runs row-sparse (dlcs_sense_normal_rows). */
static int sense_cg_impl(void* x, const void* b, const void* maps, const float* weights, int64_t weights_coils,
                         const void* table, int64_t jcap,
                         float lamda, int num_iter, int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                         void* workspace, size_t workspace_bytes, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(x && b && maps && num_iter >= 0 && B > 0 && E > 0 && C > 0 && T > 0);
    if (!workspace || workspace_bytes < dlcs_sense_cg_workspace_bytes(B, E, C, T, Y, X)) return DLCS_ERR_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    const long n = (long)(B * E * T * Y * X);
    const size_t kbytes = dlcs_sense_workspace_bytes(B, C, T, Y, X);
    char* w = (char*)workspace;
    float2* r = (float2*)(w + kbytes);
    float2* p = r + n;
    float2* ap = p + n;
    CgScalars* sc = (CgScalars*)(ap + n);
    const int nblk = (int)std::min<long>(kCgBlocks, std::max<long>(1, (n + 4L * kCgThreads - 1) / (4L * kCgThreads)));
    auto normal = [&](const void* in, void* o, const void* sub, float bs, float stp) {
        if (table)
            return dlcs_sense_normal_rows(in, maps, weights, weights_coils, table, jcap, o, sub, bs, stp,
                                          B, E, C, T, Y, X, workspace, kbytes, stream);
        return dlcs_sense_normal(in, maps, weights, weights_coils, o, sub, bs, stp, B, E, C, T, Y, X,
                                 workspace, kbytes, stream);
    };
    // r = b - (A^H A + lamda) x
    int rc = normal(x, r, b, -lamda, -1.0f);
    if (rc) return rc;
    if (hipMemcpyAsync(p, r, n * sizeof(float2), hipMemcpyDeviceToDevice, st) != hipSuccess) return dlcs_launch_status();
    hipLaunchKernelGGL(cg_norm_kernel, dim3(nblk), dim3(kCgThreads), 0, st, r, n, sc);
    hipLaunchKernelGGL(cg_init_rs_kernel, dim3(1), dim3(kCgThreads), 0, st, sc, nblk);
    for (int it = 0; it < num_iter; ++it) {
        const int slot = it & 1;
        rc = normal(p, ap, nullptr, lamda, 1.0f);
        if (rc) return rc;
        hipLaunchKernelGGL(cg_dot_kernel, dim3(nblk), dim3(kCgThreads), 0, st, p, ap, n, sc);
        hipLaunchKernelGGL(cg_update_kernel, dim3(nblk), dim3(kCgThreads), 0, st, (float2*)x, r, p, ap, n, sc, nblk, slot);
        hipLaunchKernelGGL(cg_direction_kernel, dim3(nblk), dim3(kCgThreads), 0, st, p, r, n, sc, nblk, slot);
    }
    return dlcs_launch_status();
}

int dlcs_sense_cg(void* x, const void* b, const void* maps, const float* weights, int64_t weights_coils,
                  float lamda, int num_iter, int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                  void* workspace, size_t workspace_bytes, dlcs_stream_t stream) {
    return sense_cg_impl(x, b, maps, weights, weights_coils, nullptr, 0, lamda, num_iter, B, E, C, T, Y, X,
                         workspace, workspace_bytes, stream);
}

int dlcs_sense_cg_rows(void* x, const void* b, const void* maps, const float* weights, int64_t weights_coils,
                       const void* table, int64_t jcap, float lamda, int num_iter,
                       int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                       void* workspace, size_t workspace_bytes, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(weights && table);
    return sense_cg_impl(x, b, maps, weights, weights_coils, table, jcap, lamda, num_iter, B, E, C, T, Y, X,
                         workspace, workspace_bytes, stream);
}

}  // extern "C"
