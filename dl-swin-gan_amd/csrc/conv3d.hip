// Conv3d(k=3, s=1, p=1) implicit-GEMM kernels on MFMA (gfx950): the ConvBlocks
// of s3d:225-273 (SFE 4->160, ResSwin tail 160->160, DFE tail 160->160, final
// 160->4), which carry ~92 % of the regularizer FLOPs.
//
// Activations live in the patch-blocked channels-last layout (see layout.hip):
//   row(b,t,y,x) = patch(b,t/4,y/4,x/4)*64 + (t%4)*16 + (y%4)*4 + x%4,  elem = row*ld + c
//
// Forward / dgrad kernel: one workgroup = 1x2x2 patches (4x8x8 = 256 output
// voxels) x all output channels; 4 waves, one patch (64 voxels = 2 M-tiles)
// each, NT 32-wide N-tiles.  K = 27 taps x Cin, walked as (32-channel chunk,
// tap): the 6x10x10 input halo of a chunk is staged once in LDS (ReLU of the
// pre-activation fused into the staging, s3d:256-259) and re-read for all 27
// taps; the [Cout][32] weight slice of each (chunk, tap) is double-buffered in
// LDS with register-staged prefetch.  Epilogue: bias, optional multiply by
// (mask > 0) (ReLU backward), optional scaled residual add (s3d:339-340,
// :368, :427), optional accumulate; bf16 or fp32 output.
// dgrad = the same kernel on weights packed transposed and tap-flipped.
//
// wgrad kernel: dW[tap][co][ci] += sum_v g[v][co] * act(x)[v + off(tap)][ci],
// one workgroup per (tap, voxel range), one wave per 32-row co tile, operands
// staged transposed (voxel-contiguous) in LDS, fp32 atomics per workgroup tile.
#include "dlcs_common.h"

#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>

namespace {

// Library-internal scratch (the producers' column-sum partials, the split-K / tail /
// slab partials of the f16x3 kernels): one buffer per (slot, device, stream), grown on
// demand and kept for the process (a stream's launches are ordered, so its buffers are
// never shared with a concurrent launch on another stream).  Sizes at the BASELINE
// slice, per stream: h3r split-K 69 MB, f16x3 weight-gradient slabs 88 MB, tail split
// 42 MB, thin weight gradient 21 MB, column sums < 3 MB.  They bypass torch's caching
// allocator: dlcs_scratch_bytes() reports them and dlcs_release_scratch() frees them
// (after a device synchronisation) for a caller that needs the memory back.  Growing a
// buffer synchronises its stream once (the old one may still be read); every size is
// reached on the first step, so a steady step never grows one.
enum ScratchSlot { kScrColsum, kScrH3r, kScrSplit2, kScrH3Tail, kScrWgH3, kScrTwp, kScrV6Tail, kScrBiasPart,
                   kScrSlots };
std::mutex g_scr_mu;
std::map<std::tuple<int, int, hipStream_t>, std::pair<void*, size_t>> g_scr;

void* scratch(int slot, hipStream_t st, size_t bytes) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_scr_mu);
    auto& e = g_scr[{slot, dev, st}];
    if (e.second < bytes) {
        if (e.first) {
            if (hipStreamSynchronize(st) != hipSuccess) return nullptr;
            (void)hipFree(e.first);
        }
        e.first = nullptr;
        e.second = 0;
        if (hipMalloc(&e.first, bytes) != hipSuccess) return nullptr;
        e.second = bytes;
    }
    return e.first;
}

constexpr int kHaloT = 6, kHaloY = 10, kHaloX = 10;
constexpr int kHalo = kHaloT * kHaloY * kHaloX;     // 600 voxels
constexpr int CK = 32;                              // channel chunk (K per tap step)

template <typename T> struct ConvPad;
template <> struct ConvPad<bf16> { static constexpr int v = 8; };
template <> struct ConvPad<float> { static constexpr int v = 4; };

DLCS_DEV long brow(int b, int t, int y, int x, int nT, int nY, int nX) {
    const long patch = (((long)b * nT + (t >> 2)) * nY + (y >> 2)) * nX + (x >> 2);
    return patch * 64 + ((t & 3) << 4) + ((y & 3) << 2) + (x & 3);
}

struct ConvArgs {
    const void* in; const void* w; const float* bias; void* out;
    const void* mask; const void* res;
    int B, D, H, W, Cin, cin_ld, cin_pad, Cout, cout_pad, cout_ld;
    int mask_ld, res_ld, relu_in, out_f32, res_f32, accumulate, relu_out;
    float res_scale;
};

template <typename T>
DLCS_DEV Frag8<T> relu8(Frag8<T> f) {
#pragma unroll
    for (int i = 0; i < 8; ++i) f.v[i] = (to_f(f.v[i]) > 0.0f) ? f.v[i] : from_f<T>(0.0f);
    return f;
}

template <typename T, int NT>
__global__ void __launch_bounds__(256) conv3d_k3_kernel(ConvArgs a) {
    constexpr int LD = CK + ConvPad<T>::v;
    constexpr int COP = NT * 32;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    T* Hs = reinterpret_cast<T*>(smem_raw);          // [600][LD]
    T* Ws = Hs + kHalo * LD;                          // [2][COP][LD]

    const int nT = a.D >> 2, nY = a.H >> 2, nX = a.W >> 2;
    const int nYt = (nY + 1) >> 1, nXt = (nX + 1) >> 1;
    int bid = blockIdx.x;
    const int txx = bid % nXt; bid /= nXt;
    const int tyy = bid % nYt; bid /= nYt;
    const int pt = bid % nT;
    const int b = bid / nT;
    const int t0 = pt * 4, y0 = tyy * 8, x0 = txx * 8;
    const T* in = reinterpret_cast<const T*>(a.in);
    const T* wt = reinterpret_cast<const T*>(a.w);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hh = lane >> 5;
    const int ncc = a.cin_pad / CK;
    const int nsteps = ncc * 27;

    auto stage_halo = [&](int cc) {
        for (int i = threadIdx.x; i < kHalo * (CK / 8); i += 256) {
            const int hv = i >> 2, c8 = (i & 3) * 8;
            const int ht = hv / (kHaloY * kHaloX), hy = (hv / kHaloX) % kHaloY, hx = hv % kHaloX;
            const int t = t0 - 1 + ht, y = y0 - 1 + hy, x = x0 - 1 + hx;
            const int c = cc * CK + c8;
            Frag8<T> f = zero8<T>();
            if (t >= 0 && t < a.D && y >= 0 && y < a.H && x >= 0 && x < a.W && c < a.Cin) {
                f = load8<T>(in + brow(b, t, y, x, nT, nY, nX) * a.cin_ld + c);
                if (a.relu_in) f = relu8<T>(f);
            }
            *reinterpret_cast<decltype(f.v)*>(Hs + hv * LD + c8) = f.v;
        }
    };
    // weight slice of step s: [COP][32] from packed [27][COP][cin_pad]
    constexpr int WCH = COP * (CK / 8);
    constexpr int WPER = (WCH + 255) / 256;
    Frag8<T> wr[WPER];
    auto load_w = [&](int s) {
        const int tap = s % 27, cc = s / 27;
#pragma unroll
        for (int k = 0; k < WPER; ++k) {
            const int i = threadIdx.x + k * 256;
            if (i < WCH) {
                const int co = i >> 2, c8 = (i & 3) * 8;
                wr[k] = load8<T>(wt + ((long)tap * COP + co) * a.cin_pad + cc * CK + c8);
            }
        }
    };
    auto store_w = [&](int buf) {
        T* dst = Ws + buf * COP * LD;
#pragma unroll
        for (int k = 0; k < WPER; ++k) {
            const int i = threadIdx.x + k * 256;
            if (i < WCH) {
                const int co = i >> 2, c8 = (i & 3) * 8;
                *reinterpret_cast<decltype(wr[k].v)*>(dst + co * LD + c8) = wr[k].v;
            }
        }
    };

    f32x16 acc[2][NT];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = (f32x16)0.0f;

    // halo rows of this lane's two voxels (tap (0,0,0) corner)
    const int pyy = wave >> 1, pxx = wave & 1;
    int hbase[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int v = i * 32 + (lane & 31);
        const int lt = v >> 4, ly = pyy * 4 + ((v >> 2) & 3), lx = pxx * 4 + (v & 3);
        hbase[i] = (lt * kHaloY + ly) * kHaloX + lx;
    }

    stage_halo(0);
    load_w(0);
    store_w(0);
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
        const int tap = s % 27;
        if (s + 1 < nsteps) load_w(s + 1);
        const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
        const int toff = (kd * kHaloY + kh) * kHaloX + kw;
        const T* wb = Ws + (s & 1) * COP * LD;
#pragma unroll
        for (int kk = 0; kk < CK / 16; ++kk) {
            const int kof = kk * 16 + 8 * hh;
            Frag8<T> af[2], bfr[NT];
#pragma unroll
            for (int i = 0; i < 2; ++i) af[i] = load8<T>(Hs + (hbase[i] + toff) * LD + kof);
#pragma unroll
            for (int j = 0; j < NT; ++j) bfr[j] = load8<T>(wb + (j * 32 + (lane & 31)) * LD + kof);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j) mfma32(acc[i][j], af[i], bfr[j]);
        }
        if (s + 1 < nsteps) {
            store_w((s + 1) & 1);
            if (tap == 26) {              // next step starts a new channel chunk
                __syncthreads();
                stage_halo((s + 1) / 27);
            }
        }
        __syncthreads();
    }

    // epilogue: this wave's patch
    const int py = tyy * 2 + pyy, px = txx * 2 + pxx;
    if (py >= nY || px >= nX) return;
    const long prow = (((long)b * nT + pt) * nY + py) * nX + px;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int co = j * 32 + (lane & 31);
        if (co >= a.Cout) continue;
        const float bias = a.bias ? a.bias[co] : 0.0f;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const long row = prow * 64 + i * 32 + acc_row(r, lane);
                float v = acc[i][j][r] + bias;
                if (a.mask) {
                    const float mv = to_f(reinterpret_cast<const T*>(a.mask)[row * a.mask_ld + co]);
                    v = (mv > 0.0f) ? v : 0.0f;
                }
                if (a.res) {
                    const float rv = a.res_f32 ? reinterpret_cast<const float*>(a.res)[row * a.res_ld + co]
                                               : to_f(reinterpret_cast<const T*>(a.res)[row * a.res_ld + co]);
                    v += a.res_scale * rv;
                }
                if (a.relu_out) v = fmaxf(v, 0.0f);
                const long oi = row * a.cout_ld + co;
                if (a.out_f32) {
                    float* o = reinterpret_cast<float*>(a.out);
                    o[oi] = a.accumulate ? o[oi] + v : v;
                } else {
                    T* o = reinterpret_cast<T*>(a.out);
                    o[oi] = from_f<T>(a.accumulate ? to_f(o[oi]) + v : v);
                }
            }
        }
    }
}

// ---------------------------------------------------------------- forward / dgrad v2 (bf16)
// 512 threads = 8 waves; workgroup tile = 1x2x2 patches (256 voxels) x 160
// output channels.  Wave w: patch (w & 3) x output-channel half (w >> 2, 80 =
// 5 x 16), v_mfma_f32_16x16x32_bf16, 4 M-tiles x 5 N-tiles per wave.  K is
// walked per 32-channel chunk (halo restaged 5 times, next chunk prefetched
// into registers 6 steps ahead) x 9 steps of 3 taps (kd, kh fixed, kw = 0..2):
// one barrier per 3 taps (60 MFMAs per wave), the next step's 3 weight slices
// register-prefetched while the current step computes.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

DLCS_DEV void mfma16(f32x4_t& acc, const bf16x8_t& a, const bf16x8_t& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
}

struct ConvV2Args {
    const bf16* in; const bf16* w; const float* bias; void* out;
    const bf16* mask; const void* res;
    int B, D, H, W, cin_ld, cin_pad;
    int cout_ld, mask_ld, res_ld, out_f32, res_f32, accumulate, relu_out;
    float res_scale;
    int xcd_major;          // v5: number tiles XCD-major (neighbouring halos in one L2)
};

// Epilogue of a 256-voxel x 160-channel tile held by 8 waves as acc[4][5]
// (wave: voxel quarter pw = patch of the 1x2x2 tile, channel half nh; C/D
// rows = voxels, cols = channels).  The fp32 tile goes through LDS (Es, >=
// 256 x (160 / NPASS + 4) floats) in NPASS channel slices, then every thread
// finishes 16-B chunks (8 channels of one voxel row): bias, ReLU-backward mask
// (s3d:256-259), scaled residual, ReLU, optional accumulate -- one 16-B load /
// store per operand.
template <int NPASS>
DLCS_DEV void conv_epilogue_256x160(const ConvV2Args& a, const f32x4_t (&acc)[4][5], float* Es, int pw, int nh,
                                    int lane, int b, int pt, int pyq, int pxq, int nT, int nY, int nX) {
    constexpr int PC = 160 / NPASS, EL = PC + 4, NCH = PC / 8;
    static_assert(PC % 16 == 0, "pass width must be whole 16-channel tiles");
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int c0 = (nh * 5 + j) * 16 - pass * PC;
            if (c0 >= 0 && c0 < PC) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int vl = pw * 64 + i * 16 + (lane >> 4) * 4 + r;
                        Es[vl * EL + c0 + (lane & 15)] = acc[i][j][r];
                    }
            }
        }
        __syncthreads();
        for (int c = threadIdx.x; c < 256 * NCH; c += 512) {
            const int vl = c / NCH, ch = (c % NCH) * 8;
            const int pwv = vl >> 6;
            const int py = pyq + (pwv >> 1), px = pxq + (pwv & 1);
            if (py >= nY || px >= nX) continue;
            const long row = ((((long)b * nT + pt) * nY + py) * nX + px) * 64 + (vl & 63);
            const int co = pass * PC + ch;
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = Es[vl * EL + ch + e] + (a.bias ? a.bias[co + e] : 0.0f);
            if (a.mask) {
                const bf16x8_t m = *reinterpret_cast<const bf16x8_t*>(a.mask + row * a.mask_ld + co);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = ((float)m[e] > 0.0f) ? v[e] : 0.0f;
            }
            if (a.res) {
                if (a.res_f32) {
                    const float* rp = reinterpret_cast<const float*>(a.res) + row * a.res_ld + co;
                    const f32x4_t r0 = *reinterpret_cast<const f32x4_t*>(rp);
                    const f32x4_t r1 = *reinterpret_cast<const f32x4_t*>(rp + 4);
#pragma unroll
                    for (int e = 0; e < 4; ++e) { v[e] += a.res_scale * r0[e]; v[4 + e] += a.res_scale * r1[e]; }
                } else {
                    const bf16x8_t rr = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const bf16*>(a.res) + row * a.res_ld + co);
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += a.res_scale * (float)rr[e];
                }
            }
            if (a.relu_out) {
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.0f);
            }
            const long oi = row * a.cout_ld + co;
            if (a.out_f32) {
                float* o = reinterpret_cast<float*>(a.out) + oi;
                f32x4_t o0, o1;
#pragma unroll
                for (int e = 0; e < 4; ++e) { o0[e] = v[e]; o1[e] = v[4 + e]; }
                if (a.accumulate) { o0 += *reinterpret_cast<const f32x4_t*>(o); o1 += *reinterpret_cast<const f32x4_t*>(o + 4); }
                *reinterpret_cast<f32x4_t*>(o) = o0;
                *reinterpret_cast<f32x4_t*>(o + 4) = o1;
            } else {
                bf16* o = reinterpret_cast<bf16*>(a.out) + oi;
                bf16x8_t ov;
                if (a.accumulate) {
                    const bf16x8_t prev = *reinterpret_cast<const bf16x8_t*>(o);
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += (float)prev[e];
                }
#pragma unroll
                for (int e = 0; e < 8; ++e) ov[e] = (bf16)v[e];
                *reinterpret_cast<bf16x8_t*>(o) = ov;
            }
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(512) conv3d_k3_v2_kernel(ConvV2Args a) {
    // LDS images use 64-B rows (32 bf16 channels) with the four 16-B chunks of a
    // row XOR-swizzled so every ds_read_b128 lane group hits 16 distinct bank
    // quads (checked exhaustively for all tap offsets):
    //   halo row (hy = its halo y):  chunk c at c ^ (2 * (hy & 1))
    //   weight row co:               chunk c at c ^ ((4 - ((co & 15) >> 2)) & 3)
    constexpr int LD = 32;
    constexpr int CO = 160;
    __shared__ __attribute__((aligned(16))) bf16 smem_v2[kHalo * LD + 2 * 3 * CO * LD];   // 38.4 + 61.4 KB
    bf16* Hs = smem_v2;
    bf16* Ws = smem_v2 + kHalo * LD;

    const int nT = a.D >> 2, nY = a.H >> 2, nX = a.W >> 2;
    const int nYt = (nY + 1) >> 1, nXt = (nX + 1) >> 1;
    int bid = blockIdx.x;
    const int txx = bid % nXt; bid /= nXt;
    const int tyy = bid % nYt; bid /= nYt;
    const int pt = bid % nT;
    const int b = bid / nT;
    const int t0 = pt * 4, y0 = tyy * 8, x0 = txx * 8;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int pw = wave & 3, nh = wave >> 2;
    const int ncc = a.cin_pad / CK;
    const int nsteps = ncc * 9;

    constexpr int HPER = (kHalo * 4 + 511) / 512;          // 5
    bf16x8_t hr[HPER];
    auto load_halo = [&](int cc) {
#pragma unroll
        for (int k = 0; k < HPER; ++k) {
            const int i = threadIdx.x + k * 512;
            hr[k] = (bf16x8_t)(bf16)0.0f;
            if (i < kHalo * 4) {
                const int hv = i >> 2, c8 = (i & 3) * 8;
                const int ht = hv / (kHaloY * kHaloX), hy = (hv / kHaloX) % kHaloY, hx = hv % kHaloX;
                const int t = t0 - 1 + ht, y = y0 - 1 + hy, x = x0 - 1 + hx;
                if (t >= 0 && t < a.D && y >= 0 && y < a.H && x >= 0 && x < a.W)
                    hr[k] = *reinterpret_cast<const bf16x8_t*>(a.in + brow(b, t, y, x, nT, nY, nX) * a.cin_ld + cc * CK + c8);
            }
        }
    };
    auto store_halo = [&]() {
#pragma unroll
        for (int k = 0; k < HPER; ++k) {
            const int i = threadIdx.x + k * 512;
            if (i < kHalo * 4) {
                const int hv = i >> 2, c = i & 3;
                const int hy = (hv / kHaloX) % kHaloY;
                *reinterpret_cast<bf16x8_t*>(Hs + hv * LD + ((c ^ ((hy & 1) << 1)) << 3)) = hr[k];
            }
        }
    };
    constexpr int WPER = (3 * CO * 4 + 511) / 512;         // 4
    bf16x8_t wr[WPER];
    auto load_w = [&](int s) {
        const int cc = s / 9, t3 = (s % 9) * 3;
#pragma unroll
        for (int k = 0; k < WPER; ++k) {
            const int i = threadIdx.x + k * 512;
            if (i < 3 * CO * 4) {
                const int tl = i / (CO * 4), co = (i >> 2) % CO, c8 = (i & 3) * 8;
                wr[k] = *reinterpret_cast<const bf16x8_t*>(a.w + ((long)(t3 + tl) * CO + co) * a.cin_pad + cc * CK + c8);
            }
        }
    };
    auto store_w = [&](int buf) {
        bf16* dst = Ws + buf * 3 * CO * LD;
#pragma unroll
        for (int k = 0; k < WPER; ++k) {
            const int i = threadIdx.x + k * 512;
            if (i < 3 * CO * 4) {
                const int row = i >> 2, c = i & 3, co = row % CO;
                const int pos = c ^ ((4 - ((co & 15) >> 2)) & 3);
                *reinterpret_cast<bf16x8_t*>(dst + row * LD + (pos << 3)) = wr[k];
            }
        }
    };

    f32x4_t acc[4][5];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) acc[i][j] = (f32x4_t)0.0f;

    const int pyy = pw >> 1, pxx = pw & 1;
    const int vq = lane & 15, cq = lane >> 4;
    const int ly = pyy * 4 + ((vq >> 2) & 3), lx = pxx * 4 + (vq & 3);
    int hbase[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) hbase[i] = (i * kHaloY + ly) * kHaloX + lx;
    const int corow = nh * 80 + vq;
    const int bpos = (cq ^ ((4 - (vq >> 2)) & 3)) << 3;               // weight chunk position (elements)

    load_halo(0);
    store_halo();
    load_w(0);
    store_w(0);
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
        const int st = s % 9;
        if (s + 1 < nsteps) load_w(s + 1);
        if (st == 1 && s / 9 + 1 < ncc) load_halo(s / 9 + 1);
        const int kd = st / 3, kh = st % 3;
        const int apos = (cq ^ (((ly + kh) & 1) << 1)) << 3;         // halo chunk position (elements)
        const bf16* wb = Ws + (s & 1) * 3 * CO * LD;
        // fragments of tap kw+1 are read while the MFMAs of tap kw run
        bf16x8_t afA[4], bfA[5], afB[4], bfB[5];
        auto read_frags = [&](int kw, bf16x8_t (&af)[4], bf16x8_t (&bfr)[5]) {
            const int toff = (kd * kHaloY + kh) * kHaloX + kw;
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8_t*>(Hs + (hbase[i] + toff) * LD + apos);
#pragma unroll
            for (int j = 0; j < 5; ++j)
                bfr[j] = *reinterpret_cast<const bf16x8_t*>(wb + (kw * CO + corow + j * 16) * LD + bpos);
        };
        auto mma = [&](const bf16x8_t (&af)[4], const bf16x8_t (&bfr)[5]) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 5; ++j) mfma16(acc[i][j], af[i], bfr[j]);
        };
        read_frags(0, afA, bfA);
        read_frags(1, afB, bfB);
        mma(afA, bfA);
        read_frags(2, afA, bfA);
        mma(afB, bfB);
        mma(afA, bfA);
        if (s + 1 < nsteps) {
            store_w((s + 1) & 1);
            if (st == 8) {                      // next step opens a new channel chunk
                __syncthreads();
                store_halo();
            }
        }
        __syncthreads();
    }

    // ---- epilogue (shares the LDS of the main loop)
    conv_epilogue_256x160<2>(a, acc, reinterpret_cast<float*>(Hs), pw, nh, lane, b, pt, tyy * 2, txx * 2, nT, nY, nX);
}

// ---------------------------------------------------------------- forward / dgrad, thin input (bf16)
// Cin <= 4 -> 160: the SFE conv (s3d:384) and the dgrad of the final conv
// (s3d:391).  K = 27 taps x 4 channels (taps padded to 32, zero weights): a
// lane's 8 consecutive k are 2 taps x 4 channels of one voxel, i.e. two 8-B
// reads of the [6][10][10] x 16-B halo -- no im2col image.  The [160][128]
// weight image stays in LDS for the whole (persistent) workgroup; tiles and
// waves as in the v2 kernel, epilogue in 5 passes of 32 channels (80 KB of
// LDS; at ~210 VGPRs the kernel runs one 8-wave workgroup per CU).
template <int EPI, int NTHR, int NCO, int NPASS>
DLCS_DEV void conv_epilogue_spec(const ConvV2Args& a, const f32x4_t (&acc)[4][5], float* Es, int pw, int cw0,
                                 int co0, int lane, int b, int pt, int pyq, int pxq, int nT, int nY, int nX);
extern __device__ uint4 g_wg_zero_row[];

// The next tile's halo is register-prefetched (pointer-selected zero row for
// off-grid voxels: no guarded loads) while the current tile runs its MFMAs and
// epilogue, and the epilogue is the operand-specialised one of the v5 kernel
// (every mask / residual load of a slice in flight before its LDS round trip).
template <int EPI>
__global__ void __launch_bounds__(512) conv3d_thin_in_kernel(ConvV2Args a, int ntiles) {
    constexpr int WLD = 136;                              // 128 + 8: conflict-free B reads
    __shared__ __attribute__((aligned(16))) char smem[160 * WLD * 2 + 256 * 36 * 4];
    bf16* Wt = reinterpret_cast<bf16*>(smem);
    bf16* Hs = reinterpret_cast<bf16*>(smem + 160 * WLD * 2);     // [600][8]
    float* Es = reinterpret_cast<float*>(smem + 160 * WLD * 2);   // epilogue (halo is dead by then)
    for (int it = threadIdx.x; it < 160 * 32; it += 512) {
        const int co = it >> 5, tap = it & 31;
        uint2 v = make_uint2(0, 0);
        if (tap < 27) v = *reinterpret_cast<const uint2*>(a.w + ((long)tap * 160 + co) * a.cin_pad);
        *reinterpret_cast<uint2*>(Wt + co * WLD + tap * 4) = v;
    }
    const int nT = a.D >> 2, nY = a.H >> 2, nX = a.W >> 2;
    const int nYt = (nY + 1) >> 1, nXt = (nX + 1) >> 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int pw = wave & 3, nh = wave >> 2;
    const int vq = lane & 15, cq = lane >> 4;
    const int ly = (pw >> 1) * 4 + ((vq >> 2) & 3), lx = (pw & 1) * 4 + (vq & 3);
    // the two taps of this lane in k-step s: 8 s + 2 cq + {0, 1} (clamped; weights are 0)
    auto toff = [](int tap) {
        tap = tap < 27 ? tap : 26;
        return ((tap / 9) * kHaloY + (tap / 3) % 3) * kHaloX + tap % 3;
    };
    auto decode = [&](int tile, int& b, int& pt, int& tyy, int& txx) {
        int bid = tile;
        txx = bid % nXt; bid /= nXt;
        tyy = bid % nYt; bid /= nYt;
        pt = bid % nT;
        b = bid / nT;
    };
    static_assert((kHalo + 511) / 512 == 2, "two halo pieces per thread");
    // the next tile's halo rows in two named registers (an array captured by a lambda
    // was placed in scratch: a private-memory round trip per tile)
    uint4 hreg0 = make_uint4(0, 0, 0, 0), hreg1 = make_uint4(0, 0, 0, 0);
    const uint4* zrow = g_wg_zero_row;
    auto halo_src = [&](int tile, int k) {
        int b, pt, tyy, txx;
        decode(tile, b, pt, tyy, txx);
        const int hv = threadIdx.x + 512 * k;
        const int ht = hv / (kHaloY * kHaloX), hy = (hv / kHaloX) % kHaloY, hx = hv % kHaloX;
        const int t = pt * 4 - 1 + ht, y = tyy * 8 - 1 + hy, x = txx * 8 - 1 + hx;
        const bool ok = hv < kHalo && t >= 0 && t < a.D && y >= 0 && y < a.H && x >= 0 && x < a.W;
        return ok ? reinterpret_cast<const uint4*>(a.in + brow(b, t, y, x, nT, nY, nX) * a.cin_ld) : zrow;
    };
    int tile = blockIdx.x;
    if (tile < ntiles) {
        hreg0 = *halo_src(tile, 0);
        hreg1 = *halo_src(tile, 1);
    }
    for (; tile < ntiles; tile += gridDim.x) {
        int b, pt, tyy, txx;
        decode(tile, b, pt, tyy, txx);
        *reinterpret_cast<uint4*>(Hs + threadIdx.x * 8) = hreg0;
        if (threadIdx.x + 512 < kHalo) *reinterpret_cast<uint4*>(Hs + (threadIdx.x + 512) * 8) = hreg1;
        __syncthreads();
        if (tile + (int)gridDim.x < ntiles) {
            hreg0 = *halo_src(tile + gridDim.x, 0);
            hreg1 = *halo_src(tile + gridDim.x, 1);
        }
        f32x4_t acc[4][5];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 5; ++j) acc[i][j] = (f32x4_t)0.0f;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int oA = toff(8 * s + 2 * cq), oB = toff(8 * s + 2 * cq + 1);
            bf16x8_t af[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int hb = (i * kHaloY + ly) * kHaloX + lx;
                const uint2 lo = *reinterpret_cast<const uint2*>(Hs + (hb + oA) * 8);
                const uint2 hi = *reinterpret_cast<const uint2*>(Hs + (hb + oB) * 8);
                const uint4 both = make_uint4(lo.x, lo.y, hi.x, hi.y);
                af[i] = __builtin_bit_cast(bf16x8_t, both);
            }
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const bf16x8_t bfr = *reinterpret_cast<const bf16x8_t*>(Wt + (nh * 80 + j * 16 + vq) * WLD + 32 * s + 8 * cq);
#pragma unroll
                for (int i = 0; i < 4; ++i) mfma16(acc[i][j], af[i], bfr);
            }
        }
        __syncthreads();
        conv_epilogue_spec<EPI, 512, 160, 5>(a, acc, Es, pw, nh * 80, 0, lane, b, pt, tyy * 2, txx * 2, nT, nY, nX);
    }
}

// ---------------------------------------------------------------- forward / dgrad, thin output (bf16)
// 160 -> Cout <= 4: the final conv (s3d:391) and the dgrad of the SFE conv
// (s3d:384).  Shifting the output instead of the input:
//   out[v][co] = sum_tap P[v + off(tap)][tap][co],  P[u][tap][co] = sum_ci W[tap][co][ci] x[u][ci]
// so each x row is multiplied once (a [216 halo voxels] x [160] x [112 = 27 taps
// x 4 co] GEMM per 64-voxel patch, A fragments loaded straight from global)
// instead of once per tap.  P (fp32) lives in LDS; 64 lanes then gather the 27
// tap partials of each output voxel.  7 waves = 7 pairs of 16-row M tiles;
// persistent over patches with the next patch's A fragments prefetched.
__global__ void __launch_bounds__(448) conv3d_thin_out_kernel(ConvArgs a, int npatch) {
    constexpr int WLD = 168, PLD = 116;
    __shared__ __attribute__((aligned(16))) char smem[112 * WLD * 2 + 224 * PLD * 4];
    bf16* Wt = reinterpret_cast<bf16*>(smem);                        // [112 (tap, co)][160 ci (+8)]
    float* P = reinterpret_cast<float*>(smem + 112 * WLD * 2);        // [224 halo rows][112 (+4)]
    const bf16* in = reinterpret_cast<const bf16*>(a.in);
    const bf16* wp = reinterpret_cast<const bf16*>(a.w);
    for (int it = threadIdx.x; it < 112 * 20; it += 448) {
        const int n = it / 20, c8 = (it % 20) * 8;
        const int tap = n >> 2, co = n & 3;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (tap < 27 && co < a.Cout) v = *reinterpret_cast<const uint4*>(wp + ((long)tap * a.cout_pad + co) * a.cin_pad + c8);
        *reinterpret_cast<uint4*>(Wt + n * WLD + c8) = v;
    }
    const int nT = a.D >> 2, nY = a.H >> 2, nX = a.W >> 2;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int vq = lane & 15, cq = lane >> 4;

    bf16x8_t af[2][5];
    auto load_a = [&](int patch) {
        const int px = patch % nX;
        int r = patch / nX;
        const int py = r % nY; r /= nY;
        const int pt = r % nT;
        const int bb = r / nT;
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const int hr = (2 * wave + m) * 16 + vq;
            const int hz = hr / 36, hy = (hr / 6) % 6, hx = hr % 6;
            const int T = pt * 4 + hz - 1, Y = py * 4 + hy - 1, X = px * 4 + hx - 1;
            const bool ok = hr < 216 && (unsigned)T < (unsigned)a.D && (unsigned)Y < (unsigned)a.H && (unsigned)X < (unsigned)a.W;
            const bf16* src = in + (ok ? brow(bb, T, Y, X, nT, nY, nX) * a.cin_ld : 0) + 8 * cq;
#pragma unroll
            for (int s = 0; s < 5; ++s)
                af[m][s] = ok ? *reinterpret_cast<const bf16x8_t*>(src + 32 * s) : (bf16x8_t)(bf16)0.0f;
        }
    };
    int patch = blockIdx.x;
    if (patch < npatch) load_a(patch);
    __syncthreads();
    for (; patch < npatch; patch += gridDim.x) {
        f32x4_t acc[2][7];
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int j = 0; j < 7; ++j) acc[m][j] = (f32x4_t)0.0f;
#pragma unroll
        for (int s = 0; s < 5; ++s)
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                const bf16x8_t bfr = *reinterpret_cast<const bf16x8_t*>(Wt + (j * 16 + vq) * WLD + 32 * s + 8 * cq);
                mfma16(acc[0][j], af[0][s], bfr);
                mfma16(acc[1][j], af[1][s], bfr);
            }
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int j = 0; j < 7; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    P[((2 * wave + m) * 16 + cq * 4 + r) * PLD + j * 16 + vq] = acc[m][j][r];
        if (patch + (int)gridDim.x < npatch) load_a(patch + gridDim.x);
        __syncthreads();
        if (wave == 0) {
            const int t = lane >> 4, y = (lane >> 2) & 3, x = lane & 3;
            f32x4_t sum = (f32x4_t)0.0f;
#pragma unroll
            for (int tap = 0; tap < 27; ++tap) {
                const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
                const int row = ((t + kd) * 6 + (y + kh)) * 6 + (x + kw);
                sum += *reinterpret_cast<const f32x4_t*>(P + row * PLD + tap * 4);
            }
            const long orow = (long)patch * 64 + lane;
            if (a.bias) {
#pragma unroll
                for (int c = 0; c < 4; ++c) sum[c] += (c < a.Cout) ? a.bias[c] : 0.0f;
            }
            if (a.out_f32) {
                float* o = reinterpret_cast<float*>(a.out) + orow * a.cout_ld;
                if (a.Cout == 4) *reinterpret_cast<f32x4_t*>(o) = sum;
                else for (int c = 0; c < a.Cout; ++c) o[c] = sum[c];
            } else {
                bf16* o = reinterpret_cast<bf16*>(a.out) + orow * a.cout_ld;
                for (int c = 0; c < a.Cout; ++c) o[c] = (bf16)sum[c];
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- wgrad
struct WgradArgs {
    const void* in; const void* g; float* dw;
    int B, D, H, W, Cin, cin_ld, cin_pad, Cout, g_ld, cout_pad, relu_in;
    long vox_per_block;
    float* dbias;           // optional: += column sums of g (the conv bias gradient)
};

template <typename T, int NT>
__global__ void __launch_bounds__(320) conv3d_wgrad_kernel(WgradArgs a) {
    // waves = cout_pad / 32 (<= 5); each wave: 1 co tile x NT ci tiles
    constexpr int KV = 32;                         // voxels per K step
    constexpr int LD = KV + ConvPad<T>::v;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const int MT = a.cout_pad / 32;
    T* Gs = reinterpret_cast<T*>(smem_raw);        // [cout_pad][LD]  (co rows, voxel-contiguous)
    T* Is = Gs + a.cout_pad * LD;                   // [NT*32][LD]     (ci rows)
    const int nT = a.D >> 2, nY = a.H >> 2, nX = a.W >> 2;
    const long nvox = (long)a.B * a.D * a.H * a.W;
    const int tap = blockIdx.y;
    const int kd = tap / 9 - 1, kh = (tap / 3) % 3 - 1, kw = tap % 3 - 1;
    const long v0 = (long)blockIdx.x * a.vox_per_block;
    const long v1 = min(nvox, v0 + a.vox_per_block);
    const T* in = reinterpret_cast<const T*>(a.in);
    const T* g = reinterpret_cast<const T*>(a.g);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hh = lane >> 5;
    const int nthr = blockDim.x;

    f32x16 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = (f32x16)0.0f;

    for (long vb = v0; vb < v1; vb += KV) {
        __syncthreads();
        // stage g rows [KV][cout] -> Gs[co][v] and neighbour input rows -> Is[ci][v]
        const int gch = KV * (a.cout_pad / 8);
        for (int i = threadIdx.x; i < gch; i += nthr) {
            const int vl = i / (a.cout_pad / 8), c8 = (i % (a.cout_pad / 8)) * 8;
            const long row = vb + vl;
            Frag8<T> f = zero8<T>();
            if (row < v1 && c8 < a.Cout) f = load8<T>(g + row * a.g_ld + c8);
#pragma unroll
            for (int e = 0; e < 8; ++e) Gs[(c8 + e) * LD + vl] = (c8 + e < a.Cout) ? f.v[e] : from_f<T>(0.0f);
        }
        const int ich = KV * (NT * 32 / 8);
        for (int i = threadIdx.x; i < ich; i += nthr) {
            const int vl = i / (NT * 32 / 8), c8 = (i % (NT * 32 / 8)) * 8;
            const long row = vb + vl;
            Frag8<T> f = zero8<T>();
            if (row < v1 && c8 < a.Cin) {
                // decode the blocked output row, step to the tap neighbour
                const long patch = row >> 6;
                const int ip = (int)(row & 63);
                const int px = (int)(patch % nX), py = (int)((patch / nX) % nY), pt = (int)((patch / ((long)nX * nY)) % nT);
                const int bb = (int)(patch / ((long)nX * nY * nT));
                const int t = pt * 4 + (ip >> 4) + kd, y = py * 4 + ((ip >> 2) & 3) + kh, x = px * 4 + (ip & 3) + kw;
                if (t >= 0 && t < a.D && y >= 0 && y < a.H && x >= 0 && x < a.W) {
                    f = load8<T>(in + brow(bb, t, y, x, nT, nY, nX) * a.cin_ld + c8);
                    if (a.relu_in) f = relu8<T>(f);
                }
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) Is[(c8 + e) * LD + vl] = (c8 + e < a.Cin) ? f.v[e] : from_f<T>(0.0f);
        }
        __syncthreads();
        if (wave < MT) {
#pragma unroll
            for (int kk = 0; kk < KV / 16; ++kk) {
                const int kof = kk * 16 + 8 * hh;
                const Frag8<T> af = load8<T>(Gs + (wave * 32 + (lane & 31)) * LD + kof);
#pragma unroll
                for (int j = 0; j < NT; ++j) {
                    const Frag8<T> bfr = load8<T>(Is + (j * 32 + (lane & 31)) * LD + kof);
                    mfma32(acc[j], af, bfr);
                }
            }
        }
    }
    if (wave >= MT) return;
    // dw packed [27][cout_pad][cin_pad] fp32
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int ci = j * 32 + (lane & 31);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int co = wave * 32 + acc_row(r, lane);
            atomicAdd(a.dw + ((long)tap * a.cout_pad + co) * a.cin_pad + ci, acc[j][r]);
        }
    }
}

// ---------------------------------------------------------------- wgrad (bf16 fast path)
// One workgroup = (tap, voxel range); the 27 taps of a range are placed on the
// same XCD group (blockIdx % 8) so the shifted re-reads of g and x hit L2.
// K = voxels, walked one 64-voxel patch at a time: g rows [64][co_pad] and the
// tap-shifted x rows [64][ci_pad] are staged in LDS in their natural
// (channel-contiguous) layout from register-prefetched 16-B loads, and read
// back voxel-contiguous with ds_read_b64_tr_b16 (lane = channel, 4 voxels per
// read) as the MFMA operands -- no scattered transposing writes.  Row stride
// 160 / 32 bf16 (80 / 16 dwords) keeps the transposed reads conflict-free.
typedef short v4s __attribute__((ext_vector_type(4)));

DLCS_DEV Frag8<bf16> tr_frag(const bf16* base, int ld, int lane) {
    // lane l: 16-lane group g = l>>4 covers channels 16*(g&1)..+15 and voxels 8*(g>>1)..+7
    const int g = lane >> 4, i = lane & 15;
    const int q = i >> 2, p = i & 3;
    const int ch = 16 * (g & 1) + 4 * p;
    const int v = 8 * (g >> 1) + q;
    typedef __attribute__((address_space(3))) v4s lds_v4s;
    const bf16* a0 = base + v * ld + ch;
    const bf16* a1 = base + (v + 4) * ld + ch;
    v4s r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(const_cast<bf16*>(a0)));
    v4s r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(const_cast<bf16*>(a1)));
    typedef short v8s __attribute__((ext_vector_type(8)));
    const v8s both = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3]};
    Frag8<bf16> f;
    f.v = __builtin_bit_cast(bf16x8, both);
    return f;
}

template <int MT, int NT>
__global__ void __launch_bounds__(320) conv3d_wgrad_tr_kernel(WgradArgs a, int nrange, long patches_per_range) {
    constexpr int WAVES = 5;
    constexpr int COP = MT * 32, CIP = NT * 32;
    constexpr int PERW = (MT == 1) ? 1 : NT;             // ci tiles per wave
    constexpr int GCH = 64 * COP / 8, XCH = 64 * CIP / 8;
    constexpr int PER = (GCH + XCH + WAVES * 64 - 1) / (WAVES * 64);
    __shared__ __attribute__((aligned(16))) bf16 Gs[64 * COP];
    __shared__ __attribute__((aligned(16))) bf16 Xs[64 * CIP];

    // XCD-aware (range, tap) decode: blocks b with equal b % 8 share an XCD
    const int b = blockIdx.x, xg = b & 7, slot = b >> 3;
    const int range = xg + 8 * (slot / 27), tap = slot % 27;
    if (range >= nrange) return;
    const int kd = tap / 9 - 1, kh = (tap / 3) % 3 - 1, kw = tap % 3 - 1;
    const int nT = a.D >> 2, nY = a.H >> 2, nX = a.W >> 2;
    const long npatch = (long)a.B * nT * nY * nX;
    const long p0 = (long)range * patches_per_range;
    const long p1 = min(npatch, p0 + patches_per_range);
    const bf16* in = reinterpret_cast<const bf16*>(a.in);
    const bf16* g = reinterpret_cast<const bf16*>(a.g);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

    f32x16 acc[PERW];
#pragma unroll
    for (int j = 0; j < PERW; ++j) acc[j] = (f32x16)0.0f;

    Frag8<bf16> rr[PER];
    auto load_chunk = [&](long patch) {
        const int px = (int)(patch % nX), py = (int)((patch / nX) % nY), pt = (int)((patch / ((long)nX * nY)) % nT);
        const int bb = (int)(patch / ((long)nX * nY * nT));
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int c = threadIdx.x + k * WAVES * 64;
            rr[k] = zero8<bf16>();
            if (c < GCH) {
                const int vl = c / (COP / 8), c8 = (c % (COP / 8)) * 8;
                if (c8 < a.Cout) rr[k] = load8<bf16>(g + (patch * 64 + vl) * a.g_ld + c8);
            } else if (c < GCH + XCH) {
                const int cx = c - GCH;
                const int vl = cx / (CIP / 8), c8 = (cx % (CIP / 8)) * 8;
                const int t = pt * 4 + (vl >> 4) + kd, y = py * 4 + ((vl >> 2) & 3) + kh, x = px * 4 + (vl & 3) + kw;
                if (c8 < a.Cin && t >= 0 && t < a.D && y >= 0 && y < a.H && x >= 0 && x < a.W) {
                    rr[k] = load8<bf16>(in + brow(bb, t, y, x, nT, nY, nX) * a.cin_ld + c8);
                    if (a.relu_in) rr[k] = relu8<bf16>(rr[k]);
                }
            }
        }
    };
    auto store_chunk = [&]() {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int c = threadIdx.x + k * WAVES * 64;
            if (c < GCH) {
                const int vl = c / (COP / 8), c8 = (c % (COP / 8)) * 8;
                Frag8<bf16> f = rr[k];
#pragma unroll
                for (int e = 0; e < 8; ++e) if (c8 + e >= a.Cout) f.v[e] = (bf16)0.0f;
                *reinterpret_cast<bf16x8*>(Gs + vl * COP + c8) = f.v;
            } else if (c < GCH + XCH) {
                const int cx = c - GCH;
                const int vl = cx / (CIP / 8), c8 = (cx % (CIP / 8)) * 8;
                Frag8<bf16> f = rr[k];
#pragma unroll
                for (int e = 0; e < 8; ++e) if (c8 + e >= a.Cin) f.v[e] = (bf16)0.0f;
                *reinterpret_cast<bf16x8*>(Xs + vl * CIP + c8) = f.v;
            }
        }
    };

    if (p0 < p1) load_chunk(p0);
    for (long patch = p0; patch < p1; ++patch) {
        __syncthreads();
        store_chunk();
        __syncthreads();
        if (patch + 1 < p1) load_chunk(patch + 1);
        const int mt = (MT == 1) ? 0 : wave;             // co tile of this wave
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {                // 4 x 16 voxels
            const Frag8<bf16> af = tr_frag(Gs + kk * 16 * COP + mt * 32, COP, lane);
#pragma unroll
            for (int j = 0; j < PERW; ++j) {
                const int nt = (MT == 1) ? wave : j;
                const Frag8<bf16> bfr = tr_frag(Xs + kk * 16 * CIP + nt * 32, CIP, lane);
                mfma32(acc[j], af, bfr);
            }
        }
    }
    // flush: dw packed [27][co_pad][ci_pad]
    const int mt = (MT == 1) ? 0 : wave;
#pragma unroll
    for (int j = 0; j < PERW; ++j) {
        const int nt = (MT == 1) ? wave : j;
        const int ci = nt * 32 + (lane & 31);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int co = mt * 32 + acc_row(r, lane);
            atomicAdd(a.dw + ((long)tap * COP + co) * CIP + ci, acc[j][r]);
        }
    }
}

// ---------------------------------------------------------------- wgrad, 160 -> 160 (bf16)
// One workgroup = tap row (kd, kh) x voxel range; its 12 waves = 3 kw taps x
// 2 co halves x 2 ci halves, each owning an 80 x 80 block of dW[tap] (5 x 5
// 16x16x32 MFMA tiles, 100 fp32 accumulators per lane).  Per 64-voxel patch the
// g rows [64][160] and the tap row's x halo [4 t][4 y][6 x][160] -- shared by
// the 3 kw taps, so a patch costs 50 KB of loads instead of 3 x 40 KB -- are
// DMA'd global -> LDS with global_load_lds_dwordx4 (no VGPR staging) into one of
// two buffers while the other is multiplied, one barrier per patch.  Operands
// are read voxel-contiguous with ds_read_b64_tr_b16; the 16-channel tiles of a
// row are XOR-swizzled by bit 1 of the patch-local y so that the two 16-lane
// groups of a read (voxel rows 8 apart) hit disjoint banks.  The 9 tap rows of
// a voxel range run on one XCD (blockIdx % 8) at the same pace, so 8 of every
// 9 loads of a patch are L2 hits.
constexpr int kWgC = 160;
constexpr int kWgRows = 64 + 96;                       // g rows + halo rows per patch
constexpr int kWgChunks = kWgRows * kWgC / 8;          // 3200 16-B chunks
constexpr int kWgBuf = kWgRows * kWgC;                 // bf16 per LDS buffer (51200 B)
constexpr int kWgRangesPerXcd = 3;                     // 27 of the XCD's 32 CUs busy

__device__ uint4 g_wg_zero_row[kWgC / 8];  // zero source rows (halo voxels off the grid)              // zero source for halo rows off the grid

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
typedef __attribute__((address_space(3))) v4s lds_v4s_t;

// global -> LDS DMA of 16 B per lane to (wave-uniform lds_addr) + 16 * lane.
// Issued from inline asm on purpose: hipcc cannot tell which LDS buffer a
// builtin DMA writes and waits vmcnt(0) before every later ds_read, which would
// serialise the prefetch of patch p+1 with the MFMAs of patch p.  The caller
// waits (s_waitcnt vmcnt(0)) before the barrier that publishes the buffer.
DLCS_DEV void glds16(const void* gptr, unsigned lds_addr) {
    // m0 is saved and restored around the DMA (the compiler may keep a value in it)
    unsigned saved;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(saved) : "v"(gptr), "s"(__builtin_amdgcn_readfirstlane(lds_addr)) : "memory");
}

// the same DMA with a wave-uniform 64-bit base in SGPRs and a per-lane 32-bit
// byte offset (the saddr form: no per-lane 64-bit address arithmetic)
DLCS_DEV void glds16_s(const void* sbase, unsigned voff, unsigned lds_addr) {
    unsigned saved;
    const unsigned long long sb = (unsigned long long)(uintptr_t)sbase;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)sb);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(sb >> 32));
    const unsigned long long sbu = ((unsigned long long)hi << 32) | lo;
    // s_nop 4: the saddr pair may come straight from v_readfirstlane
    // (cdna_hip_programming.md 5.7 item 2)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 4\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(saved) : "v"(voff), "s"(sbu), "s"(__builtin_amdgcn_readfirstlane(lds_addr)) : "memory");
}

DLCS_DEV unsigned lds_offset(const void* p) {
    return (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)(p));
}

DLCS_DEV bf16x8_t tr_read16(const bf16* p0, const bf16* p1) {
    const v4s r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(const_cast<bf16*>(p0)));
    const v4s r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(const_cast<bf16*>(p1)));
    typedef short v8s __attribute__((ext_vector_type(8)));
    const v8s both = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3]};
    return __builtin_bit_cast(bf16x8_t, both);
}

// Round 5: the per-unit DMA address math (divisions of the piece index, neighbour-
// patch arithmetic, bounds tests: ~250 VALU per patch and wave, which left the three
// waves of a SIMD VALU-issue-bound beside 150 MFMAs) is computed once per lane
// relative to a per-patch scalar base, as in the f16x3 weight gradient; the raw
// per-(range, tap row) partials go to slabs summed in a fixed order (no float
// atomics: run-to-run deterministic).  28 voxel ranges x 9 tap rows = 252 workgroups.
__global__ void __launch_bounds__(768) conv3d_wgrad_c160_kernel(WgradArgs a, int nrange, int ppr, float* part) {
    __shared__ __attribute__((aligned(16))) bf16 smem[2 * kWgBuf];
    const int b = blockIdx.x;
    int range, grp;
    {                                                // the 9 tap rows of a range on one XCD (b % 8)
        const int xcd = b & 7, slot = b >> 3, q = nrange >> 3;
        if ((nrange & 7) == 0) { range = (slot / 9) * 8 + xcd; grp = slot % 9; }
        else if ((nrange & 7) == 4) {
            if (slot < 9 * q) { range = (slot / 9) * 8 + xcd; grp = slot % 9; }
            else { range = 8 * q + (xcd & 3); grp = (slot - 9 * q) + (xcd < 4 ? 0 : 5); }
        } else { range = b / 9; grp = b % 9; }
    }
    if (range >= nrange || grp >= 9) return;
    const int kd = grp / 3 - 1, kh = grp % 3 - 1;
    const int nT = a.D >> 2, nY = a.H >> 2, nX = a.W >> 2, nYX = nY * nX;
    const int npatch = a.B * nT * nYX;
    const int p0 = range * ppr, p1 = min(npatch, p0 + ppr);
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int kwi = wave >> 2, coh = (wave >> 1) & 1, cih = wave & 1;
    const int bias_rows = (nYX + nX + 1) * 64;

    // DMA of one patch: 50 wave-instructions of 64 x 16 B (20 for the g rows, 30 for
    // the halo); chunk c of the buffer = row c / 20, physical 16-B slot c % 20 holding
    // logical chunk slot ^ swz.  pk[k] = byte offset / 16 from the piece's base
    // (g: the patch's first row; halo: bias_rows before it) << 6 | 6 neighbour bits.
    unsigned pk[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const int wi = k * 12 + wave;
        const int c = wi * 64 + lane;
        const int row = c / 20, kp = c - row * 20;
        unsigned off16, req = 0;
        if (wi < 20) {
            const int kl = kp ^ (((row >> 3) & 1) << 1);
            off16 = (unsigned)(row * (a.g_ld / 8) + kl);
        } else {
            const int hr = row - 64, ty = hr / 6, xh = hr - ty * 6;
            const int t = ty >> 2, y = ty & 3;
            const int kl = kp ^ (((y >> 1) & 1) << 1);
            const int tt = t + kd, yy = y + kh, xx = xh - 1;
            req = (tt < 0 ? 1u : 0u) | (tt >= 4 ? 2u : 0u) | (yy < 0 ? 4u : 0u) | (yy >= 4 ? 8u : 0u) |
                  (xx < 0 ? 16u : 0u) | (xx >= 4 ? 32u : 0u);
            const int vrow = (((tt >> 2) * nYX + (yy >> 2) * nX + (xx >> 2)) << 6) + ((tt & 3) << 4) + ((yy & 3) << 2) +
                             (xx & 3);
            off16 = (unsigned)((vrow + bias_rows) * (a.cin_ld / 8) + kl);
        }
        pk[k] = wi < 50 ? (off16 << 6) | req : 0u;
    }
    const unsigned long long zrow = (unsigned long long)(uintptr_t)g_wg_zero_row;
    const unsigned lds0 = __builtin_amdgcn_readfirstlane(lds_offset(smem));
    int ip = p0, ipt, ipy, ipx;
    {
        const int r = ip % (nT * nYX);
        ipt = r / nYX;
        ipy = (r / nX) % nY;
        ipx = r % nX;
    }
    auto issue = [&](int buf) {                     // DMA of patch ip into buffer buf
        const unsigned miss = (ipt == 0 ? 1u : 0u) | (ipt == nT - 1 ? 2u : 0u) | (ipy == 0 ? 4u : 0u) |
                              (ipy == nY - 1 ? 8u : 0u) | (ipx == 0 ? 16u : 0u) | (ipx == nX - 1 ? 32u : 0u);
        const char* gb = reinterpret_cast<const char*>(a.g) + (long)ip * 64 * a.g_ld * 2;
        const unsigned long long xb = (unsigned long long)(uintptr_t)(reinterpret_cast<const char*>(a.in) +
                                                                     ((long)ip * 64 - bias_rows) * a.cin_ld * 2);
        const unsigned dst = lds0 + (unsigned)(buf * kWgBuf * 2);
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const int wi = k * 12 + wave;
            if (wi >= 50) break;
            const unsigned v = pk[k];
            const unsigned off = (v >> 2) & ~15u;
            if (wi < 20) {
                glds16_s(gb, off, dst + wi * 1024);
            } else {
                const unsigned long long addr = (v & miss) ? zrow : xb + off;
                glds16(reinterpret_cast<const void*>(addr), dst + wi * 1024);
            }
        }
        ++ip;                                        // advance (x, y, t) with carries
        if (++ipx == nX) {
            ipx = 0;
            if (++ipy == nY) {
                ipy = 0;
                if (++ipt == nT) ipt = 0;
            }
        }
    };

    f32x4_t acc[5][5];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) acc[i][j] = (f32x4_t)0.0f;
    // (the conv bias gradient is not summed here: g^T 1 accumulators beside the 100 of
    // the tile pushed the kernel past its 168 registers into scratch, 0.88 -> 1.33 ms per
    // launch; the entry point's column-sum pass takes it, 66 us)
    // lane -> (16-lane group gq: voxels 8gq..8gq+7 of a 32-voxel k-step; q: row
    // within a 4-row read; p4: channel quad).  Voxel v = 32 s + 8 gq + 4 h + q:
    // g row v; halo row 64 + (4 t + y) * 6 + (v & 3) + kwi with t = 2 s + gq/2,
    // y = 2 (gq & 1) + h.  Swizzle bit = gq & 1 for every row a lane reads.
    const int gq = lane >> 4, q = (lane >> 2) & 3, p4 = (lane & 3) * 4, swb = gq & 1;
    const int grow = (8 * gq + q) * kWgC;
    const int xrow = (64 + (4 * (gq >> 1) + 2 * swb) * 6 + q + kwi) * kWgC;
    auto acol = [&](int i) { return (((coh * 5 + i) ^ swb) << 4) + p4; };
    auto bcol = [&](int j) { return (((cih * 5 + j) ^ swb) << 4) + p4; };

    if (p0 < p1) issue(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int patch = p0; patch < p1; ++patch) {
#pragma unroll
        for (int k = 0; k < 5; ++k) asm volatile("" : "+v"(pk[k]));   // no hoisted, spilled decodes
        const int cur = (patch - p0) & 1;
        if (patch + 1 < p1) issue(cur ^ 1);
        const bf16* Gb = smem + cur * kWgBuf + grow;
        const bf16* Xb = smem + cur * kWgBuf + xrow;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bf16x8_t af[5];
#pragma unroll
            for (int i = 0; i < 5; ++i)
                af[i] = tr_read16(Gb + (32 * s) * kWgC + acol(i), Gb + (32 * s + 4) * kWgC + acol(i));
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const bf16x8_t bfr = tr_read16(Xb + (48 * s) * kWgC + bcol(j), Xb + (48 * s + 6) * kWgC + bcol(j));
#pragma unroll
                for (int i = 0; i < 5; ++i) mfma16(acc[i][j], af[i], bfr);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    // raw partial part[range][tap][co][ci]; C/D row -> co, col -> ci
    const int tap = (kd + 1) * 9 + (kh + 1) * 3 + kwi;
    float* pp = part + ((long)range * 27 + tap) * kWgC * kWgC;
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = coh * 80 + 16 * i + gq * 4 + r, ci = cih * 80 + 16 * j + (lane & 15);
                pp[co * kWgC + ci] = acc[i][j][r];
            }
}

// dbias[c] += sum over ranges (fixed order) of the bias-gradient partials [ranges][160]
__global__ void __launch_bounds__(160) bias_part_reduce_kernel(const float* bpart, int nrange, float* dbias) {
    const int c = threadIdx.x;
    float v = 0.0f;
    for (int r = 0; r < nrange; ++r) v += bpart[(long)r * 160 + c];
    dbias[c] += v;
}

// dW[tap][co][ci] += sum over ranges (fixed order) of the raw bf16-wgrad partials
__global__ void __launch_bounds__(256) wgrad_c160_reduce_kernel(const float* part, float* dw, int nrange) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;        // float4 index
    if (i >= 27L * 160 * 40) return;
    const f32x4_t* src = reinterpret_cast<const f32x4_t*>(part);
    f32x4_t s = src[i];
    for (int r = 1; r < nrange; ++r) s += src[(long)r * 27 * 160 * 40 + i];
    f32x4_t* d = reinterpret_cast<f32x4_t*>(dw) + i;
    *d = *d + s;
}

// ---------------------------------------------------------------- forward / dgrad v5 (bf16)
// Tile and wave map of v2 (256 voxels x 160 output channels, 8 waves = patch pw
// x channel half nh, v_mfma_f32_16x16x32_bf16, one step = 3 kw taps x 32 input
// channels), re-pipelined after in-kernel timestamps (s_memtime per phase, see
// DESIGN.md) showed v2 spending ~40 % of a step outside the MFMA stream:
//  * weights: a 2-slot LDS ring filled by global->LDS DMA (global_load_lds_dwordx4
//    in its saddr form: uniform base in SGPRs + precomputed per-lane offsets, the
//    XOR swizzle applied on the source side) -- no VGPR staging, no ds_write, no
//    per-lane 64-bit address math; waves 0-3 issue their pieces before tap 0 and
//    their SIMD partners 4-7 after it, so one wave's DMA issue overlaps the
//    other's MFMAs; waves 4-7 run at s_setprio 1 (MI355X_MICROARCH.md, two waves
//    per SIMD, item 4);
//  * halo: two buffers; the next 32-channel chunk's halo is register-prefetched
//    one step before the seam and written into the idle buffer, so a chunk seam
//    costs no extra barrier;
//  * epilogue: specialised on its operand set (EPI bits) so no registers are held
//    for operands the launch does not have, and every global operand load of a
//    slice is in flight before the slice's LDS round trip (49k -> 18k cycles).
// LDS: 2 x 38.4 KB halo + 2 x 30.7 KB weight slices = 138 KB, one workgroup per CU.
enum { kEpiRes = 1, kEpiResF32 = 2, kEpiMask = 4, kEpiAcc = 8, kEpiOutF32 = 16, kEpiGeneric = 32 };

template <int EPI>
struct EpiFlags {
    const ConvV2Args& a;
    DLCS_DEV bool res() const { return (EPI & kEpiGeneric) ? a.res != nullptr : (EPI & kEpiRes); }
    DLCS_DEV bool res_f32() const { return (EPI & kEpiGeneric) ? a.res_f32 != 0 : (EPI & kEpiResF32); }
    DLCS_DEV bool mask() const { return (EPI & kEpiGeneric) ? a.mask != nullptr : (EPI & kEpiMask); }
    DLCS_DEV bool accum() const { return (EPI & kEpiGeneric) ? a.accumulate != 0 : (EPI & kEpiAcc); }
    DLCS_DEV bool out_f32() const { return (EPI & kEpiGeneric) ? a.out_f32 != 0 : (EPI & kEpiOutF32); }
};

template <int EPI, int NTHR, int NCO, int NPASS>
DLCS_DEV void conv_epilogue_spec(const ConvV2Args& a, const f32x4_t (&acc)[4][5], float* Es, int pw, int cw0,
                                 int co0, int lane, int b, int pt, int pyq, int pxq, int nT, int nY, int nX) {
    constexpr int PC = NCO / NPASS, EL = PC + 4, NCH = PC / 8, PER = 256 * NCH / NTHR;
    static_assert(256 * NCH % NTHR == 0, "whole chunks per thread");
    const EpiFlags<EPI> F{a};
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
        long orow[PER];
        bool ok[PER];
        f32x4_t r0[PER], r1[PER], p0[PER], p1[PER];
        bf16x8_t rb[PER], pb[PER], mk[PER];      // raw loads: converted at use, after the LDS round trip
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int c = threadIdx.x + k * NTHR;
            const int vl = c / NCH, ch = (c % NCH) * 8;
            const int pwv = vl >> 6;
            const int py = pyq + (pwv >> 1), px = pxq + (pwv & 1);
            ok[k] = py < nY && px < nX;
            orow[k] = ((((long)b * nT + pt) * nY + py) * nX + px) * 64 + (vl & 63);
            const int co = co0 + pass * PC + ch;
            if (!ok[k]) continue;
            if (F.res()) {
                if (F.res_f32()) {
                    const float* rp = reinterpret_cast<const float*>(a.res) + orow[k] * a.res_ld + co;
                    r0[k] = *reinterpret_cast<const f32x4_t*>(rp);
                    r1[k] = *reinterpret_cast<const f32x4_t*>(rp + 4);
                } else {
                    rb[k] = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const bf16*>(a.res) + orow[k] * a.res_ld + co);
                }
            }
            if (F.mask()) mk[k] = *reinterpret_cast<const bf16x8_t*>(a.mask + orow[k] * a.mask_ld + co);
            if (F.accum()) {
                if (F.out_f32()) {
                    const float* o = reinterpret_cast<const float*>(a.out) + orow[k] * a.cout_ld + co;
                    p0[k] = *reinterpret_cast<const f32x4_t*>(o);
                    p1[k] = *reinterpret_cast<const f32x4_t*>(o + 4);
                } else {
                    pb[k] = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const bf16*>(a.out) + orow[k] * a.cout_ld + co);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int c0 = cw0 + j * 16 - pass * PC;
            if (c0 + 16 <= 0 || c0 >= PC) continue;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int vl = pw * 64 + i * 16 + (lane >> 4) * 4 + r;
                    const int cl = c0 + (lane & 15);
                    if (cl >= 0 && cl < PC) Es[vl * EL + cl] = acc[i][j][r];
                }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            if (!ok[k]) continue;
            const int c = threadIdx.x + k * NTHR;
            const int vl = c / NCH, ch = (c % NCH) * 8;
            const int co = co0 + pass * PC + ch;
            const f32x4_t e0 = *reinterpret_cast<const f32x4_t*>(Es + vl * EL + ch);
            const f32x4_t e1 = *reinterpret_cast<const f32x4_t*>(Es + vl * EL + ch + 4);
            float v[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) { v[e] = e0[e]; v[4 + e] = e1[e]; }
            if (a.bias) {
                const f32x4_t b0 = *reinterpret_cast<const f32x4_t*>(a.bias + co);
                const f32x4_t b1 = *reinterpret_cast<const f32x4_t*>(a.bias + co + 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) { v[e] += b0[e]; v[4 + e] += b1[e]; }
            }
            if (F.mask()) {
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = ((float)mk[k][e] > 0.0f) ? v[e] : 0.0f;
            }
            if (F.res()) {
                if (F.res_f32()) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) { v[e] += a.res_scale * r0[k][e]; v[4 + e] += a.res_scale * r1[k][e]; }
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += a.res_scale * (float)rb[k][e];
                }
            }
            if (a.relu_out) {
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.0f);
            }
            if (F.accum()) {
                if (F.out_f32()) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) { v[e] += p0[k][e]; v[4 + e] += p1[k][e]; }
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += (float)pb[k][e];
                }
            }
            const long oi = orow[k] * a.cout_ld + co;
            if (F.out_f32()) {
                float* o = reinterpret_cast<float*>(a.out) + oi;
                f32x4_t o0, o1;
#pragma unroll
                for (int e = 0; e < 4; ++e) { o0[e] = v[e]; o1[e] = v[4 + e]; }
                *reinterpret_cast<f32x4_t*>(o) = o0;
                *reinterpret_cast<f32x4_t*>(o + 4) = o1;
            } else {
                bf16x8_t ov;
#pragma unroll
                for (int e = 0; e < 8; ++e) ov[e] = (bf16)v[e];
                *reinterpret_cast<bf16x8_t*>(reinterpret_cast<bf16*>(a.out) + oi) = ov;
            }
        }
        __syncthreads();
    }
}

constexpr int kV5Slot = 3 * 160 * 32;                   // bf16 per weight slice (3 taps x 160 co x 32 ci)
__device__ unsigned long long g_conv_stamps[4096 * 4];    // per-workgroup timestamps (DLCS_CONV_STAMP=1)

template <int EPI, int STAMP>
__global__ void __launch_bounds__(512) conv3d_k3_v5_kernel(ConvV2Args a) {
    constexpr int LD = 32;
    constexpr int CO = 160;
    constexpr int HSZ = kHalo * LD;                      // bf16 per halo buffer
    __shared__ __attribute__((aligned(16))) bf16 smem_v5[2 * HSZ + 2 * kV5Slot];   // 138.2 KB
    bf16* Ws = smem_v5 + 2 * HSZ;
    const unsigned long long ts0 = STAMP ? __builtin_readcyclecounter() : 0;

    const int nT = a.D >> 2, nY = a.H >> 2, nX = a.W >> 2;
    const int nYt = (nY + 1) >> 1, nXt = (nX + 1) >> 1;
    int bid = blockIdx.x;
    if (a.xcd_major) {                                   // XCD x = b % 8 runs one contiguous run of tiles
        const int nblk = a.B * nT * nYt * nXt, q8 = nblk >> 3, r8 = nblk & 7, xcd = bid & 7;
        bid = xcd * q8 + min(xcd, r8) + (bid >> 3);
    }
    const int txx = bid % nXt; bid /= nXt;
    const int tyy = bid % nYt; bid /= nYt;
    const int pt = bid % nT;
    const int b = bid / nT;
    const int t0 = pt * 4, y0 = tyy * 8, x0 = txx * 8;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int pw = wave & 3, nh = wave >> 2;
    const int ncc = a.cin_pad / CK;
    const int nsteps = ncc * 9;                          // step s: chunk s / 9, tap row s % 9

    constexpr int HPER = (kHalo * 4 + 511) / 512;        // 5
    bf16x8_t hr[HPER];
    // per-lane element offsets of this thread's halo chunks (channel chunk 0), -1 off the grid
    int hoff[HPER];
#pragma unroll
    for (int k = 0; k < HPER; ++k) {
        const int i = threadIdx.x + k * 512;
        hoff[k] = -1;
        if (i < kHalo * 4) {
            const int hv = i >> 2, c8 = (i & 3) * 8;
            const int ht = hv / (kHaloY * kHaloX), hy = (hv / kHaloX) % kHaloY, hx = hv % kHaloX;
            const int t = t0 - 1 + ht, y = y0 - 1 + hy, x = x0 - 1 + hx;
            if (t >= 0 && t < a.D && y >= 0 && y < a.H && x >= 0 && x < a.W)
                hoff[k] = (int)(brow(b, t, y, x, nT, nY, nX) * a.cin_ld + c8);
        }
    }
    auto load_halo = [&](int cc) {
        const bf16* base = a.in + cc * CK;
#pragma unroll
        for (int k = 0; k < HPER; ++k) {
            hr[k] = (bf16x8_t)(bf16)0.0f;
            if (hoff[k] >= 0) hr[k] = *reinterpret_cast<const bf16x8_t*>(base + hoff[k]);
        }
    };
    // halo rows are 64 B (32 channels); the four 16-B chunks of row hv (halo y
    // hy) sit XOR-swizzled by 2 (hy & 1) so every ds_read_b128 lane group hits 16
    // distinct bank quads
    auto store_halo = [&](int buf) {
        bf16* Hs = smem_v5 + buf * HSZ;
#pragma unroll
        for (int k = 0; k < HPER; ++k) {
            const int i = threadIdx.x + k * 512;
            if (i < kHalo * 4) {
                const int hv = i >> 2, c = i & 3;
                const int hy = (hv / kHaloX) % kHaloY;
                *reinterpret_cast<bf16x8_t*>(Hs + hv * LD + ((c ^ ((hy & 1) << 1)) << 3)) = hr[k];
            }
        }
    };
    // weight DMA of step s into slice s & 1: 30 pieces of 64 x 16 B, piece
    // wave + 8k issued by this wave.  LDS chunk c (row c >> 2 = tap * 160 + co,
    // position c & 3) receives the logical 8-channel chunk (c & 3) ^ swz(co).
    const unsigned wbase = lds_offset(Ws);
    unsigned woff[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int wi = k * 8 + wave;
        const int c = wi * 64 + lane;
        const int row = c >> 2, pos = c & 3;
        const int tl = row >= 2 * CO ? 2 : (row >= CO ? 1 : 0);
        const int co = row - tl * CO;
        const int kl = pos ^ ((4 - ((co & 15) >> 2)) & 3);
        woff[k] = (unsigned)(((tl * CO + co) * a.cin_pad + (kl << 3)) * 2);
    }
    auto issue_w = [&](int s) {
        const int cc = s / 9, t3 = (s % 9) * 3;
        const unsigned dst = wbase + (unsigned)((s & 1) * kV5Slot * 2);
        const bf16* src = a.w + (long)t3 * CO * a.cin_pad + cc * CK;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int wi = k * 8 + wave;
            if (wi < 30) glds16_s(src, woff[k], dst + wi * 1024);
        }
    };

    f32x4_t acc[4][5];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) acc[i][j] = (f32x4_t)0.0f;

    const int pyy = pw >> 1, pxx = pw & 1;
    const int vq = lane & 15, cq = lane >> 4;
    const int ly = pyy * 4 + ((vq >> 2) & 3), lx = pxx * 4 + (vq & 3);
    const int hb0 = ly * kHaloX + lx;
    const int corow = nh * 80 + vq;
    const int bpos = (cq ^ ((4 - (vq >> 2)) & 3)) << 3;

    auto read_frags = [&](int s, int kw, bf16x8_t (&af)[4], bf16x8_t (&bfr)[5]) {
        const int st = s % 9, kd = st / 3, kh = st % 3;
        const int apos = (cq ^ (((ly + kh) & 1) << 1)) << 3;
        const int toff = (kd * kHaloY + kh) * kHaloX + kw;
        const bf16* Hs = smem_v5 + ((s / 9) & 1) * HSZ;
        const bf16* wb = Ws + (s & 1) * kV5Slot;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            af[i] = *reinterpret_cast<const bf16x8_t*>(Hs + (hb0 + i * kHaloY * kHaloX + toff) * LD + apos);
#pragma unroll
        for (int j = 0; j < 5; ++j)
            bfr[j] = *reinterpret_cast<const bf16x8_t*>(wb + (kw * CO + corow + j * 16) * LD + bpos);
    };
    auto mma = [&](const bf16x8_t (&af)[4], const bf16x8_t (&bfr)[5]) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 5; ++j) mfma16(acc[i][j], af[i], bfr[j]);
    };

    load_halo(0);
    issue_w(0);
    store_halo(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long ts1 = STAMP ? __builtin_readcyclecounter() : 0;

    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    for (int s = 0; s < nsteps; ++s) {
        const int sc = s % 9;                            // position inside the chunk (seam after sc == 8)
        const bool seam = (sc == 8) && (s + 1 < nsteps);
        if (sc == 7 && s + 2 < nsteps) load_halo(s / 9 + 1);
        const bool dma = s + 1 < nsteps;
        bf16x8_t afA[4], bfA[5], afB[4], bfB[5];
        if (dma && wave < 4) issue_w(s + 1);
        read_frags(s, 0, afA, bfA);
        read_frags(s, 1, afB, bfB);
        mma(afA, bfA);
        if (dma && wave >= 4) issue_w(s + 1);
        read_frags(s, 2, afA, bfA);
        mma(afB, bfB);
        mma(afA, bfA);
        if (seam) store_halo((s / 9 + 1) & 1);           // the idle buffer: no reader before the barrier
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // step s+1's weight slice has landed
        __syncthreads();
    }
    const unsigned long long ts2 = STAMP ? __builtin_readcyclecounter() : 0;
    conv_epilogue_spec<EPI, 512, 160, 2>(a, acc, reinterpret_cast<float*>(smem_v5), pw, nh * 80, 0, lane, b, pt,
                                         tyy * 2, txx * 2, nT, nY, nX);
    if (STAMP && threadIdx.x == 0 && blockIdx.x < 4096) {
        const unsigned long long ts3 = __builtin_readcyclecounter();
        g_conv_stamps[blockIdx.x * 4 + 0] = ts0;
        g_conv_stamps[blockIdx.x * 4 + 1] = ts1;
        g_conv_stamps[blockIdx.x * 4 + 2] = ts2;
        g_conv_stamps[blockIdx.x * 4 + 3] = ts3;
    }
}

// ---------------------------------------------------------------- wgrad, 160 <-> thin (bf16)
// The ConvBlocks' thin ends: SFE 4 -> 160 (dW[tap][co][ci<4]) and the final
// 160 -> 4 (dW[tap][co<4][ci]).  With u = v + off the sum
//   dW[tap][co][ci] = sum_v g[v][co] x[v + off][ci] = sum_u x[u][ci] g[u - off][co]
// always puts the tap shift on the thin side: Big[u][b] (160 channels,
// unshifted) times Thin[u + sgn * off][s] (SC <= 8 channels, 16-B rows).  Per
// 64-voxel patch the thin side's 6x6x6 halo is DMA'd to LDS and expanded to an
// im2col image [27 * SC (pad 16) columns][64 voxels] (4 taps x 4 channels per
// 16-wide MFMA tile), so one pass is a [160] x [112] GEMM over voxels; the big
// side is DMA'd as in the 160 kernel and read with ds_read_b64_tr_b16.
// 5 waves x 32 big channels, 2 workgroups per CU.
struct ThinWgArgs {
    const bf16* big; const bf16* thin; float* dw;
    int big_ld, sgn, big_is_co, thin_ch, cout_pad, cin_pad;
    int B, D, H, W;
    float* bpart;           // optional: per-range column sums of the big side [ranges][160] (SFE bias gradient)
};

template <int SC>
__global__ void __launch_bounds__(320) conv3d_wgrad_thin_kernel(ThinWgArgs a, int nrange, int ppr) {
    constexpr int NCOL = 27 * SC, NTL = (NCOL + 15) / 16, IMLD = 72;
    constexpr int BIGB = 64 * kWgC * 2, HALB = 216 * 16, BUFB = BIGB + HALB;
    __shared__ __attribute__((aligned(16))) char smem[2 * BUFB + NTL * 16 * IMLD * 2];
    bf16* im = reinterpret_cast<bf16*>(smem + 2 * BUFB);
    const int range = blockIdx.x;
    if (range >= nrange) return;
    const int nT = a.D >> 2, nY = a.H >> 2, nX = a.W >> 2;
    const int npatch = a.B * nT * nY * nX;
    const int p0 = range * ppr, p1 = min(npatch, p0 + ppr);
    if (p0 >= p1) return;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bf16* zrow = reinterpret_cast<const bf16*>(g_wg_zero_row);
    const unsigned sbase = lds_offset(smem);

    auto issue = [&](int patch, int buf) {
        const int px = patch % nX;
        int r = patch / nX;
        const int py = r % nY; r /= nY;
        const int pt = r % nT;
        const int bb = r / nT;
        const unsigned dst = sbase + buf * BUFB;
        int ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int k = 0; k < 4; ++k) {                  // big rows: 20 wave-instructions
            const int wi = k * 5 + wave;
            const int c = wi * 64 + ln;
            const int row = c / 20, kp = c - row * 20;
            const int kl = kp ^ (((row >> 3) & 1) << 1);
            glds16(a.big + (long)(patch * 64 + row) * a.big_ld + (kl << 3), dst + wi * 1024);
        }
        if (wave < 4) {                                // thin halo: 216 rows of 16 B
            const int c = wave * 64 + ln;
            if (c < 216) {
                const int hz = c / 36, hy = (c / 6) % 6, hx = c % 6;
                const int T = pt * 4 + hz - 1, Y = py * 4 + hy - 1, X = px * 4 + hx - 1;
                const bool ok = (unsigned)T < (unsigned)a.D && (unsigned)Y < (unsigned)a.H && (unsigned)X < (unsigned)a.W;
                const int vrow = ((((bb * nT + (T >> 2)) * nY + (Y >> 2)) * nX + (X >> 2)) << 6) + ((T & 3) << 4) +
                                 ((Y & 3) << 2) + (X & 3);
                glds16(ok ? a.thin + (long)vrow * 8 : zrow, dst + BIGB + wave * 1024);
            }
        }
    };

    // padding columns of the im2col image stay zero
    for (int i = threadIdx.x; i < (NTL * 16 - NCOL) * (IMLD / 8); i += 320)
        *reinterpret_cast<uint4*>(im + NCOL * IMLD + i * 8) = make_uint4(0, 0, 0, 0);

    f32x4_t acc[2][NTL];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j) acc[i][j] = (f32x4_t)0.0f;
    f32x4_t csacc[2] = {(f32x4_t)0.0f, (f32x4_t)0.0f};
    const bf16x8_t ones = (bf16x8_t)(bf16)1.0f;
    const int gq = lane >> 4, q = (lane >> 2) & 3, p4 = (lane & 3) * 4, swb = gq & 1;
    const int grow = (8 * gq + q) * kWgC;

    issue(p0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int patch = p0; patch < p1; ++patch) {
        const int cur = (patch - p0) & 1;
        __syncthreads();
        if (patch + 1 < p1) issue(patch + 1, cur ^ 1);
        // im2col: item = (tap, group of 8 consecutive patch voxels)
        const bf16* hal = reinterpret_cast<const bf16*>(smem + cur * BUFB + BIGB);
        for (int it = threadIdx.x; it < 27 * 8; it += 320) {
            const int tap = it >> 3, vg = it & 7;
            const int kd = tap / 9 - 1, kh = (tap / 3) % 3 - 1, kw = tap % 3 - 1;
            const int t = vg >> 1, y0 = 2 * (vg & 1);
            float v[8][SC];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int y = y0 + (e >> 2), x = e & 3;
                const int hr = ((t + 1 + a.sgn * kd) * 6 + (y + 1 + a.sgn * kh)) * 6 + (x + 1 + a.sgn * kw);
                const bf16x8_t r8 = *reinterpret_cast<const bf16x8_t*>(hal + hr * 8);
#pragma unroll
                for (int c = 0; c < SC; ++c) v[e][c] = (float)r8[c];
            }
#pragma unroll
            for (int c = 0; c < SC; ++c) {
                bf16x8_t o;
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e][c];
                *reinterpret_cast<bf16x8_t*>(im + (tap * SC + c) * IMLD + vg * 8) = o;
            }
        }
        __syncthreads();
        const bf16* Gb = reinterpret_cast<const bf16*>(smem + cur * BUFB) + grow;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bf16x8_t af[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int col = (((2 * wave + i) ^ swb) << 4) + p4;
                af[i] = tr_read16(Gb + (32 * s) * kWgC + col, Gb + (32 * s + 4) * kWgC + col);
            }
            if (a.bpart) {                             // Big^T 1: the big side's column sums
#pragma unroll
                for (int i = 0; i < 2; ++i) mfma16(csacc[i], af[i], ones);
            }
#pragma unroll
            for (int j = 0; j < NTL; ++j) {
                const bf16x8_t bfr = *reinterpret_cast<const bf16x8_t*>(im + (j * 16 + (lane & 15)) * IMLD + 32 * s + 8 * gq);
#pragma unroll
                for (int i = 0; i < 2; ++i) mfma16(acc[i][j], af[i], bfr);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (a.bpart && (lane & 15) == 0) {                 // every column of the ones tile holds the sums
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) a.bpart[(long)range * kWgC + 32 * wave + 16 * i + 4 * gq + r] = csacc[i][r];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int bch = 32 * wave + 16 * i + 4 * gq + r, n = 16 * j + (lane & 15);
                const int tap = n / SC, sc = n - tap * SC;
                if (n < NCOL && sc < a.thin_ch) {
                    const int co = a.big_is_co ? bch : sc, ci = a.big_is_co ? sc : bch;
                    atomicAdd(a.dw + ((long)tap * a.cout_pad + co) * a.cin_pad + ci, acc[i][j][r]);
                }
            }
}

#include "conv3d_f32.inc"
#ifdef DLCS_DIAG_BUILD
#include "conv3d_x6.inc"                                // superseded bf16 3-plane conv (DIAG build)
#endif
#include "conv3d_f16x3.inc"
#include "conv3d_v6.inc"
#include "conv3d_v7.inc"
#include "conv3d_thin_f16x3.inc"
#include "conv3d_thin_planes.inc"
#include "gemm_h3r.inc"
#include "gemm_f8r.inc"

// ---------------------------------------------------------------- weight packing
// mode 0 (forward):  P[tap][co][ci] = W[co][ci][tap]
// mode 1 (dgrad):    P[tap][ci][co] = W[co][ci][26 - tap]
template <typename T>
__global__ void pack_weights_kernel(const float* w, T* p, int Cout, int Cin, int rows_pad, int cols_pad, int mode) {
    const long total = 27L * rows_pad * cols_pad;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int c = (int)(i % cols_pad);
        const int r = (int)((i / cols_pad) % rows_pad);
        const int tap = (int)(i / ((long)cols_pad * rows_pad));
        float v = 0.0f;
        if (mode == 0) {
            if (r < Cout && c < Cin) v = w[((long)r * Cin + c) * 27 + tap];
        } else {
            if (r < Cin && c < Cout) v = w[((long)c * Cin + r) * 27 + (26 - tap)];
        }
        p[i] = from_f<T>(v);
    }
}

// grad[co][ci][tap] (+)= dw_packed[tap][co][ci]
__global__ void unpack_wgrad_kernel(const float* dwp, float* grad, int Cout, int Cin, int cout_pad, int cin_pad,
                                    int accumulate) {
    const long total = (long)Cout * Cin * 27;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int tap = (int)(i % 27);
        const int ci = (int)((i / 27) % Cin);
        const int co = (int)(i / (27L * Cin));
        const float v = dwp[((long)tap * cout_pad + co) * cin_pad + ci];
        grad[i] = accumulate ? grad[i] + v : v;
    }
}

// DLCS_CONV_V2=1 selects the v2 forward / dgrad kernel (A/B timing only);
// DLCS_CONV_STAMP=1 makes the v5 kernel record per-workgroup timestamps
// (dlcs_debug_conv_stamps, tools/conv_stamps.py)
static bool conv_v2_forced() {
    static const bool f = [] { const char* e = dlcs_knob("DLCS_CONV_V2"); return e && e[0] == '1'; }();
    return f;
}
// DLCS_CONV_V5=1 (DIAG build): the 160-channel bf16 forward / dgrad on the v5 kernel
// (one tap row per step) instead of v6 (conv3d_v6.inc), for A/B timing
static bool conv_v5_forced() {
    static const bool f = [] { const char* e = dlcs_knob("DLCS_CONV_V5"); return e && e[0] == '1'; }();
    return f;
}
static bool conv_stamps_on() {
    static const bool f = [] { const char* e = dlcs_knob("DLCS_CONV_STAMP"); return e && e[0] == '1'; }();
    return f;
}

template <typename T>
size_t conv_smem(int nt) { return (size_t)(kHalo + 2 * nt * 32) * (CK + ConvPad<T>::v) * sizeof(T); }

template <typename T>
int conv_launch(const ConvArgs& a, hipStream_t st) {
    const int nT = a.D / 4, nY = a.H / 4, nX = a.W / 4;
    const unsigned nblk = (unsigned)((long)a.B * nT * ((nY + 1) / 2) * ((nX + 1) / 2));
    if constexpr (std::is_same<T, bf16>::value) {
        // v2 epilogue uses 16-B accesses: row strides multiple of 8 elements
        // and 16-B aligned bases (torch allocations are)
        auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
        const bool vec_ok = a.cout_ld % 8 == 0 && al16(a.out) && (!a.mask || (a.mask_ld % 8 == 0 && al16(a.mask))) &&
                            (!a.res || (a.res_ld % 8 == 0 && al16(a.res)));
        if (a.Cout <= 4 && a.Cin == 160 && a.cin_pad == 160 && a.cin_ld % 8 == 0 && al16(a.in) && !a.relu_in &&
            !a.mask && !a.res && !a.relu_out && !a.accumulate && a.cout_ld % 4 == 0 && al16(a.out)) {
            const int npatch = a.B * nT * nY * nX;
            hipLaunchKernelGGL(conv3d_thin_out_kernel, dim3(std::min(npatch, 256)), dim3(448), 0, st, a, npatch);
            return dlcs_launch_status();
        }
        if (a.cout_pad == 160 && a.Cout == 160 && !a.relu_in && a.Cin <= 4 && a.cin_ld == 8 && a.cin_pad % 4 == 0 &&
            vec_ok && al16(a.in)) {
            ConvV2Args v{};
            v.in = (const bf16*)a.in; v.w = (const bf16*)a.w; v.bias = a.bias; v.out = a.out;
            v.mask = (const bf16*)a.mask; v.res = a.res;
            v.B = a.B; v.D = a.D; v.H = a.H; v.W = a.W; v.cin_ld = a.cin_ld; v.cin_pad = a.cin_pad;
            v.cout_ld = a.cout_ld; v.mask_ld = a.mask_ld; v.res_ld = a.res_ld; v.out_f32 = a.out_f32;
            v.res_f32 = a.res_f32; v.accumulate = a.accumulate; v.relu_out = a.relu_out; v.res_scale = a.res_scale;
            int epi;
            if (!v.res && !v.mask && !v.accumulate && !v.out_f32) epi = 0;
            else if (!v.res && v.mask && !v.accumulate && !v.out_f32) epi = kEpiMask;
            else epi = kEpiGeneric;
            const dim3 g(std::min(nblk, 512u));
            if (epi == 0) hipLaunchKernelGGL(conv3d_thin_in_kernel<0>, g, dim3(512), 0, st, v, (int)nblk);
            else if (epi == kEpiMask) hipLaunchKernelGGL(conv3d_thin_in_kernel<kEpiMask>, g, dim3(512), 0, st, v, (int)nblk);
            else hipLaunchKernelGGL(conv3d_thin_in_kernel<kEpiGeneric>, g, dim3(512), 0, st, v, (int)nblk);
            return dlcs_launch_status();
        }
        if (a.cout_pad == 160 && a.Cout == 160 && !a.relu_in && a.cin_ld % 8 == 0 && a.Cin == a.cin_pad && vec_ok) {
            ConvV2Args v{};
            v.in = (const bf16*)a.in; v.w = (const bf16*)a.w; v.bias = a.bias; v.out = a.out;
            v.mask = (const bf16*)a.mask; v.res = a.res;
            v.B = a.B; v.D = a.D; v.H = a.H; v.W = a.W; v.cin_ld = a.cin_ld; v.cin_pad = a.cin_pad;
            v.cout_ld = a.cout_ld; v.mask_ld = a.mask_ld; v.res_ld = a.res_ld; v.out_f32 = a.out_f32;
            v.res_f32 = a.res_f32; v.accumulate = a.accumulate; v.relu_out = a.relu_out; v.res_scale = a.res_scale;
            if (conv_v2_forced()) {
                hipLaunchKernelGGL(conv3d_k3_v2_kernel, dim3(nblk), dim3(512), 0, st, v);
            } else if (v.cin_pad == 160 && !conv_v5_forced()) {
                // v6; DLCS_CONV_V7=1 (test hook) runs the two-workgroups-per-CU v7 kernel
                // (same-box A/B at parity: conv3d_v7.inc header, DESIGN round-6 item 1)
                const char* f7 = dlcs_test_hook("DLCS_CONV_V7");
                if (f7 && f7[0] == '1') return conv_v7_launch(v, st);
                return conv_v6_launch(v, st);
            } else {
                // the two production epilogues (ResSwin / DFE tail forward: bf16 residual;
                // dgrad: ReLU mask) and one runtime-flag variant for everything else
                int epi;
                if (!v.res && !v.mask && !v.accumulate && !v.out_f32) epi = 0;
                else if (v.res && !v.res_f32 && !v.mask && !v.accumulate && !v.out_f32) epi = kEpiRes;
                else if (!v.res && v.mask && !v.accumulate && !v.out_f32) epi = kEpiMask;
                else epi = kEpiGeneric;
                const bool stamp = conv_stamps_on();
                static const int xcd_env = [] { const char* e = dlcs_knob("DLCS_CONV_XCD"); return e ? atoi(e) : 1; }();
                v.xcd_major = xcd_env;
#define V5_LAUNCH(E) do { if (stamp) hipLaunchKernelGGL((conv3d_k3_v5_kernel<E, 1>), dim3(nblk), dim3(512), 0, st, v); \
                          else hipLaunchKernelGGL((conv3d_k3_v5_kernel<E, 0>), dim3(nblk), dim3(512), 0, st, v); } while (0)
                if (epi == 0) V5_LAUNCH(0);
                else if (epi == kEpiRes) V5_LAUNCH(kEpiRes);
                else if (epi == kEpiMask) V5_LAUNCH(kEpiMask);
                else V5_LAUNCH(kEpiGeneric);
#undef V5_LAUNCH
            }
            return dlcs_launch_status();
        }
    }
    if constexpr (std::is_same<T, float>::value) {
        auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
        const long rows = (long)a.B * a.D * a.H * a.W;
        if (a.cout_pad == 160 && a.Cout == 160 && a.Cin == 160 && a.cin_pad == 160 && !a.relu_in && a.out_f32 &&
            a.cin_ld % 4 == 0 && a.cout_ld % 4 == 0 && al16(a.in) && al16(a.out) && al16(a.w) &&
            (!a.mask || (a.mask_ld % 4 == 0 && al16(a.mask))) && (!a.res || (a.res_f32 && a.res_ld % 4 == 0 && al16(a.res))) &&
            (!a.bias || al16(a.bias)) && rows * a.cin_ld < (1L << 31))
            return conv_f32_c160_launch(a, st);
        // thin input (SFE forward, final-conv dgrad): Cin <= 4 in 16-B rows
        if (a.cout_pad == 160 && a.Cout == 160 && a.Cin <= 4 && a.cin_pad >= 4 && !a.relu_in && a.out_f32 &&
            a.cin_ld % 4 == 0 && a.cout_ld % 4 == 0 && al16(a.in) && al16(a.out) &&
            (!a.mask || (a.mask_ld % 4 == 0 && al16(a.mask))) && (!a.res || (a.res_f32 && a.res_ld % 4 == 0 && al16(a.res))) &&
            (!a.bias || al16(a.bias)) && rows * a.cout_ld < (1L << 31))
            return conv_f32_thin_launch(a, st, true);
        // thin output (final conv forward, SFE dgrad): Cout <= 4 written as one 16-B row chunk
        if (a.Cin == 160 && a.cin_pad == 160 && a.Cout <= 4 && a.cout_ld >= 4 && !a.relu_in && a.out_f32 && !a.mask &&
            !a.res && a.cin_ld % 4 == 0 && a.cout_ld % 4 == 0 && al16(a.in) && al16(a.out) && al16(a.w) &&
            rows * a.cin_ld < (1L << 31))
            return conv_f32_thin_launch(a, st, false);
    }
    const int nt = a.cout_pad / 32;
    const size_t sm = conv_smem<T>(nt);
    if (nt == 5) {
        (void)hipFuncSetAttribute((const void*)conv3d_k3_kernel<T, 5>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipLaunchKernelGGL((conv3d_k3_kernel<T, 5>), dim3(nblk), dim3(256), sm, st, a);
    } else if (nt == 1) {
        (void)hipFuncSetAttribute((const void*)conv3d_k3_kernel<T, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipLaunchKernelGGL((conv3d_k3_kernel<T, 1>), dim3(nblk), dim3(256), sm, st, a);
    } else if (nt == 2) {
        (void)hipFuncSetAttribute((const void*)conv3d_k3_kernel<T, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipLaunchKernelGGL((conv3d_k3_kernel<T, 2>), dim3(nblk), dim3(256), sm, st, a);
    } else if (nt == 4) {
        (void)hipFuncSetAttribute((const void*)conv3d_k3_kernel<T, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        hipLaunchKernelGGL((conv3d_k3_kernel<T, 4>), dim3(nblk), dim3(256), sm, st, a);
    } else {
        return DLCS_ERR_UNSUPPORTED_SIZE;
    }
    return dlcs_launch_status();
}

template <typename T>
int wgrad_launch(const WgradArgs& a, hipStream_t st, bool* bias_done);

template <>
int wgrad_launch<bf16>(const WgradArgs& a, hipStream_t st, bool* bias_done) {
    const int mt = a.cout_pad / 32, nt = a.cin_pad / 32;
    const long npatch = (long)a.B * (a.D / 4) * (a.H / 4) * (a.W / 4);
    int nrange = (int)(a.vox_per_block > 0 ? (npatch * 64 + a.vox_per_block - 1) / a.vox_per_block : 40);
    if (nrange < 1) nrange = 1;
    const long ppr = (npatch + nrange - 1) / nrange;
    nrange = (int)((npatch + ppr - 1) / ppr);
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (mt == 5 && nt == 5 && a.Cin == 160 && a.Cout == 160 && !a.relu_in && a.cin_ld % 8 == 0 && a.g_ld % 8 == 0 &&
        al16(a.in) && al16(a.g)) {
        const long bias_rows = ((long)(a.H / 4) * (a.W / 4) + a.W / 4 + 1) * 64;
        if ((2 * bias_rows + 128) * (std::max(a.cin_ld, a.g_ld) / 8) >= (1L << 26) || npatch >= (1L << 30) ||
            ((long)a.g_ld * 128 * 2) >= (1L << 31))
            return DLCS_ERR_UNSUPPORTED_SIZE;       // 32-bit lane offsets (16-B units << 6)
        int nr = (int)std::min<long>(28, npatch);
        const long pp = (npatch + nr - 1) / nr;
        nr = (int)((npatch + pp - 1) / pp);
        float* part = wgh3_workspace(st);           // the f16x3 weight gradient's slabs (same stream order)
        if (!part) return (int)hipErrorOutOfMemory;
        hipLaunchKernelGGL(conv3d_wgrad_c160_kernel, dim3((unsigned)(9 * nr)), dim3(768), 0, st, a, nr, (int)pp, part);
        hipLaunchKernelGGL(wgrad_c160_reduce_kernel, dim3((unsigned)cdiv(27L * 160 * 40, 256)), dim3(256), 0, st,
                           (const float*)part, a.dw, nr);
        return dlcs_launch_status();                // the bias (if asked) by the caller's column-sum pass
    }
    // thin ends (<= 8 channels on one side, 16-B rows there; 160 on the other)
    const bool thin_sfe = a.Cout == 160 && mt == 5 && a.Cin <= 8 && a.cin_ld == 8 && a.g_ld % 8 == 0;
    const bool thin_fin = a.Cin == 160 && nt == 5 && a.Cout <= 8 && a.g_ld == 8 && a.cin_ld % 8 == 0;
    if ((thin_sfe || thin_fin) && !a.relu_in && al16(a.in) && al16(a.g) && npatch < (1L << 24)) {
        ThinWgArgs t{};
        t.big = (const bf16*)(thin_sfe ? a.g : a.in);
        t.thin = (const bf16*)(thin_sfe ? a.in : a.g);
        t.dw = a.dw; t.big_ld = thin_sfe ? a.g_ld : a.cin_ld; t.sgn = thin_sfe ? 1 : -1; t.big_is_co = thin_sfe;
        t.thin_ch = thin_sfe ? a.Cin : a.Cout; t.cout_pad = a.cout_pad; t.cin_pad = a.cin_pad;
        t.B = a.B; t.D = a.D; t.H = a.H; t.W = a.W;
        int nr = (int)std::min<long>(512, npatch);
        const int pp = (int)((npatch + nr - 1) / nr);
        nr = (int)((npatch + pp - 1) / pp);            // every range non-empty (each writes its bias partial)
        if (a.dbias && thin_sfe) {                     // the SFE bias gradient = column sums of g (the big side)
            t.bpart = static_cast<float*>(scratch(kScrBiasPart, st, (size_t)nr * 160 * sizeof(float)));
            if (!t.bpart) return (int)hipErrorOutOfMemory;
        }
        if (t.thin_ch <= 4)
            hipLaunchKernelGGL(conv3d_wgrad_thin_kernel<4>, dim3(nr), dim3(320), 0, st, t, nr, pp);
        else
            hipLaunchKernelGGL(conv3d_wgrad_thin_kernel<8>, dim3(nr), dim3(320), 0, st, t, nr, pp);
        if (t.bpart) {
            hipLaunchKernelGGL(bias_part_reduce_kernel, dim3(1), dim3(160), 0, st, (const float*)t.bpart, nr, a.dbias);
            *bias_done = true;
        }
        return dlcs_launch_status();
    }
    const int groups = (nrange + 7) / 8;
    dim3 grid((unsigned)(groups * 8 * 27)), block(320);
    if (mt == 5 && nt == 5) hipLaunchKernelGGL((conv3d_wgrad_tr_kernel<5, 5>), grid, block, 0, st, a, nrange, ppr);
    else if (mt == 5 && nt == 1) hipLaunchKernelGGL((conv3d_wgrad_tr_kernel<5, 1>), grid, block, 0, st, a, nrange, ppr);
    else if (mt == 1 && nt == 5) hipLaunchKernelGGL((conv3d_wgrad_tr_kernel<1, 5>), grid, block, 0, st, a, nrange, ppr);
    else return DLCS_ERR_UNSUPPORTED_SIZE;
    return dlcs_launch_status();
}

template <>
int wgrad_launch<float>(const WgradArgs& a, hipStream_t st, bool* bias_done) {
    (void)bias_done;
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (a.cout_pad == 160 && a.cin_pad == 160 && a.Cin == 160 && a.Cout == 160 && !a.relu_in && a.cin_ld % 4 == 0 &&
        a.g_ld % 4 == 0 && al16(a.in) && al16(a.g))
        return wgrad_f32_c160_launch(a, st);
    {
        // thin ends (<= 4 channels on one side in 16-B-aligned rows, 160 on the other)
        const long npatch = (long)a.B * (a.D / 4) * (a.H / 4) * (a.W / 4);
        const bool thin_sfe = a.Cout == 160 && a.cout_pad == 160 && a.Cin <= 4 && a.cin_ld % 4 == 0 && a.g_ld % 4 == 0;
        const bool thin_fin = a.Cin == 160 && a.cin_pad == 160 && a.Cout <= 4 && a.g_ld % 4 == 0 && a.cin_ld % 4 == 0;
        if ((thin_sfe || thin_fin) && !a.relu_in && al16(a.in) && al16(a.g) && npatch * 64 * 160 < (1L << 31)) {
            ThinWgF32Args t{};
            t.big = (const float*)(thin_sfe ? a.g : a.in);
            t.thin = (const float*)(thin_sfe ? a.in : a.g);
            t.dw = a.dw; t.big_ld = thin_sfe ? a.g_ld : a.cin_ld; t.thin_ld = thin_sfe ? a.cin_ld : a.g_ld;
            t.sgn = thin_sfe ? 1 : -1; t.big_is_co = thin_sfe;
            t.thin_ch = thin_sfe ? a.Cin : a.Cout; t.cout_pad = a.cout_pad; t.cin_pad = a.cin_pad;
            t.B = a.B; t.D = a.D; t.H = a.H; t.W = a.W;
            const int nr = (int)std::min<long>(256, npatch);
            const int pp = (int)((npatch + nr - 1) / nr);
            hipLaunchKernelGGL(conv3d_wgrad_thin_f32_kernel, dim3(nr), dim3(512), 0, st, t, nr, pp);
            return dlcs_launch_status();
        }
    }
    const long nvox = (long)a.B * a.D * a.H * a.W;
    const unsigned nb = cdiv(nvox, a.vox_per_block);
    const int mt = a.cout_pad / 32, nt = a.cin_pad / 32;
    const size_t sm = (size_t)(a.cout_pad + nt * 32) * (32 + ConvPad<float>::v) * sizeof(float);
    dim3 grid(nb, 27);
    dim3 block(mt * 64 < 64 ? 64 : mt * 64);
    if (nt == 5) hipLaunchKernelGGL((conv3d_wgrad_kernel<float, 5>), grid, block, sm, st, a);
    else if (nt == 1) hipLaunchKernelGGL((conv3d_wgrad_kernel<float, 1>), grid, block, sm, st, a);
    else if (nt == 2) hipLaunchKernelGGL((conv3d_wgrad_kernel<float, 2>), grid, block, sm, st, a);
    else if (nt == 4) hipLaunchKernelGGL((conv3d_wgrad_kernel<float, 4>), grid, block, sm, st, a);
    else return DLCS_ERR_UNSUPPORTED_SIZE;
    return dlcs_launch_status();
}

static unsigned grid_for(long n) {
    long g = (n + 255) / 256;
    return (unsigned)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" {

size_t dlcs_scratch_bytes(void) {
    std::lock_guard<std::mutex> lk(g_scr_mu);
    size_t n = 0;
    for (const auto& e : g_scr) n += e.second.second;
    return n;
}

int dlcs_release_scratch(void) {
    std::lock_guard<std::mutex> lk(g_scr_mu);
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return dlcs_launch_status();
    int st = 0;
    std::map<int, bool> synced;
    for (auto& e : g_scr) {
        const int dev = std::get<1>(e.first);
        if (!synced[dev]) {
            synced[dev] = true;
            if (hipSetDevice(dev) != hipSuccess || hipDeviceSynchronize() != hipSuccess) st = dlcs_launch_status();
        }
        if (e.second.first && hipFree(e.second.first) != hipSuccess && !st) st = dlcs_launch_status();
    }
    g_scr.clear();
    (void)hipSetDevice(cur);
    return st;
}

#ifdef DLCS_DIAG_BUILD
int dlcs_debug_h3_stamps(void* host, int64_t n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_h3_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}

int dlcs_debug_conv_stamps(void* host, int64_t n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_conv_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
#endif

int dlcs_conv3d_k3(int dtype, const void* in, int64_t cin, int64_t cin_ld, const void* wpacked,
                   int64_t cin_pad, const float* bias, void* out, int out_dtype, int64_t cout,
                   int64_t cout_pad, int64_t cout_ld, int64_t B, int64_t D, int64_t H, int64_t W,
                   int relu_in, const void* mask, int64_t mask_ld, const void* residual, int res_dtype,
                   int64_t res_ld, float res_scale, int accumulate, int relu_out, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(in && wpacked && out && B > 0);
    if (D % 4 || H % 4 || W % 4 || cin_pad % CK || cout_pad % 32 || cin_ld % 8 || cin > cin_pad || cout > cout_pad)
        return DLCS_ERR_UNSUPPORTED_SIZE;
    ConvArgs a{};
    a.in = in; a.w = wpacked; a.bias = bias; a.out = out; a.mask = mask; a.res = residual;
    a.B = (int)B; a.D = (int)D; a.H = (int)H; a.W = (int)W; a.Cin = (int)cin; a.cin_ld = (int)cin_ld;
    a.cin_pad = (int)cin_pad; a.Cout = (int)cout; a.cout_pad = (int)cout_pad; a.cout_ld = (int)cout_ld;
    a.mask_ld = (int)mask_ld; a.res_ld = (int)res_ld; a.relu_in = relu_in; a.out_f32 = (out_dtype == DLCS_F32);
    a.res_f32 = (res_dtype == DLCS_F32); a.accumulate = accumulate; a.res_scale = res_scale;
    a.relu_out = relu_out;
    hipStream_t st = (hipStream_t)stream;
    return dtype == DLCS_F32 ? conv_launch<float>(a, st) : conv_launch<bf16>(a, st);
}

int dlcs_conv3d_k3_wgrad(int dtype, const void* in, int64_t cin, int64_t cin_ld, int64_t cin_pad, int relu_in,
                         const void* gout, int64_t cout, int64_t g_ld, int64_t cout_pad, float* dw_packed,
                         float* dbias, int64_t B, int64_t D, int64_t H, int64_t W, int64_t vox_per_block,
                         dlcs_stream_t stream) {
    DLCS_CHECK_ARG(in && gout && dw_packed && B > 0);
    if (D % 4 || H % 4 || W % 4 || cin_pad % 32 || cout_pad % 32 || cout_pad > 160 || cin_ld % 8 || g_ld % 8)
        return DLCS_ERR_UNSUPPORTED_SIZE;
    WgradArgs a{};
    a.in = in; a.g = gout; a.dw = dw_packed;
    a.B = (int)B; a.D = (int)D; a.H = (int)H; a.W = (int)W; a.Cin = (int)cin; a.cin_ld = (int)cin_ld;
    a.cin_pad = (int)cin_pad; a.Cout = (int)cout; a.g_ld = (int)g_ld; a.cout_pad = (int)cout_pad;
    a.relu_in = relu_in; a.vox_per_block = vox_per_block > 0 ? ((vox_per_block + 31) / 32) * 32 : 16384;
    hipStream_t st = (hipStream_t)stream;
    a.dbias = dbias;
    bool done = false;                            // the 160-channel bf16 kernel sums the columns itself
    const int rc = dtype == DLCS_F32 ? wgrad_launch<float>(a, st, &done) : wgrad_launch<bf16>(a, st, &done);
    if (rc || !dbias || done) return rc;
    const long rows = B * D * H * W;
    return dlcs_colsum(dtype, gout, rows, cout, g_ld, dbias, stream);
}

int dlcs_conv3d_pack_weights(int dtype, const float* w, void* packed, int64_t cout, int64_t cin,
                             int64_t rows_pad, int64_t cols_pad, int mode, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(w && packed && cout > 0 && cin > 0 && mode >= 0 && mode <= 3);
    const long n = 27L * rows_pad * cols_pad;
    hipStream_t st = (hipStream_t)stream;
    if (mode >= 2) {
#ifdef DLCS_DIAG_BUILD
        // 3-plane bf16 packing of the fp32 weights for dlcs_conv3d_k3_x6: WA then WB
        if (cout != 160 || cin != 160) return DLCS_ERR_UNSUPPORTED_SIZE;
        bf16* wa = (bf16*)packed;
        hipLaunchKernelGGL(pack_weights_x6_kernel, dim3(grid_for(27L * 160 * 160)), dim3(256), 0, st, w, wa,
                           wa + 27L * 160 * 320, mode - 2);
        return dlcs_launch_status();
#else
        return DLCS_ERR_UNSUPPORTED_SIZE;                 // the x6 packings: DIAG build only
#endif
    }
    if (dtype == DLCS_F32)
        hipLaunchKernelGGL(pack_weights_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, w, (float*)packed, (int)cout, (int)cin, (int)rows_pad, (int)cols_pad, mode);
    else
        hipLaunchKernelGGL(pack_weights_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, w, (bf16*)packed, (int)cout, (int)cin, (int)rows_pad, (int)cols_pad, mode);
    return dlcs_launch_status();
}

#ifdef DLCS_DIAG_BUILD
int dlcs_split3_bf16(const float* x, int64_t rows, int64_t ld, void* xa, void* xb, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(x && xa && xb && rows > 0 && ld >= 160);
    if (ld % 4 || ((uintptr_t)x & 15) || ((uintptr_t)xa & 15) || ((uintptr_t)xb & 15)) return DLCS_ERR_UNSUPPORTED_SIZE;
    hipLaunchKernelGGL(split3_kernel, dim3(grid_for(rows * 20)), dim3(256), 0, (hipStream_t)stream, x, (long)rows,
                       (int)ld, (bf16*)xa, (bf16*)xb);
    return dlcs_launch_status();
}

int dlcs_conv3d_k3_x6(const void* xa, const void* xb, const void* wpacked, const float* bias, float* out,
                      int64_t cout_ld, int64_t B, int64_t D, int64_t H, int64_t W, const float* mask, int64_t mask_ld,
                      const float* residual, int64_t res_ld, float res_scale, int accumulate, int relu_out,
                      dlcs_stream_t stream) {
    DLCS_CHECK_ARG(xa && xb && wpacked && out && B > 0);
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (D % 4 || H % 4 || W % 4 || cout_ld % 4 || !al16(xa) || !al16(xb) || !al16(wpacked) || !al16(out) ||
        (mask && (mask_ld % 4 || !al16(mask))) || (residual && (res_ld % 4 || !al16(residual))) || (bias && !al16(bias)) ||
        B * D * H * W * 320 >= (1L << 31))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    ConvX6Args v{};
    v.xa = (const bf16*)xa; v.xb = (const bf16*)xb; v.w = (const bf16*)wpacked; v.bias = bias; v.out = out;
    v.mask = mask; v.res = residual; v.B = (int)B; v.D = (int)D; v.H = (int)H; v.W = (int)W;
    v.cout_ld = (int)cout_ld; v.mask_ld = (int)mask_ld; v.res_ld = (int)res_ld; v.accumulate = accumulate;
    v.relu_out = relu_out; v.res_scale = res_scale;
    return conv_x6_launch(v, (hipStream_t)stream);
}

int dlcs_conv3d_k3_wgrad_x6(const void* xa, const void* xb, const void* ga, const void* gb, float* dw_packed,
                            int64_t B, int64_t D, int64_t H, int64_t W, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(xa && xb && ga && gb && dw_packed && B > 0);
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (D % 4 || H % 4 || W % 4 || !al16(xa) || !al16(xb) || !al16(ga) || !al16(gb) ||
        B * D * H * W * 320 >= (1L << 40))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    WgradX6Args v{};
    v.xa = (const bf16*)xa; v.xb = (const bf16*)xb; v.ga = (const bf16*)ga; v.gb = (const bf16*)gb;
    v.dw = dw_packed; v.B = (int)B; v.D = (int)D; v.H = (int)H; v.W = (int)W;
    return wgrad_x6_launch(v, (hipStream_t)stream);
}
#endif  // DLCS_DIAG_BUILD

// planes [rows][320] f16, the 256-B trailer (max |x| bits in its first word) and one
// 640-B zero row (the weight gradient's source for halo voxels off the grid)
size_t dlcs_split2_f16_bytes(int64_t rows) { return (size_t)rows * 640 + 256 + 640; }

int dlcs_split2_f16(const float* x, int64_t rows, int64_t ld, void* planes, int have_max, float* colsum,
                    dlcs_stream_t stream) {
    DLCS_CHECK_ARG(x && planes && rows > 0 && ld >= 160);
    if (ld % 4 || ((uintptr_t)x & 15) || ((uintptr_t)planes & 15)) return DLCS_ERR_UNSUPPORTED_SIZE;
    hipStream_t st = (hipStream_t)stream;
    unsigned* mx = (unsigned*)((char*)planes + (size_t)rows * 640);
    if (!have_max) {
        if (hipMemsetAsync(mx, 0, 4, st) != hipSuccess) return dlcs_launch_status();
        hipLaunchKernelGGL(absmax_kernel, dim3(std::min(h3_grid(rows * 10), 2048u)), dim3(256), 0, st, x, (long)rows,
                           (int)ld, mx);
    }
    // grid stride a multiple of 20 (each thread keeps one 8-channel group)
    const unsigned g = (unsigned)std::min<long>(kSplit2Blocks, std::max<long>(5, (rows * 20 + 255) / 256 / 5 * 5));
    if (colsum) {
        float* cpart = split2_colsum_workspace(st);
        if (!cpart) return (int)hipErrorOutOfMemory;
        hipLaunchKernelGGL(split2_f16_kernel<true>, dim3(g), dim3(256), 0, st, x, (long)rows, (int)ld,
                           (const unsigned*)mx, (f16*)planes, cpart);
        hipLaunchKernelGGL(colsum_parts_kernel, dim3(160), dim3(256), 0, st, (const float*)cpart, (int)g, colsum);
    } else {
        hipLaunchKernelGGL(split2_f16_kernel<false>, dim3(g), dim3(256), 0, st, x, (long)rows, (int)ld,
                           (const unsigned*)mx, (f16*)planes, nullptr);
    }
    return dlcs_launch_status();
}

size_t dlcs_conv3d_pack_weights_f16x3_bytes(void) { return (size_t)5 * 27 * 160 * 64 * 2 + 256; }

int dlcs_conv3d_pack_weights_f16x3(const float* w, int mode, void* packed, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(w && packed && (mode == 0 || mode == 1));
    if (((uintptr_t)w & 15) || ((uintptr_t)packed & 15)) return DLCS_ERR_UNSUPPORTED_SIZE;
    hipStream_t st = (hipStream_t)stream;
    unsigned* mx = (unsigned*)((char*)packed + (size_t)5 * 27 * 160 * 64 * 2);
    if (hipMemsetAsync(mx, 0, 4, st) != hipSuccess) return dlcs_launch_status();
    hipLaunchKernelGGL(absmax_kernel, dim3(h3_grid(4320L * 10)), dim3(256), 0, st, w, 4320L, 160, mx);
    hipLaunchKernelGGL(pack_weights_f16x3_kernel, dim3(h3_grid(27L * 160 * 160)), dim3(256), 0, st, w,
                       (const unsigned*)mx, (f16*)packed, mode);
    return dlcs_launch_status();
}

// column-sum partials of the producers that also sum their output's columns (the
// f16x3 conv: one row of 160 per tile; the K = 160 GEMM: per 64 x 160 tile)
static float* colsum_part_workspace(hipStream_t st, long nwg) {
    return static_cast<float*>(scratch(kScrColsum, st, (size_t)nwg * 160 * sizeof(float)));
}

int dlcs_conv3d_k3_f16x3(const void* xplanes, const void* wpacked, const float* bias, float* out, int64_t cout_ld,
                         int64_t B, int64_t D, int64_t H, int64_t W, const float* mask, int64_t mask_ld,
                         const float* residual, int64_t res_ld, float res_scale, int accumulate, int relu_out,
                         unsigned* out_max, void* out_planes, float* colsum, const void* mask_planes,
                         dlcs_stream_t stream) {
    DLCS_CHECK_ARG(xplanes && wpacked && B > 0 && (out || (out_planes && !accumulate)) && !(mask && mask_planes));
    if (!out) cout_ld = 160;
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    const long rows = (long)B * D * H * W;
    if (D % 4 || H % 4 || W % 4 || cout_ld % 4 || !al16(xplanes) || !al16(wpacked) || !al16(out) ||
        (mask && (mask_ld % 4 || !al16(mask))) || (residual && (res_ld % 4 || !al16(residual))) || (bias && !al16(bias)) ||
        rows * 320 >= (1L << 31))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    ConvH3Args v{};
    v.xp = (const f16*)xplanes; v.wp = (const f16*)wpacked;
    v.xmax = (const unsigned*)((const char*)xplanes + rows * 640);
    v.wmax = (const unsigned*)((const char*)wpacked + (size_t)5 * 27 * 160 * 64 * 2);
    v.bias = bias; v.out = out; v.mask = mask; v.res = residual;
    v.B = (int)B; v.D = (int)D; v.H = (int)H; v.W = (int)W;
    v.cout_ld = (int)cout_ld; v.mask_ld = (int)mask_ld; v.res_ld = (int)res_ld; v.accumulate = accumulate;
    v.relu_out = relu_out; v.res_scale = res_scale; v.omax = out_max;
    if (mask_planes && !al16(mask_planes)) return DLCS_ERR_UNSUPPORTED_SIZE;
    v.mplanes = mask_planes;
    if (out_planes) {
        if (cout_ld != 160 || !al16(out_planes)) return DLCS_ERR_UNSUPPORTED_SIZE;
        v.oplanes = (f16*)out_planes;
        v.opmax = (const unsigned*)((const char*)out_planes + rows * 640);
    }
#ifdef DLCS_DIAG_BUILD
    v.stamp = conv_stamps_on() ? 1 : 0;
    static const int h3_exp = [] { const char* e = dlcs_knob("DLCS_H3_EXP"); return e ? atoi(e) : 0; }();
    v.exp = h3_exp;
#endif
    hipStream_t st = (hipStream_t)stream;
    const long ntile = (long)B * (D / 4) * ((H / 4 + 1) / 2) * ((W / 4 + 1) / 2);
    if (colsum) {
        v.cpart = colsum_part_workspace(st, ntile);           // one row of 160 per tile
        if (!v.cpart) return (int)hipErrorOutOfMemory;
    }
    const int rc = conv_f16x3_launch(v, st);
    if (rc || !colsum) return rc;
    hipLaunchKernelGGL(colsum_parts_kernel, dim3(160), dim3(256), 0, st, (const float*)v.cpart, (int)ntile, colsum);
    return dlcs_launch_status();
}

int dlcs_conv3d_k3_wgrad_f16x3(const void* xplanes, const void* gplanes, float* dw_packed, int64_t B, int64_t D,
                               int64_t H, int64_t W, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(xplanes && gplanes && dw_packed && B > 0);
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    const long rows = (long)B * D * H * W;
    if (D % 4 || H % 4 || W % 4 || !al16(xplanes) || !al16(gplanes) || rows * 320 >= (1L << 40))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    WgradH3Args v{};
    v.xp = (const f16*)xplanes; v.gp = (const f16*)gplanes;
    v.xmax = (const unsigned*)((const char*)xplanes + rows * 640);
    v.gmax = (const unsigned*)((const char*)gplanes + rows * 640);
    v.dw = dw_packed; v.B = (int)B; v.D = (int)D; v.H = (int)H; v.W = (int)W;
    return wgrad_f16x3_launch(v, (hipStream_t)stream);
}

int dlcs_gemm_k160_f16x3(const void* aplanes, int64_t M, const void* bplanes, int64_t N, float* C, int64_t ldc,
                         const float* bias, int act, float alpha, const float* residual, int64_t ldr, float res_scale,
                         const float* residual2, int64_t ldr2, float res2_scale, int accumulate, unsigned* out_max,
                         void* out_planes, float* colsum, const void* res_planes, const void* res2_planes,
                         dlcs_stream_t stream) {
    DLCS_CHECK_ARG(aplanes && bplanes && M > 0 && N > 0 && (act == 0 || act == 3) &&
                   (C || (out_planes && !accumulate)) && !(residual && res_planes) && !(residual2 && res2_planes));
    if (!C) ldc = N;
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (N % 160 || ldc % 4 || !al16(aplanes) || !al16(bplanes) || !al16(C) || (bias && !al16(bias)) ||
        (residual && (ldr % 4 || !al16(residual))) || (residual2 && (ldr2 % 4 || !al16(residual2))) ||
        M * 320 >= (1L << 40))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    GemmH3Args g{};
    g.ap = (const f16*)aplanes; g.bp = (const f16*)bplanes;
    g.amax = (const unsigned*)((const char*)aplanes + M * 640);
    g.bmax = (const unsigned*)((const char*)bplanes + N * 640);
    g.c = C; g.ldc = ldc; g.bias = bias; g.act = act; g.alpha = alpha;
    g.res = residual; g.ldr = ldr; g.res_scale = res_scale;
    g.res2 = residual2; g.ldr2 = ldr2; g.res2_scale = res2_scale;
    g.accumulate = accumulate; g.M = (int)M; g.N = (int)N; g.omax = out_max;
    const long prows = M * (N / 160);                          // rows of the [M N / 160][160] view
    if (res_planes) {
        if (!al16(res_planes)) return DLCS_ERR_UNSUPPORTED_SIZE;
        g.rp = (const f16*)res_planes;
        g.rpmax = (const unsigned*)((const char*)res_planes + prows * 640);
    }
    if (res2_planes) {
        if (!al16(res2_planes)) return DLCS_ERR_UNSUPPORTED_SIZE;
        g.rp2 = (const f16*)res2_planes;
        g.rp2max = (const unsigned*)((const char*)res2_planes + prows * 640);
    }
    if (out_planes) {
        if (ldc != N || !al16(out_planes)) return DLCS_ERR_UNSUPPORTED_SIZE;
        g.oplanes = (f16*)out_planes;
        g.opmax = (const unsigned*)((const char*)out_planes + M * (N / 160) * 640);
    }
    hipStream_t st = (hipStream_t)stream;
    const long nwg = cdiv(M, 64) * (N / 160);
    if (colsum) {
        if (g.row_map || nwg > (1L << 24)) return DLCS_ERR_UNSUPPORTED_SIZE;
        g.cpart = colsum_part_workspace(st, nwg);
        if (!g.cpart) return (int)hipErrorOutOfMemory;
    }
    const int rc = gemm_k160_launch(g, st);
    if (rc || !colsum) return rc;
    hipLaunchKernelGGL(colsum_parts_kernel, dim3(160), dim3(256), 0, st, (const float*)g.cpart, (int)nwg, colsum);
    return dlcs_launch_status();
}

int dlcs_linear_k160_f16x3(const void* xplanes, int64_t M, const void* wplanes, int64_t N, float* C, int64_t ldc,
                           const float* bias, int act, const float* aux, float* aux_out, int64_t ldaux, float alpha,
                           const float* residual, int64_t ldr, const int32_t* row_map, int accumulate,
                           dlcs_stream_t stream) {
    DLCS_CHECK_ARG(xplanes && wplanes && C && M > 0 && N > 0 && act >= 0 && act <= 3 && (act != 2 || aux));
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (N % 160 || ldc % 4 || !al16(xplanes) || !al16(wplanes) || !al16(C) || (bias && !al16(bias)) ||
        (residual && (ldr % 4 || !al16(residual))) || ((aux || aux_out) && ldaux % 4) || (aux && !al16(aux)) ||
        (aux_out && !al16(aux_out)) || M * 320 >= (1L << 40))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    GemmH3Args g{};
    g.ap = (const f16*)xplanes; g.bp = (const f16*)wplanes;
    g.amax = (const unsigned*)((const char*)xplanes + M * 640);
    g.bmax = (const unsigned*)((const char*)wplanes + N * 640);
    g.c = C; g.ldc = ldc; g.bias = bias; g.act = act; g.alpha = alpha;
    g.res = residual; g.ldr = ldr; g.res_scale = 1.0f;
    g.accumulate = accumulate; g.M = (int)M; g.N = (int)N;
    g.aux = aux; g.aux_out = aux_out; g.ldaux = ldaux; g.row_map = row_map;
    return gemm_k160_launch(g, (hipStream_t)stream);
}

size_t dlcs_h3r_pack_bytes(int64_t rows, int64_t K) {
    return (size_t)rows * K * 4 + (size_t)rows * 4 + (size_t)rows * kH3rKSplit * 4 + 256;
}

int dlcs_h3r_pack_multi(int n, const float* const* src, const int64_t* ld, const int* trans, const int64_t* rows,
                        const int64_t* K, void* const* dst, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(n >= 0 && (n == 0 || (src && ld && trans && rows && K && dst)));
    for (int i0 = 0; i0 < n; i0 += kH3rPackMax) {
        H3rPackBatch bt{};
        const int cnt = std::min(n - i0, kH3rPackMax);
        int64_t maxrows = 0;
        int maxks = 1;
        for (int j = 0; j < cnt; ++j) {
            const int i = i0 + j;
            DLCS_CHECK_ARG(src[i] && dst[i] && rows[i] > 0 && K[i] > 0 && K[i] % 32 == 0 && ld[i] > 0 &&
                           ((uintptr_t)dst[i] & 15) == 0 && (trans[i] || (ld[i] % 4 == 0 && ((uintptr_t)src[i] & 15) == 0)));
            if (rows[i] > (1 << 20) || K[i] > 16384 || rows[i] * K[i] * 4 >= (1L << 31)) return DLCS_ERR_UNSUPPORTED_SIZE;
            H3rPackJob& jb = bt.j[j];
            jb.src = src[i]; jb.dst = (f16*)dst[i]; jb.inv = (float*)((char*)dst[i] + rows[i] * K[i] * 4);
            jb.part = jb.inv + rows[i];
            jb.rows = (int)rows[i]; jb.K = (int)K[i]; jb.ld = (int)ld[i]; jb.trans = trans[i];
            // K splits: at least 4 chunks of 32 per split (one per wave), at most kH3rKSplit --
            // the packing is latency-bound (16 splits of K = 10240 ran 52 us on 96 workgroups)
            jb.nks = (int)std::max<int64_t>(1, std::min<int64_t>(kH3rKSplit, K[i] / 128));
            maxrows = std::max(maxrows, rows[i]);
            maxks = std::max(maxks, jb.nks);
        }
        const dim3 grid((unsigned)cdiv(maxrows, 64), (unsigned)cnt, (unsigned)maxks);
        hipLaunchKernelGGL(h3r_rowmax_kernel, grid, dim3(256), 0, (hipStream_t)stream, bt);
        hipLaunchKernelGGL(h3r_pack_kernel, grid, dim3(256), 0, (hipStream_t)stream, bt);
        const int st = dlcs_launch_status();
        if (st) return st;
    }
    return 0;
}

// partial-tile buffer of the split-K h3r
static float* h3r_ksplit_workspace(hipStream_t st, size_t floats) {
    return static_cast<float*>(scratch(kScrH3r, st, floats * sizeof(float)));
}

int dlcs_gemm_h3r(const float* A, int64_t M, int64_t K, int64_t lda, const void* bpacked, int64_t N, float* C,
                  int64_t ldc, const float* bias, int act, const float* aux, float* aux_out, int64_t ldaux, float alpha,
                  const float* residual, int64_t ldr, const int32_t* row_map, int accumulate, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(A && bpacked && C && M > 0 && N > 0 && K > 0 && act >= 0 && act <= 7 &&
                   ((act != 2 && act != 5 && act != 6) || aux) && lda >= K);
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    // tile shape: N % 160 (the Swin Linears, the unembed input gradient) with K in
    // segments of 160, else N tiles of 128 or 64 with K in segments of 192, 128 or 64
    int nj = 0, nch = 0;
    if (N % 160 == 0 && K % 160 == 0) { nj = 5; nch = 5; }
    else if (N % 64 == 0 && K % 64 == 0) { nj = N % 128 == 0 ? 4 : 2; nch = K % 192 == 0 ? 6 : K % 128 == 0 ? 4 : 2; }
    if (!nj || lda % 4 || ldc % 4 || !al16(A) || !al16(bpacked) || !al16(C) || (bias && !al16(bias)) ||
        (residual && (ldr % 4 || !al16(residual))) || ((aux || aux_out) && ldaux % 4) || (aux && !al16(aux)) ||
        (aux_out && !al16(aux_out)) || M >= (1L << 31) || K > 16384 || N * K * 4 >= (1L << 31))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    GemmH3rArgs g{};
    g.a = A; g.lda = lda; g.M = (int)M;
    g.bp = (const f16*)bpacked; g.binv = (const float*)((const char*)bpacked + N * K * 4); g.N = (int)N;
    g.c = C; g.ldc = ldc; g.bias = bias; g.act = act; g.alpha = alpha;
    g.res = residual; g.ldr = ldr; g.row_map = row_map; g.accumulate = accumulate;
    g.aux = aux; g.aux_out = aux_out; g.ldaux = ldaux;
    g.ntn = (int)(N / (32 * nj));
    g.ntiles = (int)cdiv(M, 64) * g.ntn;
    g.nseg = (int)(K / (32 * nch));
    hipStream_t st = (hipStream_t)stream;
    // deep K with a plain epilogue (the unembed input gradient and patch-embed forward,
    // K = 10240 in 64 segments of 160 on 210 row tiles): ksplit K ranges on disjoint
    // XCD groups (8: each XCD streams its own 0.8 MB of B from its L2), raw partial
    // tiles summed in a fixed order by h3r_ksplit_reduce_kernel.  tools/embed_bench.py:
    // 272 us unsplit, 238 / 250 / 235 us at 2 / 4 / 8 ranges (x6 NT GEMM: 290 us)
    g.ksplit = 1;
    if (nj == 5 && K / 160 >= 16 && act == 0 && !row_map && !aux_out) {
        static const int ks_env = [] { const char* e = dlcs_knob("DLCS_H3R_KSPLIT"); return e ? atoi(e) : 0; }();
        const int ks = ks_env == 1 || ks_env == 2 || ks_env == 4 || ks_env == 8 ? ks_env : 8;
        if (ks > 1) {
            g.part = h3r_ksplit_workspace(st, (size_t)ks * M * N);
            if (!g.part) return (int)hipErrorOutOfMemory;
            g.ksplit = ks;
        }
    }
    g.per_xcd = (int)cdiv(g.ntiles, 8 / g.ksplit);
    const dim3 grid((unsigned)(8 * g.per_xcd)), block(512);
    if (nj == 5) {
        // K = 480 / 640 in 160-wide segments: the per-segment fold (fp32 VALU add of the
        // segment's tile) keeps the matrix core's accumulate chain at 15 MFMAs
        g.nseg = (int)(K / 160);
        if (g.nseg == 1) hipLaunchKernelGGL((gemm_h3r_kernel<5, 5, false>), grid, block, 0, st, g);
        else hipLaunchKernelGGL((gemm_h3r_kernel<5, 5, true>), grid, block, 0, st, g);
        if (g.ksplit > 1)
            hipLaunchKernelGGL(h3r_ksplit_reduce_kernel, dim3((unsigned)std::min<long>(2048, cdiv(M * N / 4, 256))),
                               dim3(256), 0, st, g);
    } else if (nj == 4) {
        if (nch == 6) hipLaunchKernelGGL((gemm_h3r_kernel<6, 4, true>), grid, block, 0, st, g);
        else if (nch == 4) hipLaunchKernelGGL((gemm_h3r_kernel<4, 4, true>), grid, block, 0, st, g);
        else hipLaunchKernelGGL((gemm_h3r_kernel<2, 4, true>), grid, block, 0, st, g);
    } else {
        if (nch == 6) hipLaunchKernelGGL((gemm_h3r_kernel<6, 2, true>), grid, block, 0, st, g);
        else if (nch == 4) hipLaunchKernelGGL((gemm_h3r_kernel<4, 2, true>), grid, block, 0, st, g);
        else hipLaunchKernelGGL((gemm_h3r_kernel<2, 2, true>), grid, block, 0, st, g);
    }
    return dlcs_launch_status();
}

int dlcs_f8r_quant(const float* x, int64_t rows, int64_t K, int64_t ld, void* q, float* inv, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(x && q && inv && rows > 0 && K > 0 && ld >= K);
    if (K % 4 || ld % 4 || ((uintptr_t)x & 15) || ((uintptr_t)q & 3) || K > (1 << 20))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    hipLaunchKernelGGL(quant_f8r_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, (hipStream_t)stream, x, (long)rows, (int)K,
                       (long)ld, (unsigned*)q, inv);
    return dlcs_launch_status();
}

int dlcs_gemm_f8r(const void* aq, const float* ainv, int64_t M, int64_t K, const void* bq, const float* binv,
                  int64_t N, float* C, int64_t ldc, const float* bias, int act, float* aux_out, int64_t ldaux,
                  float alpha, const float* residual, int64_t ldr, const int32_t* row_map, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(aq && ainv && bq && binv && C && M > 0 && N > 0 && K > 0 && (act == 0 || act == 1 || act == 4));
    if (K % 64 || N % 64 || ((uintptr_t)aq & 15) || ((uintptr_t)bq & 15) || M * K >= (1L << 40))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    GemmF8rArgs g{};
    g.a = (const unsigned char*)aq; g.ainv = ainv; g.M = (int)M;
    g.b = (const unsigned char*)bq; g.binv = binv; g.N = (int)N; g.K = (int)K;
    g.c = C; g.ldc = ldc; g.bias = bias; g.act = act; g.alpha = alpha;
    g.res = residual; g.ldr = ldr; g.row_map = row_map; g.aux_out = aux_out; g.ldaux = ldaux;
    hipLaunchKernelGGL(gemm_f8r_kernel, dim3(cdiv(M, 64), (unsigned)(N / 64)), dim3(256), 0, (hipStream_t)stream, g);
    return dlcs_launch_status();
}

size_t dlcs_conv3d_thin_pack_f16x3_bytes(int kind) {
    return (size_t)(kind == 0 ? kThinInHalfs : kThinOutHalfs) * 2 + 256;
}

int dlcs_conv3d_thin_pack_f16x3(const float* wpacked, int64_t cout, int64_t cout_pad, int64_t cin, int64_t cin_pad,
                                int kind, void* out, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(wpacked && out && (kind == 0 || kind == 1) && cout <= cout_pad && cin <= cin_pad);
    if (kind == 0 ? !(cout == 160 && cout_pad == 160 && cin >= 1 && cin <= 4)
                  : !(cin == 160 && cin_pad == 160 && cout >= 1 && cout <= 4))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    if ((uintptr_t)out & 15) return DLCS_ERR_UNSUPPORTED_SIZE;
    hipStream_t st = (hipStream_t)stream;
    const int halfs = kind == 0 ? kThinInHalfs : kThinOutHalfs;
    // max |w| word past the scale float (the buffer has 256 B of trailer)
    unsigned* mx = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(out) + (size_t)halfs * 2 + 16);
    if (hipMemsetAsync(mx, 0, 4, st) != hipSuccess) return dlcs_launch_status();
    const long n = 27L * cout_pad * cin_pad;
    hipLaunchKernelGGL(absmax_flat_kernel, dim3((unsigned)std::min<long>(64, (n / 4 + 255) / 256)), dim3(256), 0, st,
                       wpacked, n, mx);
    hipLaunchKernelGGL(pack_thin_f16x3_grid_kernel, dim3((unsigned)((halfs / 2 + 255) / 256)), dim3(256), 0, st,
                       wpacked, (int)cout, (int)cout_pad, (int)cin, (int)cin_pad, kind, (const unsigned*)mx, (f16*)out);
    return dlcs_launch_status();
}

int dlcs_abs_row_sum_max(const float* w, int64_t rows, int64_t row_stride, int64_t n_outer, int64_t outer_stride,
                         int64_t inner, unsigned* out, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(w && out && rows > 0 && rows < (1L << 31) && n_outer > 0 && inner > 0 && n_outer * inner < (1L << 31));
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(out, 0, 4, st) != hipSuccess) return dlcs_launch_status();
    if (n_outer * inner > 2048)
        hipLaunchKernelGGL(absrow_max_kernel<true>, dim3((unsigned)rows), dim3(256), 0, st, w, (int)rows,
                           (long)row_stride, (int)n_outer, (long)outer_stride, (int)inner, out);
    else
        hipLaunchKernelGGL(absrow_max_kernel<false>, dim3((unsigned)std::min<int64_t>((rows + 3) / 4, 256)), dim3(256), 0, st,
                           w, (int)rows,
                           (long)row_stride, (int)n_outer, (long)outer_stride, (int)inner, out);
    return dlcs_launch_status();
}

int dlcs_planes_bound(void* planes, int64_t rows, const unsigned* m0, const unsigned* n0, float c0,
                      const unsigned* m1, const unsigned* n1, float c1, const float* vec, int64_t nvec, float cvec,
                      dlcs_stream_t stream) {
    DLCS_CHECK_ARG(planes && rows > 0 && nvec >= 0 && nvec < (1L << 31) && (vec || nvec == 0));
    if ((uintptr_t)planes & 15) return DLCS_ERR_UNSUPPORTED_SIZE;
    hipLaunchKernelGGL(planes_bound_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream,
                       (unsigned*)((char*)planes + (size_t)rows * 640), m0, n0, c0, m1, n1, c1, vec, (int)nvec, cvec);
    return dlcs_launch_status();
}

int dlcs_absmax_f32(const float* x, int64_t n, unsigned* out, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(x && out && n >= 0);
    if ((uintptr_t)x & 15) return DLCS_ERR_UNSUPPORTED_SIZE;
    if (n == 0) return 0;
    hipLaunchKernelGGL(absmax_flat_kernel, dim3(std::min(h3_grid(n / 4 + 1), 1024u)), dim3(256), 0,
                       (hipStream_t)stream, x, (long)n, out);
    return dlcs_launch_status();
}

int dlcs_conv3d_thin_f16x3(const float* in, int64_t cin, int64_t cin_ld, const unsigned* in_max, const void* wthin,
                           const float* bias, float* out, int64_t cout, int64_t cout_ld, int64_t B, int64_t D,
                           int64_t H, int64_t W, const float* mask, int64_t mask_ld, const float* residual,
                           int64_t res_ld, float res_scale, int accumulate, int relu_out, unsigned* out_max,
                           void* out_planes, float* colsum, const void* mask_planes, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(in && in_max && wthin && B > 0 && (out || out_planes) && !(mask && mask_planes));
    if (!out) cout_ld = 160;
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    const long rows = (long)B * D * H * W;
    if (D % 4 || H % 4 || W % 4 || cin_ld % 4 || cout_ld % 4 || !al16(in) || !al16(out) || !al16(wthin) ||
        (bias && !al16(bias)) || rows * std::max(cin_ld, cout_ld) >= (1L << 31) || rows / 64 >= (1L << 24))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    const bool thin_in = cin >= 1 && cin <= 4 && cout == 160;
    const bool thin_out = cin == 160 && cout >= 1 && cout <= 4;
    if (!thin_in && !thin_out) return DLCS_ERR_UNSUPPORTED_SIZE;
    if (thin_in && ((mask && (mask_ld % 4 || !al16(mask))) || (residual && (res_ld % 4 || !al16(residual)))))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    if (thin_out && (mask || residual || out_max || cout_ld < 4)) return DLCS_ERR_UNSUPPORTED_SIZE;
    ConvF32Args v{};
    v.in = in; v.bias = bias; v.out = out; v.mask = mask; v.res = residual;
    v.B = (int)B; v.D = (int)D; v.H = (int)H; v.W = (int)W; v.cin_ld = (int)cin_ld; v.cin_pad = (int)cin;
    v.cout_ld = (int)cout_ld; v.mask_ld = (int)mask_ld; v.res_ld = (int)res_ld; v.accumulate = accumulate;
    v.relu_out = relu_out; v.res_scale = res_scale; v.cout = (int)cout; v.cout_pad = (int)cout; v.omax = out_max;
    v.mplanes = mask_planes;
    hipStream_t st = (hipStream_t)stream;
    if (!thin_in && (out_planes || colsum || mask_planes || !out)) return DLCS_ERR_UNSUPPORTED_SIZE;
    if (mask_planes && !al16(mask_planes)) return DLCS_ERR_UNSUPPORTED_SIZE;
    if (out_planes && (!al16(out_planes) || cout_ld != 160)) return DLCS_ERR_UNSUPPORTED_SIZE;
    const unsigned* opmax = out_planes ? (const unsigned*)((const char*)out_planes + rows * 640) : nullptr;
    const long ntile = (long)B * (D / 4) * ((H / 4 + 1) / 2) * ((W / 4 + 1) / 2);
    float* cpart = nullptr;
    if (colsum) {
        cpart = colsum_part_workspace(st, ntile);
        if (!cpart) return (int)hipErrorOutOfMemory;
    }
    const int rc = conv_thin_f16x3_launch(v, (const f16*)wthin, in_max, (int)cin, thin_in, st, (f16*)out_planes, opmax,
                                          cpart);
    if (rc || !colsum) return rc;
    hipLaunchKernelGGL(colsum_parts_kernel, dim3(160), dim3(256), 0, st, (const float*)cpart, (int)ntile, colsum);
    return dlcs_launch_status();
}

int dlcs_conv3d_thin_wgrad_f16x3(const float* in, int64_t cin, int64_t cin_ld, const unsigned* in_max,
                                 const float* g, int64_t cout, int64_t g_ld, const unsigned* g_max, float* dw_packed,
                                 int64_t cout_pad, int64_t cin_pad, float* colsum, int64_t B, int64_t D, int64_t H,
                                 int64_t W, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(in && in_max && g && g_max && dw_packed && B > 0 && cout <= cout_pad && cin <= cin_pad);
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    const bool thin_sfe = cout == 160 && cin >= 1 && cin <= 4;
    const bool thin_fin = cin == 160 && cout >= 1 && cout <= 4;
    const long npatch = B * (D / 4) * (H / 4) * (W / 4);
    if ((!thin_sfe && !thin_fin) || (colsum && !thin_sfe) || D % 4 || H % 4 || W % 4 || cin_ld % 4 || g_ld % 4 ||
        !al16(in) || !al16(g) || npatch >= (1L << 24))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    ThinWgH3Args t{};
    t.big = thin_sfe ? g : in;
    t.thin = thin_sfe ? in : g;
    t.big_max = thin_sfe ? g_max : in_max;
    t.thin_max = thin_sfe ? in_max : g_max;
    t.dw = dw_packed; t.colsum = colsum;
    t.big_ld = (int)(thin_sfe ? g_ld : cin_ld); t.thin_ld = (int)(thin_sfe ? cin_ld : g_ld);
    t.sgn = thin_sfe ? 1 : -1; t.big_is_co = thin_sfe; t.thin_ch = (int)(thin_sfe ? cin : cout);
    t.cout_pad = (int)cout_pad; t.cin_pad = (int)cin_pad;
    t.B = (int)B; t.D = (int)D; t.H = (int)H; t.W = (int)W;
    const int nr = (int)std::min<long>(256, npatch);
    const int pp = (int)((npatch + nr - 1) / nr);
    hipLaunchKernelGGL(conv3d_wgrad_thin_f16x3_kernel, dim3(nr), dim3(512), 0, (hipStream_t)stream, t, nr, pp);
    return dlcs_launch_status();
}

int dlcs_conv3d_thin_out_planes_f16x3(const void* xplanes, const void* wthin, const float* bias, float* out,
                                      int64_t cout, int64_t cout_ld, int64_t B, int64_t D, int64_t H, int64_t W,
                                      int accumulate, int relu_out, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(xplanes && wthin && out && B > 0 && cout >= 1 && cout <= 4 && cout_ld >= 4);
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (D % 4 || H % 4 || W % 4 || cout_ld % 4 || !al16(xplanes) || !al16(wthin) || !al16(out))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    ConvF32Args v{};
    v.bias = bias; v.out = out;
    v.B = (int)B; v.D = (int)D; v.H = (int)H; v.W = (int)W;
    v.cout_ld = (int)cout_ld; v.accumulate = accumulate; v.relu_out = relu_out; v.cout = (int)cout;
    v.cout_pad = (int)cout;
    return conv_thin_out_p_launch(v, (const f16*)xplanes, (const f16*)wthin, (hipStream_t)stream);
}

int dlcs_conv3d_thin_wgrad_planes_f16x3(const void* bigplanes, const float* thin, int64_t thin_ch, int64_t thin_ld,
                                        const unsigned* thin_max, int big_is_co, float* dw_packed, int64_t cout_pad,
                                        int64_t cin_pad, int64_t B, int64_t D, int64_t H, int64_t W,
                                        dlcs_stream_t stream) {
    DLCS_CHECK_ARG(bigplanes && thin && thin_max && dw_packed && B > 0 && thin_ch >= 1 && thin_ch <= 4 &&
                   thin_ld >= 4);
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (D % 4 || H % 4 || W % 4 || thin_ld % 4 || !al16(bigplanes) || !al16(thin) ||
        (big_is_co ? (cout_pad < 160 || cin_pad < thin_ch) : (cin_pad < 160 || cout_pad < thin_ch)))
        return DLCS_ERR_UNSUPPORTED_SIZE;
    ThinWgPArgs t{};
    t.bp = (const f16*)bigplanes; t.thin = thin; t.dw = dw_packed; t.thin_max = thin_max;
    t.rows = (long)B * D * H * W;
    t.thin_ld = (int)thin_ld; t.sgn = big_is_co ? 1 : -1; t.big_is_co = big_is_co ? 1 : 0; t.thin_ch = (int)thin_ch;
    t.cout_pad = (int)cout_pad; t.cin_pad = (int)cin_pad;
    t.B = (int)B; t.D = (int)D; t.H = (int)H; t.W = (int)W;
    return wgrad_thin_p_launch(t, (hipStream_t)stream);
}

int dlcs_conv3d_unpack_wgrad(const float* dw_packed, float* grad, int64_t cout, int64_t cin, int64_t cout_pad,
                             int64_t cin_pad, int accumulate, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(dw_packed && grad && cout > 0 && cin > 0);
    hipLaunchKernelGGL(unpack_wgrad_kernel, dim3(grid_for(cout * cin * 27)), dim3(256), 0, (hipStream_t)stream,
                       dw_packed, grad, (int)cout, (int)cin, (int)cout_pad, (int)cin_pad, accumulate);
    return dlcs_launch_status();
}

}  // extern "C"
