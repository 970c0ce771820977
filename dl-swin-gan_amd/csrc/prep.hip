// Cine preprocessing on the GPU: the per-voxel parts of
// CinePreprocess (preprocess.py:54-180) and of reconstruct.py's DataTransform
// (reconstruct.py:114-152) that the reference runs on CPU DataLoader workers.
// The 2-D FFTs and the SENSE adjoints of those paths are dlcs_fft2 /
// dlcs_sense_adj; the host keeps only the random choices (crop centres, flips,
// the VDkt mask), so the RNG stream matches the reference's.
//
//   dlcs_kt_window_average  time_average / sliding_window over the T axis of
//                           complex k-space (ut:29-49, get_mask ut:69-79)
//   dlcs_kth_largest_abs    k-th largest |x| (torch.topk(...).values.min(),
//                           preprocess.py:149-153) by an in-LDS radix select
//   dlcs_cplx_mask_scale    y = x * mask / scale with the scale read on the
//                           device (preprocess.py:146, :156-157)
//   dlcs_crop_flip          crop + flips of complex volumes (preprocess.py:59-120)
//
// All memory-bound: one read and one write of each complex element, 8-B
// accesses along the contiguous Y*X axis.
#include "dlcs_common.h"

namespace {

// one thread per (plane p, pixel yx); loops over the T frames of its column
__global__ void kt_window_kernel(const float2* __restrict__ k, float2* __restrict__ out, long P, int T, long YX,
                                 int window, int full) {
    const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (i >= P * YX) return;
    const long p = i / YX, yx = i - p * YX;
    const float2* col = k + p * T * YX + yx;
    if (full) {                                     // time_average over all T frames (keepdim)
        float sr = 0.0f, si = 0.0f, cnt = 0.0f;
        for (int t = 0; t < T; ++t) {
            const float2 v = col[(long)t * YX];
            sr += v.x; si += v.y;
            cnt += (hypotf(v.x, v.y) > 1e-12f) ? 1.0f : 0.0f;
        }
        const float d = cnt + 1e-6f;
        out[p * YX + yx] = make_float2(sr / d, si / d);
        return;
    }
    // sliding window with circular boundary: frame t averages frames
    // (t - window / 2 + j) mod T, j = 0 .. window - 1 (ut:37-49)
    const int h = window / 2;
    for (int t = 0; t < T; ++t) {
        float sr = 0.0f, si = 0.0f, cnt = 0.0f;
        for (int j = 0; j < window; ++j) {
            int s = t - h + j;
            s = ((s % T) + T) % T;
            const float2 v = col[(long)s * YX];
            sr += v.x; si += v.y;
            cnt += (hypotf(v.x, v.y) > 1e-12f) ? 1.0f : 0.0f;
        }
        const float d = cnt + 1e-6f;
        out[p * T * YX + (long)t * YX + yx] = make_float2(sr / d, si / d);
    }
}

// |x| rounded once to float from the exact double-precision value (re^2 and im^2
// are exact in double): the correctly rounded hypot that the reference's CPU
// torch.abs returns, so the selected magnitude is bit-identical.
DLCS_DEV float cabs_rn(float2 v) {
    return (float)sqrt((double)v.x * (double)v.x + (double)v.y * (double)v.y);
}

// k-th largest |x| of n complex values: 4 passes of an 8-bit radix select on the
// IEEE bits of |x| (non-negative floats order as unsigned integers), one
// workgroup, 256-bin LDS histogram per pass.
__global__ void __launch_bounds__(1024) kth_largest_abs_kernel(const float2* __restrict__ x, long n, long k,
                                                               float* __restrict__ out) {
    __shared__ unsigned hist[256];
    __shared__ unsigned prefix_s, remain_s;
    if (threadIdx.x == 0) { prefix_s = 0u; remain_s = (unsigned)k; }
    unsigned himask = 0u;
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int b = threadIdx.x; b < 256; b += blockDim.x) hist[b] = 0u;
        __syncthreads();
        const unsigned prefix = prefix_s;
        for (long i = threadIdx.x; i < n; i += blockDim.x) {
            const float2 v = x[i];
            const unsigned key = __float_as_uint(cabs_rn(v));
            if ((key & himask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned rem = remain_s, bin = 0;
            for (int b = 255; b >= 0; --b) {
                if (hist[b] >= rem) { bin = (unsigned)b; break; }
                rem -= hist[b];
            }
            remain_s = rem;
            prefix_s = prefix | (bin << shift);
        }
        himask |= 255u << shift;
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = __uint_as_float(prefix_s);
}

// y[p, t, yx] = x[p, t, yx] * (mask ? mask[p % mask_planes or 0, t, yx] : 1) / scale[0]
__global__ void cplx_mask_scale_kernel(const float2* __restrict__ x, const float* __restrict__ mask, float2* y,
                                       long P, long TYX, long mask_planes, const float* __restrict__ scale,
                                       int divide) {
    const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (i >= P * TYX) return;
    float f = 1.0f;
    if (mask) {
        const long p = i / TYX, r = i - p * TYX;
        f = mask[(mask_planes > 1 ? p % mask_planes : 0) * TYX + r];
    }
    float2 v = x[i];
    if (scale) {
        const float s = scale[0];
        if (divide) { v.x = v.x / s; v.y = v.y / s; }
        else { v.x *= s; v.y *= s; }
    }
    y[i] = make_float2(v.x * f, v.y * f);
}

// out[p, t, y, x] = in[p, ft(t), y0 + fy(y), x0 + fx(x)] on the cropped extent,
// f*(i) = n - 1 - i when flipped
__global__ void crop_flip_kernel(const float2* __restrict__ in, float2* __restrict__ out, long P, int T, int Y,
                                 int X, int y0, int ny, int x0, int nx, int flip_t, int flip_y, int flip_x) {
    const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    const long total = P * T * (long)ny * nx;
    if (i >= total) return;
    const int xo = (int)(i % nx);
    long r = i / nx;
    const int yo = (int)(r % ny); r /= ny;
    const int to = (int)(r % T);
    const long p = r / T;
    const int ti = flip_t ? T - 1 - to : to;
    const int yi = y0 + (flip_y ? ny - 1 - yo : yo);
    const int xi = x0 + (flip_x ? nx - 1 - xo : xo);
    out[i] = in[((p * T + ti) * (long)Y + yi) * X + xi];
}

unsigned grid1(long n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

extern "C" {

int dlcs_kt_window_average(const void* k, void* out, int64_t P, int64_t T, int64_t YX, int64_t window,
                           int full, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(k && out && P > 0 && T > 0 && YX > 0 && (full || (window > 0 && window <= T)));
    hipLaunchKernelGGL(kt_window_kernel, dim3(grid1(P * YX, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const float2*)k, (float2*)out, (long)P, (int)T, (long)YX, (int)window, full);
    return dlcs_launch_status();
}

int dlcs_kth_largest_abs(const void* x, int64_t n, int64_t k, float* out, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(x && out && n > 0 && k >= 1 && k <= n && n < (1LL << 32));
    hipLaunchKernelGGL(kth_largest_abs_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, (const float2*)x,
                       (long)n, (long)k, out);
    return dlcs_launch_status();
}

int dlcs_cplx_mask_scale(const void* x, const float* mask, void* y, int64_t P, int64_t TYX, int64_t mask_planes,
                         const float* scale, int divide, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(x && y && P > 0 && TYX > 0);
    hipLaunchKernelGGL(cplx_mask_scale_kernel, dim3(grid1(P * TYX, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const float2*)x, mask, (float2*)y, (long)P, (long)TYX, (long)mask_planes, scale, divide);
    return dlcs_launch_status();
}

int dlcs_crop_flip(const void* in, void* out, int64_t P, int64_t T, int64_t Y, int64_t X, int64_t y0, int64_t ny,
                   int64_t x0, int64_t nx, int flip_t, int flip_y, int flip_x, dlcs_stream_t stream) {
    DLCS_CHECK_ARG(in && out && P > 0 && T > 0 && ny > 0 && nx > 0 && y0 >= 0 && x0 >= 0 && y0 + ny <= Y &&
                   x0 + nx <= X);
    hipLaunchKernelGGL(crop_flip_kernel, dim3(grid1(P * T * ny * nx, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const float2*)in, (float2*)out, (long)P, (int)T, (int)Y, (int)X, (int)y0, (int)ny, (int)x0,
                       (int)nx, flip_t, flip_y, flip_x);
    return dlcs_launch_status();
}

}  // extern "C"
