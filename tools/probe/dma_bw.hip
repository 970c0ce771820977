// Global -> LDS DMA throughput (global_load_lds_dwordx4, the saddr form the conv /
// GEMM kernels use) and, for comparison, global_load_dwordx4 into registers: 256
// workgroups (one per CU) of NW waves stream 48-KB "units" from a buffer of S bytes
// into a 2-slot LDS ring (wait vmcnt(0) + barrier per unit, no compute), for S that
// sits in L2 (2 MB), in the MALL (128 MB) or in HBM (2 GB).  Prints TB/s.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/dma_bw.hip -o tools/probe/dma_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kUnit = 48 * 1024;                       // bytes per unit (48 pieces of 1 KB)

__device__ inline void glds16_s(const void* sbase, unsigned voff, unsigned lds_addr) {
    unsigned saved;
    const unsigned long long sb = (unsigned long long)(uintptr_t)sbase;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)sb);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(sb >> 32));
    const unsigned long long sbu = ((unsigned long long)hi << 32) | lo;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 4\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(saved) : "v"(voff), "s"(sbu), "s"(__builtin_amdgcn_readfirstlane(lds_addr)) : "memory");
}

// mode 0: LDS DMA; mode 1: register loads (summed so they are not dead)
template <int MODE>
__global__ void __launch_bounds__(512) dma_kernel(const char* buf, long nunits_buf, int units, float* sink) {
    __shared__ __attribute__((aligned(16))) char lds[2 * kUnit];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    const unsigned l0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)lds);
    float acc = 0.0f;
    // workgroup b walks units b, b + grid, ... (mod the buffer's unit count)
    for (int u = 0; u < units; ++u) {
        const long uu = ((long)u * gridDim.x + blockIdx.x) % nunits_buf;
        const char* src = buf + uu * kUnit;
        if (MODE == 0) {
            for (int p = wave; p < kUnit / 1024; p += nw)
                glds16_s(src, (unsigned)(p * 1024 + lane * 16), l0 + (unsigned)((u & 1) * kUnit + p * 1024));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        } else {
            float4 v[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const int p = wave + k * nw;
                v[k] = p < kUnit / 1024 ? *reinterpret_cast<const float4*>(src + p * 1024 + lane * 16) : make_float4(0, 0, 0, 0);
            }
#pragma unroll
            for (int k = 0; k < 6; ++k) acc += v[k].x + v[k].w;
        }
    }
    if (MODE == 0) acc = reinterpret_cast<const float*>(lds)[threadIdx.x];
    if (acc == 1234.5f) sink[threadIdx.x] = acc;
}

int main() {
    const long maxb = 2L << 30;
    char* buf;
    float* sink;
    if (hipMalloc(&buf, maxb) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess) return 1;
    hipMemset(buf, 1, maxb);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const long sizes[3] = {2L << 20, 128L << 20, 2L << 30};
    const char* names[3] = {"L2 (2 MB)", "MALL (128 MB)", "HBM (2 GB)"};
    for (int nw : {4, 8}) {
        for (int mode = 0; mode < 2; ++mode) {
            for (int si = 0; si < 3; ++si) {
                const long nub = sizes[si] / kUnit;
                const int units = 200;
                auto launch = [&]() {
                    if (mode == 0) hipLaunchKernelGGL(dma_kernel<0>, dim3(256), dim3(64 * nw), 0, 0, buf, nub, units, sink);
                    else hipLaunchKernelGGL(dma_kernel<1>, dim3(256), dim3(64 * nw), 0, 0, buf, nub, units, sink);
                };
                launch();
                hipDeviceSynchronize();
                hipEventRecord(e0);
                for (int it = 0; it < 5; ++it) launch();
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                const double bytes = 5.0 * 256 * units * (double)kUnit;
                printf("%-14s waves %d  %-10s %7.2f TB/s  (%.1f B/clk/CU at 2.1 GHz)\n", mode == 0 ? "LDS-DMA" : "reg-load",
                       nw, names[si], bytes / (ms * 1e-3) / 1e12, bytes / (ms * 1e-3) / 256 / 2.1e9);
            }
        }
    }
    const hipError_t err = hipGetLastError();
    printf("status %s\n", hipGetErrorString(err));
    return err == hipSuccess ? 0 : 2;
}
