// Common device helpers for libdlcs_hip (gfx950 / CDNA4 only).
//
// Storage types: float (fp32 parity build) and __bf16 (fast path); every
// kernel accumulates in fp32.  MFMA access goes through the Mfma32<T>
// wrapper below, which gives both dtypes ONE fragment convention:
//   lane l (r = l & 31, h = l >> 5) holds 8 consecutive k of its row/column,
//   k = 8h + j, j = 0..7   (one k16 step of a 32x32 output tile)
// bf16: one v_mfma_f32_32x32x16_bf16 consumes the 8 elements.
// f32 : eight v_mfma_f32_32x32x2_f32, the j-th contracting k = {j, 8 + j}
//       (the f32 form sums over lane halves), so A and B use the same
//       permutation of k and the contraction is exact f32 FMA chains.
// C/D map (both): col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/dlcs.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));

#define DLCS_DEV __device__ __forceinline__

DLCS_DEV float to_f(float v) { return v; }
DLCS_DEV float to_f(bf16 v) { return (float)v; }
template <typename T> DLCS_DEV T from_f(float v);
template <> DLCS_DEV float from_f<float>(float v) { return v; }
template <> DLCS_DEV bf16 from_f<bf16>(float v) { return (bf16)v; }

// 8 consecutive elements of T, held as a register fragment.
template <typename T> struct Frag8;
template <> struct Frag8<bf16> { bf16x8 v; };
template <> struct Frag8<float> { f32x8 v; };

template <typename T> DLCS_DEV Frag8<T> load8(const T* p);
template <> DLCS_DEV Frag8<bf16> load8<bf16>(const bf16* p) {
    Frag8<bf16> f; f.v = *reinterpret_cast<const bf16x8*>(p); return f;
}
template <> DLCS_DEV Frag8<float> load8<float>(const float* p) {
    Frag8<float> f; f.v = *reinterpret_cast<const f32x8*>(p); return f;
}
template <typename T> DLCS_DEV Frag8<T> zero8();
template <> DLCS_DEV Frag8<bf16> zero8<bf16>() { Frag8<bf16> f; f.v = (bf16x8)(bf16)0.0f; return f; }
template <> DLCS_DEV Frag8<float> zero8<float>() { Frag8<float> f; f.v = (f32x8)0.0f; return f; }

DLCS_DEV void mfma32(f32x16& acc, const Frag8<bf16>& a, const Frag8<bf16>& b) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v, b.v, acc, 0, 0, 0);
}
DLCS_DEV void mfma32(f32x16& acc, const Frag8<float>& a, const Frag8<float>& b) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.v[j], b.v[j], acc, 0, 0, 0);
}

// row of element `reg` of a 32x32 accumulator held by lane `lane`
DLCS_DEV int acc_row(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }

DLCS_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
DLCS_DEV float gelu_erf_grad(float x) {
    const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
    const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
    return cdf + x * pdf;
}

// GELU, tanh approximation (torch approximate='tanh'; the DiT Mlp, dit:322-323)
DLCS_DEV float gelu_tanh(float x) {
    const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
    return 0.5f * x * (1.0f + tanhf(u));
}
DLCS_DEV float gelu_tanh_grad(float x) {
    const float x2 = x * x;
    const float t = tanhf(0.7978845608028654f * (x + 0.044715f * x2 * x));
    return 0.5f * (1.0f + t) + 0.5f * x * (1.0f - t * t) * 0.7978845608028654f * (1.0f + 3.0f * 0.044715f * x2);
}
// GEMM epilogue activations (dlcs_gemm act codes): 1 GELU(erf), 4 GELU(tanh) --
// pre-activation to aux_out; 2 / 5 / 6: times gelu_erf' / gelu_tanh' / (aux > 0) of
// aux (the backward of acts 1 / 4 and of a ReLU); 3 ReLU before the residuals;
// 7 ReLU after the residuals
DLCS_DEV float act_fwd(int act, float v) {
    return act == 1 ? gelu_erf(v) : act == 4 ? gelu_tanh(v) : act == 3 ? fmaxf(v, 0.0f) : v;
}
DLCS_DEV float act_grad_scale(int act, float a) {
    return act == 2 ? gelu_erf_grad(a) : act == 5 ? gelu_tanh_grad(a) : (a > 0.0f ? 1.0f : 0.0f);
}
DLCS_DEV bool act_is_fwd(int act) { return act == 1 || act == 3 || act == 4; }
DLCS_DEV bool act_is_grad(int act) { return act == 2 || act == 5 || act == 6; }

DLCS_DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// max of lanes l and l ^ 32 (l ^ 16): v_permlane32_swap / v_permlane16_swap, VALU
// instead of __shfl_xor's ds_bpermute round trip through the LDS (a max is exact, so
// the result is the same bits in any lane order)
DLCS_DEV float xor32_max(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// v_permlane32_swap(v, v) gives r[0] = lanes 0..31's value and r[1] = lanes 32..63's
// in both halves: the value of lane l ^ 32, and v + that value (a two-term sum is
// commutative, so the same bits as v + __shfl_xor(v, 32))
DLCS_DEV float xor32_peer(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float((__lane_id() & 32) ? r[0] : r[1]);
}
DLCS_DEV float xor32_sum(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
DLCS_DEV float xor16_max(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// max / sum over the 8 consecutive lanes 8k .. 8k + 7 (DPP quad_perm xor 1, xor 2, then
// row_half_mirror, which pairs each lane of one quad with one of the other): the same
// operands in the same order as the xor-1 / 2 / 4 shuffles, so the same bits
DLCS_DEV float lane8_max(float v) {
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));
    return fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)));
}
DLCS_DEV float lane8_sum(float v) {
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
}
// max over the wave: DPP within 16-lane rows (quad_perm xor 1 / xor 2, row_half_mirror,
// row_mirror: each step pairs every lane with one holding the other half of its group),
// then the row swaps -- no LDS instruction
DLCS_DEV float wave_max(float v) {
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false)));
    return xor32_max(xor16_max(v));
}

static inline int dlcs_launch_status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

static inline unsigned cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }

// Diagnostic switches (superseded kernels kept for A/B measurement, tuning
// overrides, stamps) exist only in the DIAG build (`make DIAG=1` ->
// libdlcs_hip_diag.so, which also holds the superseded bf16 3-plane conv and NT
// GEMM); there they are read under DLCS_DIAG=1.  The product library compiles
// every knob to "unset": one path per op.
static inline const char* dlcs_knob(const char* name) {
#ifdef DLCS_DIAG_BUILD
    const char* d = getenv("DLCS_DIAG");
    return d && d[0] == '1' ? getenv(name) : nullptr;
#else
    (void)name;
    return nullptr;
#endif
}
// Test hooks that pick between two equivalent schedules of the SAME kernel (the
// f16x3 conv's tail split), read in either build under DLCS_DIAG=1.
static inline const char* dlcs_test_hook(const char* name) {
    const char* d = getenv("DLCS_DIAG");
    return d && d[0] == '1' ? getenv(name) : nullptr;
}

#define DLCS_CHECK_ARG(cond) do { if (!(cond)) return DLCS_ERR_INVALID_ARG; } while (0)
