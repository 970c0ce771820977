"""ctypes binding of libdlcs_hip.so (the C-ABI declared in include/dlcs.h).

The product path has no CPU fallback: if the library is missing, or a tensor is
not on the GPU, the ops raise.  torch is imported first so that the process
shares torch's HIP runtime (libamdhip64.so.7) with the library.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DLCS_HIP_LIB", os.path.join(_HERE, "libdlcs_hip.so"))

F32, BF16 = 0, 1
_LIB = None

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_INT = ctypes.c_int
_F = ctypes.c_float
_SZ = ctypes.c_size_t

# name -> argtypes (restype is int unless listed in _RESTYPE)
SIGNATURES = {
    "dlcs_version": [],
    "dlcs_status_string": [_INT],
    "dlcs_scratch_bytes": [],
    "dlcs_release_scratch": [],
    "dlcs_sense_workspace_bytes": [_I64, _I64, _I64, _I64, _I64],
    "dlcs_sense_fwd": [_P, _P, _P, _I64, _P, _I64, _I64, _I64, _I64, _I64, _I64, _P, _SZ, _P],
    "dlcs_sense_adj": [_P, _P, _P, _I64, _P, _P, _P, _F, _I64, _I64, _I64, _I64, _I64, _I64, _P, _SZ, _P],
    "dlcs_sense_normal": [_P, _P, _P, _I64, _P, _P, _F, _F, _I64, _I64, _I64, _I64, _I64, _I64, _P, _SZ, _P],
    "dlcs_sense_cg_workspace_bytes": [_I64] * 6,
    "dlcs_sense_cg": [_P, _P, _P, _P, _I64, _F, _INT, _I64, _I64, _I64, _I64, _I64, _I64, _P, _SZ, _P],
    "dlcs_sense_rowtab_bytes": [_I64] * 4,
    "dlcs_sense_rowtab": [_P, _I64, _I64, _I64, _I64, _I64, _P, _SZ, _P],
    "dlcs_sense_rows_workspace_bytes": [_I64] * 5,
    "dlcs_sense_adj_rows": [_P, _P, _P, _I64, _P, _I64, _P, _P, _P, _F, _I64, _I64, _I64, _I64, _I64, _I64, _P,
                            _SZ, _P],
    "dlcs_sense_normal_rows": [_P, _P, _P, _I64, _P, _I64, _P, _P, _F, _F, _I64, _I64, _I64, _I64, _I64, _I64, _P,
                               _SZ, _P],
    "dlcs_sense_cg_rows": [_P, _P, _P, _P, _I64, _P, _I64, _F, _INT, _I64, _I64, _I64, _I64, _I64, _I64, _P, _SZ, _P],
    "dlcs_fft2": [_P, _P, _I64, _I64, _I64, _INT, _P, _SZ, _P],
    "dlcs_window_index": [_I64] * 10 + [_P, _P, _P, _P],
    "dlcs_gather_rows": [_INT, _INT, _P, _P, _P, _I64, _I64, _I64, _I64, _P],
    "dlcs_layernorm_fwd": [_INT, _P, _P, _P, _P, _F, _P, _P, _P, _I64, _I64, _P],
    "dlcs_layernorm_bwd_workspace_bytes": [_I64, _I64],
    "dlcs_layernorm_bwd": [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _P, _SZ, _P],
    "dlcs_colsum": [_INT, _P, _I64, _I64, _I64, _P, _P],
    "dlcs_gemm": [_INT, _I64, _I64, _I64, _P, _I64, _INT, _P, _I64, _INT, _P, _I64, _INT,
                  _P, _INT, _P, _P, _I64, _F, _P, _I64, _INT, _F, _P, _I64, _INT, _F, _P, _INT, _INT, _P],
    "dlcs_gemm_dw_workspace_bytes": [_INT, _P, _P, _I64],
    "dlcs_gemm_dw_grouped": [_INT, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _P, _SZ, _P],
    "dlcs_gemm_dw_grouped_f32": [_INT, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _P, _SZ, _P],
    "dlcs_window_attn_fwd": [_INT, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64,
                             _I64, _I64, _I64, _F, _P],
    "dlcs_window_attn_bwd": [_INT, _P, _P, _P, _P, _P, _P, _P, _I64, _P, _P, _I64, _I64, _I64, _I64,
                             _I64, _I64, _I64, _F, _P],
    "dlcs_conv3d_k3": [_INT, _P, _I64, _I64, _P, _I64, _P, _P, _INT, _I64, _I64, _I64, _I64, _I64, _I64,
                       _I64, _INT, _P, _I64, _P, _INT, _I64, _F, _INT, _INT, _P],
    "dlcs_conv3d_k3_wgrad": [_INT, _P, _I64, _I64, _I64, _INT, _P, _I64, _I64, _I64, _P, _P, _I64, _I64, _I64,
                             _I64, _I64, _P],
    "dlcs_conv3d_pack_weights": [_INT, _P, _P, _I64, _I64, _I64, _I64, _INT, _P],
    "dlcs_conv3d_unpack_wgrad": [_P, _P, _I64, _I64, _I64, _I64, _INT, _P],
    "dlcs_split2_f16_bytes": [_I64],
    "dlcs_split2_f16": [_P, _I64, _I64, _P, _INT, _P, _P],
    "dlcs_conv3d_pack_weights_f16x3_bytes": [],
    "dlcs_conv3d_pack_weights_f16x3": [_P, _INT, _P, _P],
    "dlcs_gemm_k160_f16x3": [_P, _I64, _P, _I64, _P, _I64, _P, _INT, _F, _P, _I64, _F, _P, _I64, _F, _INT, _P, _P, _P,
                             _P, _P, _P],
    "dlcs_planes_bound": [_P, _I64, _P, _P, _F, _P, _P, _F, _P, _I64, _F, _P],
    "dlcs_abs_row_sum_max": [_P, _I64, _I64, _I64, _I64, _I64, _P, _P],
    "dlcs_h3r_pack_bytes": [_I64, _I64],
    "dlcs_h3r_pack_multi": [_INT, _P, _P, _P, _P, _P, _P, _P],
    "dlcs_gemm_h3r": [_P, _I64, _I64, _I64, _P, _I64, _P, _I64, _P, _INT, _P, _P, _I64, _F, _P, _I64, _P, _INT, _P],
    "dlcs_f8r_quant": [_P, _I64, _I64, _I64, _P, _P, _P],
    "dlcs_gemm_f8r": [_P, _P, _I64, _I64, _P, _P, _I64, _P, _I64, _P, _INT, _P, _I64, _F, _P, _I64, _P, _P],
    "dlcs_linear_k160_f16x3": [_P, _I64, _P, _I64, _P, _I64, _P, _INT, _P, _P, _I64, _F, _P, _I64, _P, _INT, _P],
    "dlcs_gemm_f32_splitk_det": [_P, _I64, _P, _I64, _I64, _I64, _I64, _P, _P, _SZ, _P],
    "dlcs_gemm_f32_splitk_det_workspace_bytes": [_I64, _I64],
    "dlcs_conv3d_k3_wgrad_f16x3": [_P, _P, _P, _I64, _I64, _I64, _I64, _P],
    "dlcs_conv3d_k3_f16x3": [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _P, _I64, _P, _I64, _F, _INT, _INT, _P, _P, _P,
                             _P, _P],
    "dlcs_conv3d_thin_pack_f16x3_bytes": [_INT],
    "dlcs_conv3d_thin_pack_f16x3": [_P, _I64, _I64, _I64, _I64, _INT, _P, _P],
    "dlcs_absmax_f32": [_P, _I64, _P, _P],
    "dlcs_conv3d_thin_f16x3": [_P, _I64, _I64, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _P, _I64, _P,
                               _I64, _F, _INT, _INT, _P, _P, _P, _P, _P],
    "dlcs_conv3d_thin_out_planes_f16x3": [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _INT, _INT, _P],
    "dlcs_conv3d_thin_wgrad_planes_f16x3": [_P, _P, _I64, _I64, _P, _INT, _P, _I64, _I64, _I64, _I64, _I64, _I64,
                                            _P],
    "dlcs_conv3d_thin_wgrad_f16x3": [_P, _I64, _I64, _P, _P, _I64, _I64, _P, _P, _I64, _I64, _P, _I64, _I64, _I64,
                                     _I64, _P],
    "dlcs_swin_pre": [_INT, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _P],
    "dlcs_swin_pre_bwd": [_INT, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _P],
    "dlcs_swin_post": [_INT, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _P],
    "dlcs_swin_post_bwd": [_INT, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _P],
    "dlcs_axpby": [_INT, _INT, _P, _P, _I64, _F, _F, _P],
    "dlcs_relu_grad": [_INT, _P, _INT, _P, _I64, _P],
    "dlcs_permute": [_INT, _INT, _P, _P, _I64, _P, _P, _INT, _P],
    "dlcs_fill_bias": [_P, _P, _I64, _I64, _I64, _P],
    "dlcs_block_layout": [_INT, _INT, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _INT, _P],
    "dlcs_cast_multi_bf16": [_I64, _P, _P, _P, _P],
    "dlcs_kt_window_average": [_P, _P, _I64, _I64, _I64, _I64, _INT, _P],
    "dlcs_kth_largest_abs": [_P, _I64, _I64, _P, _P],
    "dlcs_cplx_mask_scale": [_P, _P, _P, _I64, _I64, _I64, _P, _INT, _P],
    "dlcs_crop_flip": [_P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _INT, _INT, _INT, _P],
    # DiT denoiser (dit.hip)
    "dlcs_mhsa_fwd": [_INT, _P, _P, _P, _I64, _I64, _I64, _I64, _F, _P],
    "dlcs_mhsa_bwd_workspace_bytes": [_I64, _I64, _I64],
    "dlcs_mhsa_bwd": [_INT, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _F, _P, _SZ, _P],
    "dlcs_conv3d_thin_im2col": [_P, _I64, _I64, _P, _I64, _INT, _I64, _I64, _I64, _I64, _P],
    "dlcs_conv3d_thin_col2im": [_P, _I64, _I64, _P, _I64, _P, _INT, _INT, _I64, _I64, _I64, _I64, _P],
    "dlcs_dit_vec": [_INT, _P, _P, _P, _I64, _P],
    "dlcs_timestep_embedding": [_P, _I64, _I64, _F, _P, _P],
    "dlcs_scale_rows": [_P, _P, _P, _P, _P, _I64, _I64, _P],
    "dlcs_gated_linear_grad": [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _P],
    "dlcs_rows_add": [_P, _P, _P, _I64, _I64, _P],
}
# DIAG build only (libdlcs_hip_diag.so: the superseded bf16 3-plane conv and NT GEMM);
# bound when the loaded library has them
DIAG_SIGNATURES = {
    "dlcs_conv3d_k3_x6": [_P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _P, _I64, _P, _I64, _F, _INT,
                          _INT, _P],
    "dlcs_split3_bf16": [_P, _I64, _I64, _P, _P, _P],
    "dlcs_conv3d_k3_wgrad_x6": [_P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _P],
    "dlcs_gemm_nt_x6": [_P, _I64, _P, _I64, _I64, _I64, _I64, _P, _P, _SZ, _P],
    "dlcs_gemm_nt_x6_workspace_bytes": [_I64, _I64, _I64],
    "dlcs_debug_conv_stamps": [_P, _I64],
    "dlcs_debug_h3_stamps": [_P, _I64],
}
_RESTYPE = {"dlcs_status_string": ctypes.c_char_p, "dlcs_scratch_bytes": _SZ, "dlcs_sense_workspace_bytes": _SZ,
            "dlcs_sense_cg_workspace_bytes": _SZ, "dlcs_sense_rowtab_bytes": _SZ,
            "dlcs_sense_rows_workspace_bytes": _SZ, "dlcs_split2_f16_bytes": _SZ,
            "dlcs_conv3d_pack_weights_f16x3_bytes": _SZ, "dlcs_conv3d_thin_pack_f16x3_bytes": _SZ,
            "dlcs_gemm_dw_workspace_bytes": _SZ, "dlcs_layernorm_bwd_workspace_bytes": _SZ,
            "dlcs_gemm_f32_splitk_det_workspace_bytes": _SZ, "dlcs_gemm_nt_x6_workspace_bytes": _SZ,
            "dlcs_h3r_pack_bytes": _SZ, "dlcs_mhsa_bwd_workspace_bytes": _SZ}


class DlcsError(RuntimeError):
    pass


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise DlcsError(f"libdlcs_hip.so not found at {LIB_PATH}; build it with "
                            "`make -C dl-swin-gan_amd/csrc` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = _RESTYPE.get(name, _INT)
        for name, args in DIAG_SIGNATURES.items():
            if hasattr(L, name):
                fn = getattr(L, name)
                fn.argtypes = args
                fn.restype = _RESTYPE.get(name, _INT)
        _LIB = L
    return _LIB


def exported_symbols():
    """The product library's C-ABI (include/dlcs.h outside its DLCS_DIAG_BUILD blocks)."""
    return sorted(SIGNATURES.keys())


def scratch_bytes():
    """Bytes of the library's internal per-stream scratch buffers (dlcs.h)."""
    return int(lib().dlcs_scratch_bytes())


def release_scratch():
    """Synchronise and free the library's internal scratch buffers (re-allocated on demand)."""
    check(lib().dlcs_release_scratch(), "dlcs_release_scratch")


def has_symbol(name):
    return hasattr(lib(), name)


def check(status, name):
    if status != 0:
        msg = lib().dlcs_status_string(int(status))
        raise DlcsError(f"{name} failed with status {status}: {msg.decode() if msg else '?'}")


def call(name, *args):
    check(getattr(lib(), name)(*args), name)


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_GET_DEVICE = getattr(torch._C, "_cuda_getDevice", None)


def stream():
    """torch's current HIP stream on the current device as a hipStream_t.  The raw
    getter skips building a torch.cuda.Stream object per launch (that cost ~30 us of
    host time per call, ~500 calls per training step)."""
    if _RAW_STREAM is not None and _GET_DEVICE is not None:
        return ctypes.c_void_p(_RAW_STREAM(_GET_DEVICE()))
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def require_gpu(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise DlcsError("dl_cs HIP ops need GPU tensors (no CPU fallback in the product path)")


def dtype_code(dt):
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    raise DlcsError(f"unsupported dtype {dt}")
