"""Thin typed wrappers over the libdlcs_hip C-ABI (include/dlcs.h).

Every function takes / returns torch tensors that live on the GPU and only
uses torch for allocation and the current stream; the arithmetic is in the
HIP kernels.  ``T`` below is the compute storage dtype (torch.float32 for the
parity build, torch.bfloat16 for the fast path); accumulation is always fp32.
"""
import ctypes

import torch

from .. import _lib
from .. import diag as _diag

F32, BF16 = _lib.F32, _lib.BF16
_I64P = ctypes.POINTER(ctypes.c_int64)


def code(t_or_dtype):
    dt = t_or_dtype.dtype if torch.is_tensor(t_or_dtype) else t_or_dtype
    return _lib.dtype_code(dt)


p = _lib.ptr
S = _lib.stream
call = _lib.call


def empty(shape, dtype, device):
    return torch.empty(shape, dtype=dtype, device=device)


def zeros(shape, dtype, device):
    return torch.zeros(shape, dtype=dtype, device=device)


# ---------------------------------------------------------------------------- GEMM
GEMM_TRACE = None        # list -> per-call (shape key, start event, end event)


def gemm(A, B, C, M, N, K, lda, ldb, ldc, a_trans=0, b_trans=0, bias=None, act=0, aux=None,
         aux_out=None, ldaux=0, alpha=1.0, res=None, ldr=0, row_map=None, accumulate=0, splitk=1,
         res_scale=1.0, res2=None, ldr2=0, res2_scale=1.0):
    """C[row(m), n] (+)= alpha * act(A(m,:) . B(n,:) + bias[n]) + res_scale * res[row(m), n]
    + res2_scale * res2[row(m), n] (see dlcs.h)."""
    if GEMM_TRACE is not None:                     # diagnostics (tools/gemm_profile.py)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        GEMM_TRACE.append(((M, N, K, int(a_trans), int(b_trans), int(act), int(splitk), int(accumulate),
                            str(C.dtype).replace("torch.", ""), row_map is not None), e0, e1))
    call("dlcs_gemm", code(A), M, N, K, p(A), lda, int(a_trans), p(B), ldb, int(b_trans),
         p(C), ldc, code(C), p(bias), int(act), p(aux), p(aux_out), ldaux, float(alpha),
         p(res), ldr, code(res) if res is not None else F32, float(res_scale),
         p(res2), ldr2, code(res2) if res2 is not None else F32, float(res2_scale), p(row_map), int(accumulate),
         int(splitk), S())
    if GEMM_TRACE is not None:
        GEMM_TRACE[-1][2].record()
    return C


def gemm_f32_splitk_det(A, B, C, M, N, K, lda, ldb):
    """C [M, N] fp32 += A(m,:) . B(n,:) (both K-contiguous), deterministic split-K (dlcs_gemm_f32_splitk_det)."""
    nb = int(_lib.lib().dlcs_gemm_f32_splitk_det_workspace_bytes(M, N))
    ws = empty((nb // 4,), torch.float32, C.device)
    call("dlcs_gemm_f32_splitk_det", p(A), lda, p(B), ldb, M, N, K, p(C), p(ws), nb, S())
    return C


def gemm_nt_x6(A, B, C, M, N, K, lda, ldb):
    """C [M, N] fp32 += A(m,:) . B(n,:) on bf16 matrix cores, 3-plane split (dlcs_gemm_nt_x6;
    DIAG build only)."""
    if not _lib.has_symbol("dlcs_gemm_nt_x6"):
        raise _lib.DlcsError("dlcs_gemm_nt_x6 exists only in the DIAG library (make DIAG=1; select it with "
                             "DLCS_HIP_LIB=.../libdlcs_hip_diag.so): unset DLCS_EMBED_X6 / DLCS_NT_X6 for the product "
                             "library")
    nb = int(_lib.lib().dlcs_gemm_nt_x6_workspace_bytes(M, N, K))
    ws = empty((nb // 4,), torch.float32, C.device)
    call("dlcs_gemm_nt_x6", p(A), lda, p(B), ldb, M, N, K, p(C), p(ws), nb, S())
    return C


def linear(x, w, bias=None, out=None, out_dtype=None, act=0, aux_out=None, alpha=1.0, res=None,
           row_map=None, accumulate=0):
    """y = x W^T + b (nn.Linear, W [out, in]), x [M, in] row-major."""
    M, Kd = x.shape
    N = w.shape[0]
    if out is None:
        out = empty((M if row_map is None else res.shape[0], N), out_dtype or x.dtype, x.device)
    return gemm(x, w, out, M, N, Kd, Kd, Kd, N, bias=bias, act=act, aux_out=aux_out, ldaux=N,
                alpha=alpha, res=res, ldr=N, row_map=row_map, accumulate=accumulate)


def linear_dx(g, w, out=None, out_dtype=torch.float32, act=0, aux=None, accumulate=0):
    """dx = g W (W [out, in]); optional times gelu'(aux)."""
    M, No = g.shape
    Ni = w.shape[1]
    if out is None:
        out = empty((M, Ni), out_dtype, g.device)
    return gemm(g, w, out, M, Ni, No, No, Ni, Ni, b_trans=1, act=act, aux=aux, ldaux=Ni,
                accumulate=accumulate)


def h3r_pack(mats):
    """Pack fp32 weight operands for dlcs_gemm_h3r in one launch.  mats: list of
    (W, trans): trans=False -> B = W [N, K] (a Linear forward, W [out, in]);
    trans=True -> B = W^T (an input gradient).  Returns the packed buffers."""
    n = len(mats)
    if n == 0:
        return []
    outs, src, ld, tr, rows, ks = [], [], [], [], [], []
    for w, t in mats:
        assert w.dtype == torch.float32 and w.is_contiguous() and w.dim() == 2
        R, Kd = (w.shape[1], w.shape[0]) if t else (w.shape[0], w.shape[1])
        nb = int(_lib.lib().dlcs_h3r_pack_bytes(R, Kd))
        outs.append(empty((nb,), torch.uint8, w.device))
        src.append(p(w)); ld.append(w.shape[1]); tr.append(int(t)); rows.append(R); ks.append(Kd)
    arr = lambda ct, vals: (ct * n)(*vals)
    vp = lambda a_: ctypes.cast(a_, ctypes.c_void_p)
    call("dlcs_h3r_pack_multi", n, vp(arr(ctypes.c_void_p, src)), vp(arr(ctypes.c_int64, ld)),
         vp(arr(ctypes.c_int, tr)), vp(arr(ctypes.c_int64, rows)), vp(arr(ctypes.c_int64, ks)),
         vp(arr(ctypes.c_void_p, [p(o) for o in outs])), S())
    return outs


def linear_h3r(x, wpack, N, out=None, bias=None, act=0, aux=None, aux_out=None, alpha=1.0, res=None,
               row_map=None, accumulate=0):
    """fp32 y[row(m)] (+)= alpha act(x W^T + b) + res[row(m)] on fp16 matrix cores with
    a per-row split of x and of the packed weight (dlcs_gemm_h3r)."""
    M, Kd = x.shape
    if out is None:
        out = empty((M if row_map is None else res.shape[0], N), torch.float32, x.device)
    ldaux = N if (aux is not None or aux_out is not None) else 0
    call("dlcs_gemm_h3r", p(x), M, Kd, x.stride(0), p(wpack), N, p(out), out.stride(0), p(bias), int(act),
         p(aux), p(aux_out), ldaux, float(alpha), p(res), N if res is not None else 0, p(row_map),
         int(accumulate), S())
    return out


def f8r_quant(x):
    """x fp32 [rows, K] -> (q e4m3 bytes [rows, K], inv scale fp32 [rows]) (dlcs_f8r_quant)."""
    rows, Kd = x.shape
    q = empty((rows, Kd), torch.uint8, x.device)
    inv = empty((rows,), torch.float32, x.device)
    call("dlcs_f8r_quant", p(x), rows, Kd, x.stride(0), p(q), p(inv), S())
    return q, inv


def linear_f8r(xq, w8, N, out=None, bias=None, act=0, aux_out=None, alpha=1.0, res=None, row_map=None):
    """fp8 y[row(m)] = alpha act(x W^T + b) + res[row(m)] from f8r_quant outputs
    xq = (q, inv) and w8 = f8r_quant(W) (dlcs_gemm_f8r)."""
    (aq, ainv), (bq, binv) = xq, w8
    M, Kd = aq.shape
    if out is None:
        out = empty((M if row_map is None else res.shape[0], N), torch.float32, aq.device)
    call("dlcs_gemm_f8r", p(aq), p(ainv), M, Kd, p(bq), p(binv), N, p(out), out.stride(0), p(bias), int(act),
         p(aux_out), N if aux_out is not None else 0, float(alpha), p(res), res.stride(0) if res is not None else 0,
         p(row_map), S())
    return out


def linear_dw(g, x, dw, splitk=None):
    """dW [out, in] += g^T x  (g [M, out], x [M, in]), fp32 split-K atomics."""
    M, No = g.shape
    Ni = x.shape[1]
    if splitk is None:
        tiles = max(1, (No + 127) // 128) * max(1, (Ni + 127) // 128)
        splitk = max(1, min(64, 512 // tiles, M // 256))
    return gemm(g, x, dw, No, Ni, M, No, Ni, Ni, a_trans=1, b_trans=1, accumulate=1, splitk=splitk)


def dw_grouped_ok(T, pairs):
    """True if dlcs_gemm_dw_grouped(_f32) serves these (A [T, M], B [T, N]) pairs
    (both bf16 or both fp32, dense rows, 16-B aligned): M, N multiples of 160, or of
    16 for the fp32 x6 kernel (edge tiles; not with DLCS_DW_F32=1)."""
    edge = _diag.knob("DLCS_DW_F32", "0") != "1"

    def ok(A, B):
        q = 16 if (edge and A.dtype == torch.float32) else 160
        return (A.dtype == B.dtype and A.dtype in (torch.bfloat16, torch.float32) and
                A.shape[-1] % q == 0 and B.shape[-1] % q == 0 and
                all(t.dim() == 2 and t.stride(1) == 1 and t.stride(0) == t.shape[1] and t.data_ptr() % 16 == 0
                    for t in (A, B)))
    return T % 64 == 0 and all(ok(A, B) for A, B in pairs)


def gemm_dw_grouped(T, groups):
    """Grouped weight gradients: for (A [T, M], B [T, N], dW [M, N] fp32, db [P] fp32 or None, P)
    in groups: dW += A^T B, db[c] += sum over tokens and m = c mod P of A (dlcs.h)."""
    n = len(groups)
    arr = lambda ct, vals: (ct * n)(*vals)
    A = arr(ctypes.c_void_p, [p(g[0]) for g in groups])
    B = arr(ctypes.c_void_p, [p(g[1]) for g in groups])
    lda = arr(ctypes.c_int64, [g[0].shape[-1] for g in groups])
    ldb = arr(ctypes.c_int64, [g[1].shape[-1] for g in groups])
    M = arr(ctypes.c_int64, [g[0].shape[-1] for g in groups])
    N = arr(ctypes.c_int64, [g[1].shape[-1] for g in groups])
    dW = arr(ctypes.c_void_p, [p(g[2]) for g in groups])
    db = arr(ctypes.c_void_p, [p(g[3]) for g in groups])
    per = arr(ctypes.c_int64, [int(g[4]) if len(g) > 4 and g[4] else 0 for g in groups])
    nbytes = _lib.lib().dlcs_gemm_dw_workspace_bytes(n, ctypes.cast(M, ctypes.c_void_p), ctypes.cast(N, ctypes.c_void_p), T)
    ws = empty((max(1, nbytes // 4),), torch.float32, groups[0][0].device)
    vp = lambda a_: ctypes.cast(a_, ctypes.c_void_p)
    fn = "dlcs_gemm_dw_grouped_f32" if groups[0][0].dtype == torch.float32 else "dlcs_gemm_dw_grouped"
    call(fn, n, vp(A), vp(lda), vp(B), vp(ldb), vp(M), vp(N), vp(dW), vp(db), vp(per), T, p(ws), nbytes, S())


def colsum(x, out, rows=None, C=None, ld=None):
    rows = x.shape[0] if rows is None else rows
    C = x.shape[-1] if C is None else C
    ld = C if ld is None else ld
    call("dlcs_colsum", code(x), p(x), rows, C, ld, p(out), S())
    return out


# ---------------------------------------------------------------------------- rows / layout
def gather_rows(src, idx, nrows, out_dtype, C=None, out=None):
    C = src.shape[-1] if C is None else C
    if out is None:
        out = empty((nrows, C), out_dtype, src.device)
    call("dlcs_gather_rows", code(src), code(out), p(src), p(idx), p(out), nrows, C, src.shape[-1],
         out.shape[-1], S())
    return out


def cast(src, dtype):
    if src.dtype == dtype:
        return src
    out = empty(src.shape, dtype, src.device)
    call("dlcs_axpby", code(src), code(out), p(src), p(out), src.numel(), 1.0, 0.0, S())
    return out


def cast_multi_bf16(srcs):
    """bf16 copies of fp32 tensors in one launch per DLCS_CAST_MULTI_MAX tensors."""
    outs = [empty(t.shape, torch.bfloat16, t.device) for t in srcs]
    for i in range(0, len(srcs), 64):
        chunk, oc = srcs[i:i + 64], outs[i:i + 64]
        k = len(chunk)
        call("dlcs_cast_multi_bf16", k, (ctypes.c_void_p * k)(*[p(t) for t in chunk]),
             (ctypes.c_void_p * k)(*[p(t) for t in oc]), (ctypes.c_int64 * k)(*[t.numel() for t in chunk]), S())
    return outs


def scaled_copy(x, dtype, a):
    out = empty(x.shape, dtype, x.device)
    call("dlcs_axpby", code(x), code(out), p(x), p(out), x.numel(), float(a), 0.0, S())
    return out


def axpby(x, y, a, b):
    """y = a x + b y (in place on y)."""
    call("dlcs_axpby", code(x), code(y), p(x), p(y), x.numel(), float(a), float(b), S())
    return y


def permute(src, dst_shape, src_strides, dst_dtype=None, out=None, accumulate=0):
    if out is None:
        out = empty(tuple(dst_shape), dst_dtype or src.dtype, src.device)
    nd = len(dst_shape)
    shp = (ctypes.c_int64 * nd)(*dst_shape)
    st = (ctypes.c_int64 * nd)(*src_strides)
    call("dlcs_permute", code(src), code(out), p(src), p(out), nd, ctypes.cast(shp, ctypes.c_void_p),
         ctypes.cast(st, ctypes.c_void_p), int(accumulate), S())
    return out


def fill_bias(out, bias, rows, C, period):
    call("dlcs_fill_bias", p(out), p(bias), rows, C, period, S())
    return out


def layernorm_fwd(x, gamma, beta, rows, src_map=None, out_dtype=torch.float32, eps=1e-5):
    C = x.shape[-1]
    out = empty((rows, C), out_dtype, x.device)
    mean = empty((rows,), torch.float32, x.device)
    rstd = empty((rows,), torch.float32, x.device)
    call("dlcs_layernorm_fwd", code(out), p(x), p(src_map), p(gamma), p(beta), float(eps), p(out),
         p(mean), p(rstd), rows, C, S())
    return out, mean, rstd


def layernorm_bwd(dy, x, gamma, mean, rstd, dx, dgamma, dbeta, src_map=None, dx_in=None):
    """dx (+)= dLN/dx; with dx_in: dx = dx_in + dLN/dx (no clone of the residual gradient)."""
    rows, C = dy.shape
    nbytes = _lib.lib().dlcs_layernorm_bwd_workspace_bytes(rows, C)
    ws = empty((max(1, nbytes // 4),), torch.float32, dy.device)
    call("dlcs_layernorm_bwd", p(dy), p(x), p(src_map), p(gamma), p(mean), p(rstd), p(dx_in), p(dx),
         p(dgamma), p(dbeta), rows, C, p(ws), nbytes, S())
    return dx


# ---------------------------------------------------------------------------- windows
_WIN_CACHE = {}


def window_tables(B, D, H, W, ws, ss, device, want_labels):
    key = (B, D, H, W, tuple(ws), tuple(ss), str(device), bool(want_labels))
    t = _WIN_CACHE.get(key)
    if t is None:
        Dp = -(-D // ws[0]) * ws[0]
        Hp = -(-H // ws[1]) * ws[1]
        Wp = -(-W // ws[2]) * ws[2]
        nrows = B * Dp * Hp * Wp
        part = empty((nrows,), torch.int32, device)
        rev = torch.full((B * D * H * W,), -1, dtype=torch.int32, device=device)
        lab = empty((nrows,), torch.int32, device) if want_labels else None
        call("dlcs_window_index", B, D, H, W, ws[0], ws[1], ws[2], ss[0], ss[1], ss[2],
             p(part), p(rev), p(lab), S())
        t = (part, rev, lab, nrows)
        _WIN_CACHE[key] = t
    return t


def attn_fwd(qkv, table, labels, nwin, N, heads, hd, window0, scale, mask=None, mask_nw=0):
    rows = qkv.shape[0]
    out = empty((rows, heads * hd), qkv.dtype, qkv.device)
    lse = empty((nwin, heads, N), torch.float32, qkv.device)
    call("dlcs_window_attn_fwd", code(qkv), p(qkv), p(out), p(lse), p(table), p(labels), p(mask),
         int(mask_nw), nwin, N, heads, hd, window0[0], window0[1], window0[2], float(scale), S())
    return out, lse


def attn_bwd(qkv, out, dout, lse, table, labels, dtable, nwin, N, heads, hd, window0, scale,
             mask=None, mask_nw=0):
    # every element of dQ, dK, dV is written (the library zeroes the buffer itself for
    # the f32-MFMA kernels, which accumulate dQ with atomics)
    dqkv = empty(qkv.shape, torch.float32, qkv.device)
    call("dlcs_window_attn_bwd", code(qkv), p(qkv), p(out), p(dout), p(lse), p(table), p(labels),
         p(mask), int(mask_nw), p(dqkv), p(dtable), nwin, N, heads, hd, window0[0], window0[1],
         window0[2], float(scale), S())
    return dqkv


# ---------------------------------------------------------------------------- conv3d k3
def pad32(n):
    return (n + 31) // 32 * 32


def conv_pack(w, dtype, mode):
    """torch weight [cout, cin, 3, 3, 3] fp32 -> packed (mode 0 fwd, mode 1 dgrad)."""
    cout, cin = w.shape[0], w.shape[1]
    rows, cols = (pad32(cout), pad32(cin)) if mode == 0 else (pad32(cin), pad32(cout))
    out = empty((27, rows, cols), dtype, w.device)
    call("dlcs_conv3d_pack_weights", code(out), p(w.contiguous()), p(out), cout, cin, rows, cols, mode, S())
    return out


def conv3d(x, cin, packed, cout, out_ld, grid, bias=None, out=None, out_dtype=None, relu_in=0,
           mask=None, res=None, res_scale=1.0, accumulate=0, relu_out=0):
    """out[rows, out_ld] = conv3d_k3(relu?(x)) (+ epilogue); grid = (B, D, H, W)."""
    B, D, H, W = grid
    rows = B * D * H * W
    if out is None:
        out = empty((rows, out_ld), out_dtype or x.dtype, x.device)
    call("dlcs_conv3d_k3", code(x), p(x), cin, x.shape[-1], p(packed), packed.shape[2], p(bias),
         p(out), code(out), cout, packed.shape[1], out.shape[-1], B, D, H, W, int(relu_in),
         p(mask), mask.shape[-1] if mask is not None else 0, p(res),
         code(res) if res is not None else F32, res.shape[-1] if res is not None else 0,
         float(res_scale), int(accumulate), int(relu_out), S())
    return out


def split3(x, out=None):
    """fp32 [rows, ld] (160 channels) -> (xa [rows, 320], xb [rows, 160]) bf16 planes (dlcs_split3_bf16)."""
    rows = x.shape[0]
    if out is None:
        out = (empty((rows, 320), torch.bfloat16, x.device), empty((rows, 160), torch.bfloat16, x.device))
    call("dlcs_split3_bf16", p(x), rows, x.shape[-1], p(out[0]), p(out[1]), S())
    return out


def conv_pack_x6(w, mode):
    """torch weight [160, 160, 3, 3, 3] fp32 -> 3-plane packing (mode 0 fwd, 1 dgrad) for conv3d_x6."""
    packed = empty((27 * 160 * 480,), torch.bfloat16, w.device)
    call("dlcs_conv3d_pack_weights", F32, p(w.contiguous()), p(packed), 160, 160, 0, 0, 2 + mode, S())
    return packed


def conv3d_x6(planes, packed, grid, bias=None, out=None, mask=None, res=None, res_scale=1.0, accumulate=0,
              relu_out=0):
    """fp32 conv3d_k3 160 -> 160 on bf16 planes (dlcs_conv3d_k3_x6); out fp32 [rows, 160]."""
    B, D, H, W = grid
    xa, xb = planes
    if out is None:
        out = empty((xa.shape[0], 160), torch.float32, xa.device)
    call("dlcs_conv3d_k3_x6", p(xa), p(xb), p(packed), p(bias), p(out), out.shape[-1], B, D, H, W, p(mask),
         mask.shape[-1] if mask is not None else 0, p(res), res.shape[-1] if res is not None else 0,
         float(res_scale), int(accumulate), int(relu_out), S())
    return out


def conv3d_wgrad_x6(x_planes, g_planes, grid, dw_packed):
    """dw_packed [27, 160, 160] += fp32 conv weight gradient from bf16 planes (dlcs_conv3d_k3_wgrad_x6)."""
    B, D, H, W = grid
    call("dlcs_conv3d_k3_wgrad_x6", p(x_planes[0]), p(x_planes[1]), p(g_planes[0]), p(g_planes[1]), p(dw_packed),
         B, D, H, W, S())
    return dw_packed


def split2(x, out=None, have_max=False, colsum=None):
    """fp32 [rows, ld] (160 channels) -> f16 planes [rows, 320] + max|x| trailer (dlcs_split2_f16),
    as one flat uint8 tensor.  have_max: the trailer was filled by the producing kernel's out_max;
    colsum (fp32 [160]): += the column sums of x (a conv bias gradient) from the same read."""
    rows = x.shape[0]
    if out is None:
        out = empty((int(_lib.lib().dlcs_split2_f16_bytes(rows)),), torch.uint8, x.device)
    call("dlcs_split2_f16", p(x), rows, x.shape[-1], p(out), int(bool(have_max)), p(colsum), S())
    return out


def planes_alloc(rows, device):
    """An uninitialised split2 buffer for `rows` rows whose max trailer is zeroed, ready to be
    passed (planes_max) as a producer's out_max."""
    out = empty((int(_lib.lib().dlcs_split2_f16_bytes(rows)),), torch.uint8, device)
    out[rows * 640:rows * 640 + 4].zero_()
    return out


def planes_max(planes, rows):
    """Device pointer of the max trailer of a split2 buffer."""
    return ctypes.c_void_p(planes.data_ptr() + rows * 640)


def conv_pack_f16x3(w, mode):
    """torch weight [160, 160, 3, 3, 3] fp32 -> f16 2-plane packing (mode 0 fwd, 1 dgrad) for conv3d_f16x3."""
    packed = empty((int(_lib.lib().dlcs_conv3d_pack_weights_f16x3_bytes()),), torch.uint8, w.device)
    call("dlcs_conv3d_pack_weights_f16x3", p(w.contiguous()), int(mode), p(packed), S())
    return packed


def conv3d_f16x3(planes, packed, grid, bias=None, out=None, mask=None, res=None, res_scale=1.0, accumulate=0,
                 relu_out=0, out_max=None, out_planes=None, colsum=None, planes_only=False, mask_planes=None):
    """fp32 conv3d_k3 160 -> 160 on f16 planes (dlcs_conv3d_k3_f16x3); out fp32 [rows, 160].
    out_planes: a split2 buffer whose trailer holds a bound of max|out| (planes_bound) --
    the epilogue writes out's planes too (planes_only: and no fp32 out; returns None);
    colsum (fp32 [160]) += the column sums of out (the bias gradient of a dgrad); mask_planes: the
    ReLU mask as a producer's planes of a non-negative tensor, in place of mask."""
    B, D, H, W = grid
    rows = B * D * H * W
    if out is None and not planes_only:
        out = empty((rows, 160), torch.float32, planes.device)
    call("dlcs_conv3d_k3_f16x3", p(planes), p(packed), p(bias), p(out), out.shape[-1] if out is not None else 160,
         B, D, H, W, p(mask), mask.shape[-1] if mask is not None else 0, p(res), res.shape[-1] if res is not None else 0,
         float(res_scale), int(accumulate), int(relu_out), out_max, p(out_planes), p(colsum), p(mask_planes), S())
    return out


def gemm_k160_f16x3(a_planes, M, b_planes, N, C, bias=None, act=0, alpha=1.0, res=None, res_scale=1.0,
                    res2=None, res2_scale=1.0, accumulate=0, out_max=None, out_planes=None, colsum=None,
                    res_planes=None, res2_planes=None):
    """C [M, N] fp32 (+)= alpha act(A B^T + bias) + res_scale res + res2_scale res2, K = 160, A / B as
    split2 plane pairs of [M, 160] / [N, 160] (dlcs_gemm_k160_f16x3); out_planes: C's planes as
    [M N / 160][160], scale from the bound in their trailer (planes_bound); C None: planes only;
    colsum (fp32 [160]) += the column sums of that [M N / 160][160] view; res_planes / res2_planes:
    the residuals as split2 buffers of that view instead of fp32 res / res2."""
    call("dlcs_gemm_k160_f16x3", p(a_planes), M, p(b_planes), N, p(C), C.shape[-1] if C is not None else N,
         p(bias), int(act), float(alpha), p(res), res.shape[-1] if res is not None else 0, float(res_scale),
         p(res2), res2.shape[-1] if res2 is not None else 0, float(res2_scale), int(accumulate), out_max,
         p(out_planes), p(colsum), p(res_planes), p(res2_planes), S())
    return C


def _w(m):
    """A float-bits word argument: a ctypes pointer, a tensor (its first word) or None."""
    if m is None or isinstance(m, ctypes.c_void_p):
        return m
    return p(m)


def planes_bound(planes, rows, m0=None, n0=None, c0=1.0, m1=None, n1=None, c1=1.0, vec=None, cvec=1.0):
    """Trailer of the split2 buffer `planes` [rows] <- an upper bound of max|out| for a producer that
    writes the planes itself (dlcs_planes_bound): c0 m0 n0 + c1 m1 n1 + cvec max|vec|."""
    call("dlcs_planes_bound", p(planes), rows, _w(m0), _w(n0), float(c0), _w(m1), _w(n1), float(c1), p(vec),
         vec.numel() if vec is not None else 0, float(cvec), S())
    return planes


def abs_row_sum_max(w, rows, row_stride, inner, n_outer=1, outer_stride=0, out=None):
    """max_r sum |w[r row_stride + o outer_stride + i]| (o < n_outer, i < inner) as float bits in an
    int32 [1] (dlcs_abs_row_sum_max): ||W||_inf of a weight layout, for planes_bound."""
    if out is None:
        out = empty((1,), torch.int32, w.device)
    call("dlcs_abs_row_sum_max", p(w), rows, row_stride, n_outer, outer_stride, inner, p(out), S())
    return out


def linear_k160_f16x3(x_planes, M, w_planes, N, out, bias=None, act=0, aux=None, aux_out=None, alpha=1.0,
                      res=None, row_map=None, accumulate=0):
    """out [row(m), N] fp32 (+)= alpha act(x W^T + b) + res[row(m)], in_features 160, x / W as split2 plane
    pairs of [M, 160] / [N, 160] (dlcs_linear_k160_f16x3); act 1 GELU (pre-activation -> aux_out), 2 x GELU'(aux)."""
    ldaux = (aux if aux is not None else aux_out).shape[-1] if (aux is not None or aux_out is not None) else 0
    call("dlcs_linear_k160_f16x3", p(x_planes), M, p(w_planes), N, p(out), out.shape[-1], p(bias), int(act),
         p(aux), p(aux_out), ldaux, float(alpha), p(res), res.shape[-1] if res is not None else 0, p(row_map),
         int(accumulate), S())
    return out


def conv3d_wgrad_f16x3(x_planes, g_planes, grid, dw_packed):
    """dw_packed [27, 160, 160] += fp32 conv weight gradient from f16 plane pairs (dlcs_conv3d_k3_wgrad_f16x3)."""
    B, D, H, W = grid
    call("dlcs_conv3d_k3_wgrad_f16x3", p(x_planes), p(g_planes), p(dw_packed), B, D, H, W, S())
    return dw_packed


def absmax(x, out=None):
    """max |x| of a contiguous fp32 tensor as float bits in an int32 [1] (dlcs_absmax_f32); an
    existing `out` is max-accumulated -- the scale word of the thin-end f16x3 kernels."""
    if out is None:
        out = zeros((1,), torch.int32, x.device)
    call("dlcs_absmax_f32", p(x), x.numel(), p(out), S())
    return out


def _word(m):
    return m if isinstance(m, ctypes.c_void_p) else p(m)


def thin_pack_f16x3(packed, cout, cin, kind):
    """conv_pack output fp32 [27, cout_pad, cin_pad] -> the f16 2-plane image of the thin-end
    kernels (kind 0: thin input, Cin <= 4 -> 160; kind 1: thin output, 160 -> Cout <= 4)."""
    out = empty((int(_lib.lib().dlcs_conv3d_thin_pack_f16x3_bytes(kind)),), torch.uint8, packed.device)
    call("dlcs_conv3d_thin_pack_f16x3", p(packed), cout, packed.shape[1], cin, packed.shape[2], int(kind), p(out), S())
    return out


def conv3d_thin_f16x3(x, cin, x_max, wthin, cout, out_ld, grid, bias=None, out=None, mask=None, res=None,
                      res_scale=1.0, accumulate=0, relu_out=0, out_max=None, out_planes=None, colsum=None,
                      planes_only=False, mask_planes=None):
    """fp32 thin-end conv3d_k3 (4 -> 160 or 160 -> 4) on fp16 matrix cores (dlcs_conv3d_thin_f16x3);
    x_max: the max |x| word (absmax() tensor or a producer's out_max pointer); out fp32 [rows, out_ld].
    Thin input with a mask: out_planes (scale from the bound in their trailer; planes_only: no fp32
    out, returns None) and colsum (+= out's column sums)."""
    B, D, H, W = grid
    rows = B * D * H * W
    if out is None and not planes_only:
        out = empty((rows, out_ld), torch.float32, x.device)
    call("dlcs_conv3d_thin_f16x3", p(x), cin, x.shape[-1], _word(x_max), p(wthin), p(bias), p(out), cout,
         out.shape[-1] if out is not None else 160, B, D, H, W, p(mask), mask.shape[-1] if mask is not None else 0,
         p(res), res.shape[-1] if res is not None else 0, float(res_scale), int(accumulate), int(relu_out),
         _word(out_max) if out_max is not None else None, p(out_planes), p(colsum), p(mask_planes), S())
    return out


def conv3d_thin_wgrad_f16x3(x, cin, x_max, g, cout, g_max, grid, dw_packed, colsum=None):
    """dw_packed [27, cout_pad, cin_pad] += fp32 weight gradient of a thin-end conv on fp16 matrix
    cores (dlcs_conv3d_thin_wgrad_f16x3); colsum (SFE shape only): += sum over voxels of g."""
    B, D, H, W = grid
    call("dlcs_conv3d_thin_wgrad_f16x3", p(x), cin, x.shape[-1], _word(x_max), p(g), cout, g.shape[-1],
         _word(g_max), p(dw_packed), dw_packed.shape[1], dw_packed.shape[2], p(colsum), B, D, H, W, S())
    return dw_packed


def conv3d_thin_out_planes(planes, wthin, cout, out_ld, grid, bias=None, out=None, accumulate=0, relu_out=0):
    """fp32 thin-output conv3d_k3 (160 -> cout <= 4) from the split2 planes of its input
    (dlcs_conv3d_thin_out_planes_f16x3); out fp32 [rows, out_ld]."""
    B, D, H, W = grid
    rows = B * D * H * W
    if out is None:
        out = empty((rows, out_ld), torch.float32, planes.device)
    call("dlcs_conv3d_thin_out_planes_f16x3", p(planes), p(wthin), p(bias), p(out), cout, out.shape[-1], B, D, H, W,
         int(accumulate), int(relu_out), S())
    return out


def conv3d_thin_wgrad_planes(big_planes, thin, thin_ch, thin_max, big_is_co, grid, dw_packed):
    """dw_packed [27, cout_pad, cin_pad] += fp32 weight gradient between the split2 planes of the
    160-channel operand and the fp32 thin tensor (dlcs_conv3d_thin_wgrad_planes_f16x3); big_is_co:
    1 = SFE (planes = g), 0 = final conv (planes = its input)."""
    B, D, H, W = grid
    call("dlcs_conv3d_thin_wgrad_planes_f16x3", p(big_planes), p(thin), thin_ch, thin.shape[-1], _word(thin_max),
         int(big_is_co), p(dw_packed), dw_packed.shape[1], dw_packed.shape[2], B, D, H, W, S())
    return dw_packed


def conv3d_wgrad(x, cin, relu_in, g, cout, grid, dw_packed, vox_per_block=16384, dbias=None):
    """dw_packed += the conv weight gradient; dbias (fp32 [cout], optional) += the bias
    gradient (column sums of g), fused into the 160-channel bf16 kernel."""
    B, D, H, W = grid
    call("dlcs_conv3d_k3_wgrad", code(x), p(x), cin, x.shape[-1], dw_packed.shape[2], int(relu_in),
         p(g), cout, g.shape[-1], dw_packed.shape[1], p(dw_packed), p(dbias), B, D, H, W, vox_per_block, S())
    return dw_packed


def conv_unpack_grad(dw_packed, grad, cout, cin, accumulate=1):
    call("dlcs_conv3d_unpack_wgrad", p(dw_packed), p(grad), cout, cin, dw_packed.shape[1],
         dw_packed.shape[2], int(accumulate), S())
    return grad


# ---------------------------------------------------------------------------- boundary
def swin_pre(x, dtype, pad, ldc):
    B, E, T, Y, X = x.shape
    u = empty((B * (T + 2 * pad) * Y * X, ldc), dtype, x.device)
    call("dlcs_swin_pre", code(dtype), p(x), p(u), B, E, T, Y, X, pad, ldc, S())
    return u


def swin_pre_bwd(gu, shape, pad):
    B, E, T, Y, X = shape
    gx = empty(shape, torch.complex64, gu.device)
    call("dlcs_swin_pre_bwd", code(gu), p(gu), p(gx), B, E, T, Y, X, pad, gu.shape[-1], S())
    return gx


def swin_post(o, shape, pad):
    B, E, T, Y, X = shape
    out = empty(shape, torch.complex64, o.device)
    call("dlcs_swin_post", code(o), p(o), p(out), B, E, T, Y, X, pad, o.shape[-1], S())
    return out


def swin_post_bwd(gout, dtype, pad, ldc):
    B, E, T, Y, X = gout.shape
    go = empty((B * (T + 2 * pad) * Y * X, ldc), dtype, gout.device)
    call("dlcs_swin_post_bwd", code(dtype), p(gout), p(go), B, E, T, Y, X, pad, ldc, S())
    return go


def relu_grad(g, a):
    """g *= (a > 0) in place (a: stored post-ReLU activation, same element count)."""
    assert g.numel() == a.numel()
    call("dlcs_relu_grad", code(g), p(g), code(a), p(a), g.numel(), S())
    return g
