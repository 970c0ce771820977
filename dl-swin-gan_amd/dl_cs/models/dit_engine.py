"""HIP forward / hand-scheduled backward of the DiT regularizers (DiTResNet,
DiTNet; dit = dl_cs/models/DiT.py), one autograd node per network call.

Layouts (fp32; B samples, time padded to Tp = T + 2 pad, Y, X multiples of 4):
  * full-resolution activations in the patch-blocked channels-last layout of the
    Swin path (row(b,t,y,x) = patch-of-4x4x4 * 64 + (t%4) 16 + (y%4) 4 + x%4), so
    a (2,4,4) DiT patch is 32 consecutive rows: the patch embed (dit:103, :124) is
    one GEMM [subpatches, 32 C] x [32 C, D] and the final Linear's output
    (p, q, r, c) columns (dit:398, unpatchify2 dit:515-543) are exactly the 32
    rows x C channels of a subpatch -- no im2col, no unpatchify copy;
  * tokens [M = B F H W, D] in the reference's (b, f, h, w) order (dit:135);
    the per-position-over-frames attention (factorize flag 1, dit:336) reads
    its LayerNorm input through a row map into (b, h, w, f) order and its proj
    GEMM scatters back (row_map), so both attentions see contiguous sequences.
Gated residual branches g * (x W^T + b) (dit:338, :345, :348) run as one GEMM on
gate-scaled weights (dlcs_scale_rows); their gate / weight / bias gradients come
from the unscaled dW GEMM (dlcs_gated_linear_grad).  adaLN-modulated LayerNorms
(dit:22-23) are dlcs_layernorm with gamma = 1 + scale, beta = shift.
"""

import os

import numpy as np
import torch

from .. import _lib
from .. import diag as _diag
from . import _ops as K

PAD_CIN = 8
# fp8 inference path (BASELINE config 5, "fp8 MFMA path"; the reference has no fp8):
# with FP8 set and no gradient requested, the DiT blocks' token Linears (adaLN,
# qkv, proj, fc1, fc2: dit:317-323, :329-350) run as dlcs_f8r_quant +
# dlcs_gemm_f8r -- OCP e4m3 operands with one power-of-two scale per row of each
# operand, v_mfma_f32_16x16x32_fp8_fp8, fp32 accumulation and epilogue; the
# LayerNorms, attention, patch embed, final layer and convs stay fp32.  Budget
# (tests/test_gpu_dit.py): NRMSE <= 7e-2 per GEMM and <= 5e-2 on the denoiser
# output vs the fp32 oracle.  DLCS_DIT_FP8=1 or set_fp8(True).
# a feature switch (config 5's fp8 inference path), not a diagnostic one
FP8 = os.environ.get("DLCS_DIT_FP8", "0") == "1"


def set_fp8(on):
    """Select the fp8 token-Linear path for gradient-free DiT calls."""
    global FP8
    FP8 = bool(on)


# fp32 token Linears (qkv, proj, fc1, fc2 and their input gradients) on the
# row-scaled fp16 split (dlcs_gemm_h3r: three fp16 plane products per fp32
# product, one power-of-two scale per row and 192-wide K segment of the
# activation and per row of the packed weight); DLCS_DIT_H3R=0 keeps them on the
# f32 matrix cores (dlcs_gemm).  The adaLN / timestep Linears (M = B rows) stay
# on dlcs_gemm.
H3R = _diag.knob("DLCS_DIT_H3R", "1") != "0"


def _h3_ok(W, trans=False):
    N, Kd = (W.shape[1], W.shape[0]) if trans else W.shape
    return (H3R and W.dtype == torch.float32 and W.is_contiguous() and
            ((N % 160 == 0 and Kd in (160, 480, 640)) or (N % 64 == 0 and Kd % 64 == 0 and Kd <= 16384)))


def _packs(*mats):
    """dlcs_gemm_h3r packs of (W, trans) pairs in one launch (None where the shape
    is not served): trans False -> the forward's B = W, True -> the input
    gradient's B = W^T."""
    ok = [m for m in mats if _h3_ok(*m)]
    pk = iter(K.h3r_pack(ok)) if ok else iter(())
    return [next(pk) if _h3_ok(*m) else None for m in mats]


def _lin(fp8, x, W, bias=None, out=None, act=0, aux_out=None, res=None, row_map=None, hp=None):
    """y[row(m)] = act(x W^T + b) + res[row(m)]: the fp8 path, dlcs_gemm_h3r on the
    pack hp of W, or fp32 dlcs_gemm."""
    N, Kd = W.shape
    if fp8 and Kd % 64 == 0 and N % 64 == 0:
        return K.linear_f8r(K.f8r_quant(x), K.f8r_quant(W), N, out=out, bias=bias, act=act, aux_out=aux_out,
                            res=res, row_map=row_map)
    if hp is not None:
        return K.linear_h3r(x, hp, N, out=out, bias=bias, act=act, aux_out=aux_out, res=res, row_map=row_map)
    return K.linear(x, W, bias=bias, out=out, act=act, aux_out=aux_out, res=res, row_map=row_map)


def _dx(g, W, hp=None, out=None, act=0, aux=None):
    """dx = g W (times act'(aux)): dlcs_gemm_h3r on the pack hp of W^T, or dlcs_gemm."""
    if hp is not None:
        return K.linear_h3r(g, hp, W.shape[1], out=out, act=act, aux=aux)
    return K.linear_dx(g, W, out=out, act=act, aux=aux)


def _gated_pack(fp8, Wg, trans=False):
    return None if fp8 else _packs((Wg, trans))[0]
TLD = 108                      # 27 taps x 4 channels: the thin convs' GEMM depth


def _dev_i32(a, device):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(device)


_GEO = {}


class Geo:
    """Index maps of one (B, Tp, Y, X) geometry (host-built once, cached)."""

    def __init__(self, B, Tp, Y, X, device):
        self.B, self.Tp, self.Y, self.X = B, Tp, Y, X
        self.F, self.Hh, self.Ww = Tp // 2, Y // 4, X // 4
        self.V = B * Tp * Y * X
        self.M = B * self.F * self.Hh * self.Ww
        self.Mb = self.M // B
        F, Hh, Ww = self.F, self.Hh, self.Ww
        b, f, h, w = np.meshgrid(np.arange(B), np.arange(F), np.arange(Hh), np.arange(Ww), indexing="ij")
        tok = ((b * F + f) * Hh + h) * Ww + w                          # reference token order (b, f, h, w)
        sub = (((b * (Tp // 4) + f // 2) * Hh + h) * Ww + w) * 2 + f % 2   # 32-row subpatch of the blocked layout
        tim = ((b * Hh + h) * Ww + w) * F + f                          # (b, h, w, f) order of flag-1 attention
        tok, sub, tim = tok.reshape(-1), sub.reshape(-1), tim.reshape(-1)
        sub2tok = np.empty(self.M, np.int64)
        sub2tok[sub] = tok
        tok2sub = np.empty(self.M, np.int64)
        tok2sub[tok] = sub
        tim2tok = np.empty(self.M, np.int64)
        tim2tok[tim] = tok
        self.sub2tok = _dev_i32(sub2tok, device)     # GEMM row map: subpatch row -> token row
        self.tok2sub = _dev_i32(tok2sub, device)     # token row -> subpatch row
        self.tim2tok = _dev_i32(tim2tok, device)     # flag-1 sequence row -> token row

    @staticmethod
    def get(B, Tp, Y, X, device):
        key = (B, Tp, Y, X, str(device))
        g = _GEO.get(key)
        if g is None:
            g = _GEO[key] = Geo(B, Tp, Y, X, device)
        return g


def _empty(shape, dev):
    return torch.empty(shape, dtype=torch.float32, device=dev)


def _zeros(shape, dev):
    return torch.zeros(shape, dtype=torch.float32, device=dev)


def _vec(op, a, b=None, out=None):
    out = torch.empty_like(a) if out is None else out
    _lib.call("dlcs_dit_vec", int(op), K.p(a), K.p(b), K.p(out), a.numel(), K.S())
    return out


def _scale_rows(W, b, gate):
    Wo, bo = torch.empty_like(W), torch.empty_like(b)
    _lib.call("dlcs_scale_rows", K.p(W), K.p(b), K.p(gate), K.p(Wo), K.p(bo), W.shape[0], W.shape[1], K.S())
    return Wo, bo


def _gated_grad(W, b, G, cs, gate, dW, db, dgate):
    _lib.call("dlcs_gated_linear_grad", K.p(W), K.p(b), K.p(G), K.p(cs), K.p(gate), K.p(dW), K.p(db), K.p(dgate),
              W.shape[0], W.shape[1], K.S())


# Optional live profiling (bench.py): when a list, every attention forward appends
# (start_event, end_event, flops, N) recorded on the launching stream; flops =
# Q K^T + P V = 4 nseq heads N^2 hd.
PROFILE = None


def _mhsa(qkv, nseq, N, heads, hd, scale):
    out = _empty((qkv.shape[0], heads * hd), qkv.device)
    lse = _empty((nseq, heads, N), qkv.device)
    if PROFILE is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    _lib.call("dlcs_mhsa_fwd", K.F32, K.p(qkv), K.p(out), K.p(lse), nseq, N, heads, hd, float(scale), K.S())
    if PROFILE is not None:
        e1.record()
        PROFILE.append((e0, e1, 4.0 * nseq * heads * N * N * hd, N))
    return out, lse


def _mhsa_bwd(qkv, out, dout, lse, nseq, N, heads, hd, scale):
    dout = dout.contiguous()
    dqkv = torch.empty_like(qkv)
    nb = int(_lib.lib().dlcs_mhsa_bwd_workspace_bytes(nseq, N, heads))
    ws = _empty((max(1, nb // 4),), qkv.device)
    _lib.call("dlcs_mhsa_bwd", K.F32, K.p(qkv), K.p(out), K.p(dout), K.p(lse), K.p(dqkv), nseq, N,
              heads, hd, float(scale), K.p(ws), nb, K.S())
    return dqkv


def _thin_h3(D):
    """The thin convs' GEMMs (SFE / final conv of DiTResNet, hidden D) on dlcs_gemm_h3r."""
    return H3R and D % 64 == 0


def _tld(D):
    """Row length of the thin convs' im2col / tap-sum GEMM operands: 108 (27 taps x
    4 channels), zero-padded to 128 for dlcs_gemm_h3r (K and N multiples of 64)."""
    return 128 if _thin_h3(D) else TLD


def _im2col(src, C, grid, sign, tld):
    B, D, H, W = grid
    dst = _empty((B * D * H * W, tld), src.device)
    _lib.call("dlcs_conv3d_thin_im2col", K.p(src), src.shape[-1], C, K.p(dst), tld, int(sign), B, D, H, W, K.S())
    return dst


def _pad2(W, rows, cols):
    """W [r, c] zero-padded to [rows, cols] (no copy when already that shape)."""
    if tuple(W.shape) == (rows, cols):
        return W.contiguous()
    out = _zeros((rows, cols), W.device)
    out[:W.shape[0], :W.shape[1]].copy_(W)
    return out


def _gemm_h3(x, W, N, trans=False, **kw):
    """x W^T (trans False, W [N, K]) or x W (trans True, W [K, N]) on dlcs_gemm_h3r,
    W packed here (one launch); kw: out, bias, act, aux, aux_out, res, row_map."""
    return K.linear_h3r(x, _packs((W, trans))[0], N, **kw)


def _col2im(P, C, ld_out, grid, sign, bias=None):
    B, D, H, W = grid
    out = _empty((B * D * H * W, ld_out), P.device)
    _lib.call("dlcs_conv3d_thin_col2im", K.p(P), P.shape[-1], C, K.p(out), ld_out, K.p(bias), int(sign), 0,
              B, D, H, W, K.S())
    return out


def _ln(x, gamma, beta, rows, src_map=None):
    """adaLN-modulated LayerNorm (no affine, eps 1e-6, dit:317-320) with gamma = 1 + scale."""
    return K.layernorm_fwd(x, gamma, beta, rows, src_map=src_map, out_dtype=torch.float32, eps=1e-6)


# ---------------------------------------------------------------------------- parameters
def names(mod, depth):
    """State-dict names the engine reads, keyed by role."""
    d = "DiT."
    n = dict(sfe_w="SFE.layers.2.conv.weight", sfe_b="SFE.layers.2.conv.bias",
             fin_w="final_layer.layers.2.conv.weight", fin_b="final_layer.layers.2.conv.bias",
             pe_w=d + "x_embedder.proj.weight", pe_b=d + "x_embedder.proj.bias",
             t0_w=d + "t_embedder.mlp.0.weight", t0_b=d + "t_embedder.mlp.0.bias",
             t2_w=d + "t_embedder.mlp.2.weight", t2_b=d + "t_embedder.mlp.2.bias",
             y_tab=d + "y_embedder.embedding_table.weight", pos=d + "pos_embedder.pos_embed_table",
             fl_w=d + "final_layer.linear.weight", fl_b=d + "final_layer.linear.bias",
             fa_w=d + "final_layer.adaLN_modulation.1.weight", fa_b=d + "final_layer.adaLN_modulation.1.bias")
    blocks = []
    for i in range(depth):
        p = f"{d}blocks.{i}."
        blocks.append(dict(qkv_w=p + "attn.qkv.weight", qkv_b=p + "attn.qkv.bias",
                           proj_w=p + "attn.proj.weight", proj_b=p + "attn.proj.bias",
                           fc1_w=p + "mlp.fc1.weight", fc1_b=p + "mlp.fc1.bias",
                           fc2_w=p + "mlp.fc2.weight", fc2_b=p + "mlp.fc2.bias",
                           ada_w=p + "adaLN_modulation.1.weight", ada_b=p + "adaLN_modulation.1.bias"))
    n["blocks"] = blocks
    return n


# ---------------------------------------------------------------------------- DiT block
def block_forward(P, nb, tok, sc, geo, heads, hd, fp8=False):
    """dit:329-350 on tokens tok [M, D] (reference order); sc = SiLU(c) [B, D];
    fp8: the token Linears on the fp8 path (inference only)."""
    dev = tok.device
    D = tok.shape[1]
    M, Mb, B = geo.M, geo.Mb, geo.B
    scale = hd ** -0.5
    mod = _lin(fp8, sc, P[nb["ada_w"]], bias=P[nb["ada_b"]])                # [B, 9D]
    ch = lambda k: mod[:, k * D:(k + 1) * D]                                # noqa: E731
    sh_s, sc_s, g_s, g_t, sh_m, sc_m, g_m = ch(0), ch(1), ch(2), ch(5), ch(6), ch(7), ch(8)
    gam_s = _vec(2, sc_s.contiguous())
    gam_m = _vec(2, sc_m.contiguous())
    sh_s, sh_m = sh_s.contiguous(), sh_m.contiguous()
    Wqkv, bqkv, Wp, bp = P[nb["qkv_w"]], P[nb["qkv_b"]], P[nb["proj_w"]], P[nb["proj_b"]]
    W1, b1, W2, b2 = P[nb["fc1_w"]], P[nb["fc1_b"]], P[nb["fc2_w"]], P[nb["fc2_b"]]
    hq, h1p = (None, None) if fp8 else _packs((Wqkv, False), (W1, False))
    sv = dict(mod=mod, gam_s=gam_s, gam_m=gam_m, x0=tok)
    # (1) attention over the frames of each spatial position (factorize flag 1, dit:334-338)
    h1, m1, r1 = _empty((M, D), dev), _empty((M,), dev), _empty((M,), dev)
    x1 = _empty((M, D), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        o, mu, rstd = _ln(tok, gam_s[b], sh_s[b], Mb, src_map=geo.tim2tok[rs])
        h1[rs], m1[rs], r1[rs] = o, mu, rstd
    qkv1 = _lin(fp8, h1, Wqkv, bias=bqkv, hp=hq)
    a1, lse1 = _mhsa(qkv1, B * geo.Hh * geo.Ww, geo.F, heads, hd, scale)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        Wg, bg = _scale_rows(Wp, bp, g_s[b].contiguous())
        _lin(fp8, a1[rs], Wg, bias=bg, out=x1, res=tok, row_map=geo.tim2tok[rs], hp=_gated_pack(fp8, Wg))
    # (2) attention over the positions of each frame (flag 0, dit:341-345), modulated
    # with the *spatial* shift / scale as the reference (dit:342)
    h2, m2, r2 = _empty((M, D), dev), _empty((M,), dev), _empty((M,), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        h2[rs], m2[rs], r2[rs] = _ln(x1[rs], gam_s[b], sh_s[b], Mb)
    qkv2 = _lin(fp8, h2, Wqkv, bias=bqkv, hp=hq)
    a2, lse2 = _mhsa(qkv2, B * geo.F, geo.Hh * geo.Ww, heads, hd, scale)
    x2 = _empty((M, D), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        Wg, bg = _scale_rows(Wp, bp, g_t[b].contiguous())
        _lin(fp8, a2[rs], Wg, bias=bg, out=x2[rs], res=x1[rs], hp=_gated_pack(fp8, Wg))
    # (3) Mlp (GELU tanh) on the mlp-modulated LayerNorm (dit:348)
    h3, m3, r3 = _empty((M, D), dev), _empty((M,), dev), _empty((M,), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        h3[rs], m3[rs], r3[rs] = _ln(x2[rs], gam_m[b], sh_m[b], Mb)
    upre = _empty((M, W1.shape[0]), dev)
    v = _lin(fp8, h3, W1, bias=b1, act=4, aux_out=upre, hp=h1p)
    x3 = _empty((M, D), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        Wg, bg = _scale_rows(W2, b2, g_m[b].contiguous())
        _lin(fp8, v[rs], Wg, bias=bg, out=x3[rs], res=x2[rs], hp=_gated_pack(fp8, Wg))
    sv.update(x1=x1, x2=x2, h1=h1, h2=h2, h3=h3, m1=m1, r1=r1, m2=m2, r2=r2, m3=m3, r3=r3, qkv1=qkv1, qkv2=qkv2,
              a1=a1, a2=a2, lse1=lse1, lse2=lse2, upre=upre, v=v)
    return x3, sv


# The fp32 weight gradients on the grouped fp16 2-plane kernel (dlcs_gemm_dw_grouped_f32:
# per-column scales, edge tiles for D = 384 / 1152 / 1536) where the shapes allow:
# 1.32 ms per block's four Linears vs 1.73 ms on the f32-MFMA split-K GEMM (r05i,
# tools/dw_bench.py); also the per-unroll convolution / patch-embed weight gradients
# over every voxel (K = 737,280: 1.55 ms each on the f32-MFMA GEMM, r06c5).  DLCS_DIT_DW_GROUPED=0 (with DLCS_DIAG=1): the f32-MFMA GEMM.
DW_GROUPED = _diag.knob("DLCS_DIT_DW_GROUPED", "1") == "1"


def _lin_grads(g, x, dW, db):
    """dW += g^T x, db += colsum(g)."""
    if (DW_GROUPED and g.dtype == torch.float32 and dW.is_contiguous() and dW.shape == (g.shape[1], x.shape[1]) and
            K.dw_grouped_ok(g.shape[0], [(g, x)])):
        K.gemm_dw_grouped(g.shape[0], [(g, x, dW, db, g.shape[1] if db is not None else 0)])
        return
    K.linear_dw(g, x, dW)
    if db is not None:
        K.colsum(g, db)


def block_backward(P, G, nb, sv, dy, sc, dsc, geo, heads, hd):
    """Backward of block_forward: returns d tokens; accumulates parameter grads into
    G and d SiLU(c) into dsc."""
    dev = dy.device
    D = dy.shape[1]
    M, Mb, B = geo.M, geo.Mb, geo.B
    scale = hd ** -0.5
    mod = sv["mod"]
    dmod = _zeros((B, 9 * D), dev)
    dch = lambda k: dmod[:, k * D:(k + 1) * D]                              # noqa: E731
    ch = lambda k: mod[:, k * D:(k + 1) * D].contiguous()                   # noqa: E731
    g_s, g_t, g_m = ch(2), ch(5), ch(8)
    Wqkv, Wp, bp = P[nb["qkv_w"]], P[nb["proj_w"]], P[nb["proj_b"]]
    W1, W2, b2 = P[nb["fc1_w"]], P[nb["fc2_w"]], P[nb["fc2_b"]]
    dgam = {k: _zeros((B, D), dev) for k in ("s", "m")}
    dbet = {k: _zeros((B, D), dev) for k in ("s", "m")}
    dgate = {k: _zeros((B, D), dev) for k in ("s", "t", "m")}
    hqT, h1T = _packs((Wqkv, True), (W1, True))
    # (3) Mlp: x3 = x2 + g_m (v W2^T + b2)
    du = _empty((M, W1.shape[0]), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        Wg, _ = _scale_rows(W2, b2, g_m[b])
        _dx(dy[rs], Wg, _gated_pack(False, Wg, True), out=du[rs], act=5, aux=sv["upre"][rs])
        G2 = _zeros(W2.shape, dev)
        cs = _zeros((D,), dev)
        _lin_grads(dy[rs], sv["v"][rs], G2, cs)
        _gated_grad(W2, b2, G2, cs, g_m[b], G[nb["fc2_w"]], G[nb["fc2_b"]], dgate["m"][b])
    dh3 = _dx(du, W1, h1T)
    _lin_grads(du, sv["h3"], G[nb["fc1_w"]], G[nb["fc1_b"]])
    dx2 = _empty((M, D), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        K.layernorm_bwd(dh3[rs], sv["x2"][rs], sv["gam_m"][b], sv["m3"][rs], sv["r3"][rs], dx2[rs],
                        dgam["m"][b], dbet["m"][b], dx_in=dy[rs])
    # (2) per-frame attention: x2 = x1 + g_t (a2 Wp^T + bp)
    da2 = _empty((M, D), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        Wg, _ = _scale_rows(Wp, bp, g_t[b])
        _dx(dx2[rs], Wg, _gated_pack(False, Wg, True), out=da2[rs])
        Gp = _zeros(Wp.shape, dev)
        cs = _zeros((D,), dev)
        _lin_grads(dx2[rs], sv["a2"][rs], Gp, cs)
        _gated_grad(Wp, bp, Gp, cs, g_t[b], G[nb["proj_w"]], G[nb["proj_b"]], dgate["t"][b])
    dqkv2 = _mhsa_bwd(sv["qkv2"], sv["a2"], da2, sv["lse2"], B * geo.F, geo.Hh * geo.Ww, heads, hd, scale)
    dh2 = _dx(dqkv2, Wqkv, hqT)
    _lin_grads(dqkv2, sv["h2"], G[nb["qkv_w"]], G[nb["qkv_b"]])
    dx1 = _empty((M, D), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        K.layernorm_bwd(dh2[rs], sv["x1"][rs], sv["gam_s"][b], sv["m2"][rs], sv["r2"][rs], dx1[rs],
                        dgam["s"][b], dbet["s"][b], dx_in=dx2[rs])
    # (1) per-position attention: x1[tim2tok[j]] = x0[...] + g_s (a1[j] Wp^T + bp)
    dx1_t = K.gather_rows(dx1, geo.tim2tok, M, torch.float32)
    da1 = _empty((M, D), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        Wg, _ = _scale_rows(Wp, bp, g_s[b])
        _dx(dx1_t[rs], Wg, _gated_pack(False, Wg, True), out=da1[rs])
        Gp = _zeros(Wp.shape, dev)
        cs = _zeros((D,), dev)
        _lin_grads(dx1_t[rs], sv["a1"][rs], Gp, cs)
        _gated_grad(Wp, bp, Gp, cs, g_s[b], G[nb["proj_w"]], G[nb["proj_b"]], dgate["s"][b])
    dqkv1 = _mhsa_bwd(sv["qkv1"], sv["a1"], da1, sv["lse1"], B * geo.Hh * geo.Ww, geo.F, heads, hd, scale)
    dh1 = _dx(dqkv1, Wqkv, hqT)
    _lin_grads(dqkv1, sv["h1"], G[nb["qkv_w"]], G[nb["qkv_b"]])
    dx0 = _empty((M, D), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        K.layernorm_bwd(dh1[rs], sv["x0"], sv["gam_s"][b], sv["m1"][rs], sv["r1"][rs], dx0, dgam["s"][b],
                        dbet["s"][b], src_map=geo.tim2tok[rs], dx_in=dx1)
    # adaLN: mod = SiLU(c) W_ada^T + b_ada, chunks (shift_s, scale_s, gate_s, -, -, gate_t, shift_m, scale_m, gate_m)
    for k, src in ((0, dbet["s"]), (1, dgam["s"]), (2, dgate["s"]), (5, dgate["t"]), (6, dbet["m"]),
                   (7, dgam["m"]), (8, dgate["m"])):
        dch(k).copy_(src)
    _lin_grads(dmod, sc, G[nb["ada_w"]], G[nb["ada_b"]])
    K.linear_dx(dmod, P[nb["ada_w"]], out=dsc, accumulate=1)
    return dx0


# ---------------------------------------------------------------------------- whole network
def _patch_weights(P, n, D, ldsrc):
    """GEMM layouts of the patch embed [D][(kd, kh, kw)][c] (channel stride ldsrc) and of the
    final Linear for a thin (DiTNet) output: rows (p, q, r, c) at channel stride PAD_CIN."""
    Wpe = P[n["pe_w"]]                                          # [D, Cpe, 2, 4, 4]
    Cpe = Wpe.shape[1]
    g = K.permute(Wpe, (D, 32, Cpe), (Cpe * 32, 1, 32))
    if ldsrc != Cpe:
        gp = _zeros((D, 32, ldsrc), Wpe.device)
        gp[:, :, :Cpe].copy_(g)
        g = gp
    return g.view(D, 32 * ldsrc)


def _padded_final_linear(Wl, bl, cout):
    Wp_ = _zeros((32, PAD_CIN, Wl.shape[1]), Wl.device)
    Wp_[:, :cout].copy_(Wl.view(32, cout, -1))
    bp_ = _zeros((32, PAD_CIN), Wl.device)
    bp_[:, :cout].copy_(bl.view(32, cout))
    return Wp_.view(32 * PAD_CIN, -1), bp_.view(-1)


def regularizer_forward(P, n, x, t, labels, meta):
    """DiTResNet (residual_convs) / DiTNet forward: x complex [B, E, T, Y, X] -> same."""
    B, E, T, Y, X = x.shape
    pad, depth, heads = meta["pad"], meta["depth"], meta["heads"]
    Tp = T + 2 * pad
    if Tp % 4 or Y % 4 or X % 4:
        raise NotImplementedError("dl_cs HIP DiT: T + 2 pad, Y and X must be multiples of 4")
    dev = x.device
    grid = (B, Tp, Y, X)
    geo = Geo.get(B, Tp, Y, X, dev)
    cin = 2 * E
    resid = meta["residual_convs"]
    D = P[n["pe_w"]].shape[0]
    hd = D // heads
    if hd > 32 or hd % 4 or D % heads:
        raise NotImplementedError(f"dl_cs HIP DiT: head dim {D}/{heads} must be <= 32 and a multiple of 4")
    u = K.swin_pre(x.contiguous(), torch.float32, pad, PAD_CIN)                 # [V, 8]
    sv = dict(u=u, grid=grid, geo=geo, shape=(B, E, T, Y, X))
    if resid:
        col = _im2col(u, cin, grid, +1, _tld(D))                                  # [V, 108 (128)]
        Wsfe = K.permute(P[n["sfe_w"]], (D, 27, cin), (cin * 27, 1, 27))         # [D][tap][ci]
        if _thin_h3(D):
            Wsfe = _pad2(Wsfe.view(D, 27 * cin), D, col.shape[1])
            res = _gemm_h3(col, Wsfe, D, bias=P[n["sfe_b"]])                     # [V, D]  SFE (dit:1339)
        else:
            res = K.linear(col, Wsfe.view(D, 27 * cin), bias=P[n["sfe_b"]])
        sv.update(col=col, Wsfe=Wsfe, res=res)
        src, ldsrc = res, D
    else:
        src, ldsrc = u, PAD_CIN
    # patch embed + pos embed (dit:570-571)
    Wpe = _patch_weights(P, n, D, ldsrc)
    pos_idx = meta["pos_index"](geo)
    pos = K.gather_rows(P[n["pos"]].view(-1, D), pos_idx, geo.M, torch.float32)
    tok = _empty((geo.M, D), dev)
    if _h3_ok(Wpe):
        _gemm_h3(src.view(geo.M, 32 * ldsrc), Wpe, D, out=tok, bias=P[n["pe_b"]], res=pos, row_map=geo.sub2tok)
    else:
        K.gemm(src.view(geo.M, 32 * ldsrc), Wpe, tok, geo.M, D, 32 * ldsrc, 32 * ldsrc, 32 * ldsrc, D,
               bias=P[n["pe_b"]], res=pos, ldr=D, row_map=geo.sub2tok)
    sv.update(Wpe=Wpe, src=src, ldsrc=ldsrc)
    # conditioning c = t_embedder(t) + y_embedder(labels) (dit:572-574)
    tf = _empty((B, 256), dev)
    _lib.call("dlcs_timestep_embedding", K.p(t), B, 256, 10000.0, K.p(tf), K.S())
    th = K.linear(tf, P[n["t0_w"]], bias=P[n["t0_b"]])
    ts = _vec(0, th)
    te = K.linear(ts, P[n["t2_w"]], bias=P[n["t2_b"]])
    ye = K.gather_rows(P[n["y_tab"]], labels, B, torch.float32)
    c = _vec(3, te, ye)
    scv = _vec(0, c)
    sv.update(tf=tf, th=th, ts=ts, c=c, sc=scv, labels=labels)
    # blocks (dit:575-576)
    svb = []
    for i in range(depth):
        tok, s_ = block_forward(P, n["blocks"][i], tok, scv, geo, heads, hd, fp8=meta.get("fp8", False))
        svb.append(s_)
    sv["blocks"] = svb
    # final layer (dit:404-408) + unpatchify (dit:515-543) into the blocked layout
    mod = K.linear(scv, P[n["fa_w"]], bias=P[n["fa_b"]])                       # [B, 2D]: shift | scale
    gam_f = _vec(2, mod[:, D:].contiguous())
    sh_f = mod[:, :D].contiguous()
    hf, mf, rf = _empty((geo.M, D), dev), _empty((geo.M,), dev), _empty((geo.M,), dev)
    for b in range(B):
        rs = slice(b * geo.Mb, (b + 1) * geo.Mb)
        hf[rs], mf[rs], rf[rs] = _ln(tok[rs], gam_f[b], sh_f[b], geo.Mb)
    sv.update(tok_last=tok, gam_f=gam_f, hf=hf, mf=mf, rf=rf)
    Wl, bl = P[n["fl_w"]], P[n["fl_b"]]
    Cout = Wl.shape[0] // 32
    if resid:
        # r = relu(DiT(res) + res): the final ConvBlock's ReLU (dit:1344) after the residual
        r = _empty((geo.V, D), dev)
        if _h3_ok(Wl):
            _gemm_h3(hf, Wl, 32 * D, out=r.view(geo.M, 32 * D), bias=bl, res=res.view(geo.M, 32 * D),
                     row_map=geo.tok2sub, act=7)
        else:
            K.gemm(hf, Wl, r.view(geo.M, 32 * D), geo.M, 32 * D, D, D, D, 32 * D, bias=bl,
                   res=res.view(geo.M, 32 * D), ldr=32 * D, row_map=geo.tok2sub, act=7)
        # final conv D -> cin (dit:1302): P = r Wf2^T, then the 27-tap gather-sum
        Wf2 = K.permute(P[n["fin_w"]], (27, cin, D), (1, D * 27, 27)).view(27 * cin, D)
        if _thin_h3(D):
            Wf2 = _pad2(Wf2, _tld(D), D)
            Pf = _gemm_h3(r, Wf2, Wf2.shape[0])                                  # [V, 128]
        else:
            Pf = K.linear(r, Wf2)                                                # [V, 108]
        o = _col2im(Pf, cin, PAD_CIN, grid, +1, bias=P[n["fin_b"]])
        sv.update(r=r, Wf2=Wf2)
        from . import engine
        if engine.CAPTURE is not None:                     # test hook: the final ConvBlock's ReLU decisions
            engine.CAPTURE.append(dict(relu_inputs=[r], grid=grid, C=D))
    else:
        # DiTNet: the Linear's (p, q, r, c) outputs straight into the thin blocked volume
        Wlp, blp = _padded_final_linear(Wl, bl, Cout)
        o = _empty((geo.V, PAD_CIN), dev)
        if _h3_ok(Wlp):
            _gemm_h3(hf, Wlp, 32 * PAD_CIN, out=o.view(geo.M, 32 * PAD_CIN), bias=blp, row_map=geo.tok2sub)
        else:
            K.gemm(hf, Wlp, o.view(geo.M, 32 * PAD_CIN), geo.M, 32 * PAD_CIN, D, D, D, 32 * PAD_CIN, bias=blp,
                   row_map=geo.tok2sub)
        sv.update(Wlp=Wlp, cout=Cout)
    out = K.swin_post(o, (B, E, T, Y, X), pad)
    return out, sv


def regularizer_backward(P, n, sv, gout, meta, G):
    B, E, T, Y, X = sv["shape"]
    pad, depth, heads = meta["pad"], meta["depth"], meta["heads"]
    resid = meta["residual_convs"]
    geo, grid = sv["geo"], sv["grid"]
    dev = gout.device
    D = P[n["pe_w"]].shape[0]
    hd = D // heads
    cin = 2 * E
    go = K.swin_post_bwd(gout.contiguous(), torch.float32, pad, PAD_CIN)       # [V, 8]
    Wl = P[n["fl_w"]]
    if resid:
        # final conv: o = col2im(+1)(r Wf2^T) + b
        K.colsum(go, G[n["fin_b"]], rows=geo.V, C=cin, ld=PAD_CIN)
        G2c = _im2col(go, cin, grid, -1, _tld(D))                                  # [V, 108 (128)]
        dWf2 = _zeros((G2c.shape[1], D), dev)
        _lin_grads(G2c, sv["r"], dWf2, None)
        K.permute(dWf2, (cin, D, 27), (D, 1, cin * D), out=G[n["fin_w"]].view(cin, D, 27), accumulate=1)
        if _thin_h3(D):                                                            # d (DiT(res) + res) [V, D]
            ds = _gemm_h3(G2c, sv["Wf2"], D, trans=True, act=6, aux=sv["r"])
        else:
            ds = K.linear_dx(G2c, sv["Wf2"], act=6, aux=sv["r"])
        dsub = ds.view(geo.M, 32 * D)
    else:
        dsub = go.view(geo.M, 32 * PAD_CIN)
    # final Linear (row-mapped into subpatches): out[tok2sub[m]] = hf[m] Wl^T + bl (+ res)
    Wg = Wl if resid else sv["Wlp"]
    Cw = Wg.shape[0]
    dhf = _empty((geo.M, D), dev)
    if _h3_ok(Wg, True):
        _gemm_h3(dsub, Wg, D, trans=True, out=dhf, row_map=geo.sub2tok)
    else:
        K.gemm(dsub, Wg, dhf, geo.M, D, Cw, Cw, D, D, b_trans=1, row_map=geo.sub2tok)
    hf_sub = K.gather_rows(sv["hf"], geo.sub2tok, geo.M, torch.float32)
    if resid:
        _lin_grads(dsub, hf_sub, G[n["fl_w"]], G[n["fl_b"]])
    else:
        cout = sv["cout"]
        dWp_, dbp_ = _zeros((Cw, D), dev), _zeros((Cw,), dev)
        _lin_grads(dsub, hf_sub, dWp_, dbp_)
        G[n["fl_w"]].view(32, cout, D).add_(dWp_.view(32, PAD_CIN, D)[:, :cout])
        G[n["fl_b"]].view(32, cout).add_(dbp_.view(32, PAD_CIN)[:, :cout])
    dmodf = _zeros((B, 2 * D), dev)
    dtok = _zeros((geo.M, D), dev)
    for b in range(B):
        rs = slice(b * geo.Mb, (b + 1) * geo.Mb)
        K.layernorm_bwd(dhf[rs], sv["tok_last"][rs], sv["gam_f"][b], sv["mf"][rs], sv["rf"][rs], dtok[rs],
                        dmodf[b, D:], dmodf[b, :D])
    dsc = _zeros((B, D), dev)
    _lin_grads(dmodf, sv["sc"], G[n["fa_w"]], G[n["fa_b"]])
    K.linear_dx(dmodf, P[n["fa_w"]], out=dsc, accumulate=1)
    # blocks, last first
    for i in reversed(range(depth)):
        dtok = block_backward(P, G, n["blocks"][i], sv["blocks"][i], dtok, sv["sc"], dsc, geo, heads, hd)
    # conditioning: sc = SiLU(c), c = te + table[labels], te = SiLU(th) W2^T + b2, th = tf W0^T + b0
    dc = _vec(1, dsc, sv["c"])
    _lib.call("dlcs_rows_add", K.p(G[n["y_tab"]]), K.p(sv["labels"]), K.p(dc), B, D, K.S())
    _lin_grads(dc, sv["ts"], G[n["t2_w"]], G[n["t2_b"]])
    dts = K.linear_dx(dc, P[n["t2_w"]])
    dth = _vec(1, dts, sv["th"])
    _lin_grads(dth, sv["tf"], G[n["t0_w"]], G[n["t0_b"]])
    # patch embed: tok[sub2tok[j]] = src_sub[j] Wpe^T + b + pos
    dtok_sub = K.gather_rows(dtok, geo.sub2tok, geo.M, torch.float32)
    K.colsum(dtok, G[n["pe_b"]])
    ldsrc = sv["ldsrc"]
    src_sub = sv["src"].view(geo.M, 32 * ldsrc)
    dWpe = _zeros((D, 32 * ldsrc), dev)
    _lin_grads(dtok_sub, src_sub, dWpe, None)
    Cpe = P[n["pe_w"]].shape[1]
    K.permute(dWpe.view(D, 32, ldsrc)[:, :, :Cpe].contiguous(), (D, Cpe, 32), (32 * Cpe, 1, Cpe),
              out=G[n["pe_w"]].view(D, Cpe, 32), accumulate=1)
    if resid:
        # d res = ds (the final residual) + patch-embed dgrad
        dres = _empty((geo.V, D), dev)
        if _h3_ok(sv["Wpe"], True):
            _gemm_h3(dtok_sub, sv["Wpe"], 32 * D, trans=True, out=dres.view(geo.M, 32 * D), res=ds.view(geo.M, 32 * D))
        else:
            K.gemm(dtok_sub, sv["Wpe"], dres.view(geo.M, 32 * D), geo.M, 32 * D, D, D, 32 * D, 32 * D, b_trans=1,
                   res=ds.view(geo.M, 32 * D), ldr=32 * D)
        # SFE: res = col Wsfe^T + b
        tld = sv["col"].shape[1]
        dWs = _zeros((D, tld), dev)
        _lin_grads(dres, sv["col"], dWs, G[n["sfe_b"]])
        K.permute(dWs, (D, cin, 27), (tld, 1, cin), out=G[n["sfe_w"]].view(D, cin, 27), accumulate=1)
        if _thin_h3(D):
            P2 = _gemm_h3(dres, sv["Wsfe"], tld, trans=True)                    # [V, 128]
        else:
            P2 = K.linear_dx(dres, sv["Wsfe"].view(D, 27 * cin))                # [V, 108]
        du = _col2im(P2, cin, PAD_CIN, grid, -1)
    else:
        du = _empty((geo.V, PAD_CIN), dev)
        if _h3_ok(sv["Wpe"], True):
            _gemm_h3(dtok_sub, sv["Wpe"], 32 * PAD_CIN, trans=True, out=du.view(geo.M, 32 * PAD_CIN))
        else:
            K.gemm(dtok_sub, sv["Wpe"], du.view(geo.M, 32 * PAD_CIN), geo.M, 32 * PAD_CIN, D, D, 32 * PAD_CIN,
                   32 * PAD_CIN, b_trans=1)
    return K.swin_pre_bwd(du, (B, E, T, Y, X), pad)


class _DiTFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, t, labels, meta, *plist):
        P = dict(zip(meta["order"], plist))
        out, sv = regularizer_forward(P, meta["names"], x.to(torch.complex64), t, labels, meta)
        ctx.state = (P, sv, meta)
        return out

    @staticmethod
    def backward(ctx, gout):
        P, sv, meta = ctx.state
        ctx.state = None
        G = {k: (torch.zeros_like(v) if meta["trainable"][k] else None) for k, v in P.items()}
        Gz = {k: (g if g is not None else _zeros(P[k].shape, gout.device)) for k, g in G.items()}
        gx = regularizer_backward(P, meta["names"], sv, gout.to(torch.complex64), meta, Gz)
        return (gx, None, None, None) + tuple(G[k] for k in meta["order"])


def dit_regularizer_forward(mod, x, t, c):
    """DiTResNet / DiTNet forward (dit:1270-1282, :1334-1350) through the HIP engine."""
    from .swin3D import get_compute_dtype
    if get_compute_dtype() != torch.float32:
        raise NotImplementedError("dl_cs HIP DiT: fp32 compute dtype")
    if not x.is_cuda:
        raise RuntimeError("dl_cs HIP DiT needs GPU tensors (no CPU fallback in the product path)")
    dit = mod.DiT
    depth, heads = len(dit.blocks), dit.num_heads
    params = dict(mod.named_parameters())
    order = list(params.keys())
    trainable = {k: p.requires_grad for k, p in params.items()}
    t = torch.as_tensor(t, device=x.device).reshape(-1).float().contiguous()
    labels = dit.y_embedder.effective_labels(torch.as_tensor(c, device=x.device).reshape(-1), dit.training)
    B = x.shape[0]
    if t.numel() == 1 and B > 1:
        t = t.expand(B).contiguous()
    if labels.numel() == 1 and B > 1:
        labels = labels.expand(B)
    labels = labels.to(torch.int32).contiguous()
    pe = dit.pos_embedder
    # fp8 only when no gradient can be requested of this call (inside the autograd
    # Function's forward grad mode is always off, so decide here)
    grad = torch.is_grad_enabled() and (x.requires_grad or any(trainable.values()))
    meta = dict(order=order, names=names(mod, depth), depth=depth, heads=heads, pad=mod.pad_size,
                residual_convs=mod.residual_convs, trainable=trainable,
                pos_index=lambda geo: _pos_index(pe, geo), fp8=FP8 and not grad)
    return _DiTFn.apply(x, t, labels, meta, *[params[k] for k in order])


_POS = {}


def _pos_index(pe, geo):
    key = (tuple(pe.max_grid_size), geo.B, geo.F, geo.Hh, geo.Ww, str(geo.sub2tok.device))
    idx = _POS.get(key)
    if idx is None:
        one = pe.index((geo.F, geo.Hh, geo.Ww))
        idx = _POS[key] = _dev_i32(np.tile(one, geo.B), geo.sub2tok.device)
    return idx


def dit_forward_real(dit, x, t, y):
    raise NotImplementedError("dl_cs: DiT.forward on its own is not on the HIP path; call DiTResNet / DiTNet")
