"""HIP forward / hand-scheduled backward of LatteNet (lat = dl_cs/models/Latte.py),
one autograd node per network call, on the DiT engine's kernels and helpers
(dl_cs.models.dit_engine: adaLN LayerNorm, flash MHSA, gated Linears, the fp8
token-Linear path).

Layouts (fp32; B samples, time padded to F = T + 2 pad frames, Y, X multiples of 4):
  * the 2E-channel volume in the patch-blocked channels-last layout of the Swin
    path (row(b,t,y,x) = patch-of-4x4x4 * 64 + (t%4) 16 + (y%4) 4 + x%4): a 2-D
    (4, 4) patch of one frame (lat:89-147) is 16 consecutive rows, so the patch
    embed is one GEMM [patches, 16 C] x [16 C, D] and the final Linear's (p, q, c)
    columns (unpatchify2, lat:450-475) are exactly the 16 rows x C channels of a
    patch -- no im2col, no unpatchify copy;
  * tokens [M = B F Np, D] in the reference's spatial order (b, f, p), p = h W + w
    (lat:142-145): the spatial blocks attend over contiguous sequences of Np; the
    temporal blocks (lat:529-542, rearrange '(b f) t d -> (b t) f d') read their
    LayerNorm input through a row map into (b, p, f) order and their proj GEMM
    scatters back (row_map), exactly the DiT engine's per-position attention.
Gated residual branches g * (x W^T + b) (lat:313-314) run as one GEMM on
gate-scaled weights; adaLN-modulated LayerNorms (lat:33-34) are dlcs_layernorm
with gamma = 1 + scale, beta = shift; the frame table (lat:532-535) is added to
every token before the first temporal block (frozen: no gradient).
"""
import numpy as np
import torch

from .. import _lib
from . import _ops as K
from .dit_engine import (PAD_CIN, _dev_i32, _dx, _empty, _gated_grad, _gated_pack, _gemm_h3, _h3_ok, _lin,
                         _lin_grads, _ln, _mhsa, _mhsa_bwd, _packs, _scale_rows, _vec, _zeros)

_GEO = {}


class LGeo:
    """Index maps of one (B, F, Y, X) Latte geometry (host-built once, cached)."""

    def __init__(self, B, F, Y, X, device):
        self.B, self.F, self.Y, self.X = B, F, Y, X
        self.Hp, self.Wp = Y // 4, X // 4
        self.Np = self.Hp * self.Wp
        self.V = B * F * Y * X
        self.M = B * F * self.Np
        self.Mb = self.M // B
        Hp, Wp, Np = self.Hp, self.Wp, self.Np
        b, f, h, w = np.meshgrid(np.arange(B), np.arange(F), np.arange(Hp), np.arange(Wp), indexing="ij")
        tok = (b * F + f) * Np + h * Wp + w                              # (b, f, p) token order
        sub = (((b * (F // 4) + f // 4) * Hp + h) * Wp + w) * 4 + f % 4   # 16-row 2-D patch of the blocked layout
        tim = (b * Np + h * Wp + w) * F + f                              # (b, p, f): temporal sequences
        tok, sub, tim, f = tok.reshape(-1), sub.reshape(-1), tim.reshape(-1), f.reshape(-1)
        sub2tok = np.empty(self.M, np.int64)
        sub2tok[sub] = tok
        tok2sub = np.empty(self.M, np.int64)
        tok2sub[tok] = sub
        tim2tok = np.empty(self.M, np.int64)
        tim2tok[tim] = tok
        frame = np.empty(self.M, np.int64)
        frame[tok] = f
        self.sub2tok = _dev_i32(sub2tok, device)
        self.tok2sub = _dev_i32(tok2sub, device)
        self.tim2tok = _dev_i32(tim2tok, device)
        self.frame = _dev_i32(frame, device)          # token row -> frame (the frame-table rows)

    @staticmethod
    def get(B, F, Y, X, device):
        key = (B, F, Y, X, str(device))
        g = _GEO.get(key)
        if g is None:
            g = _GEO[key] = LGeo(B, F, Y, X, device)
        return g


def names(depth):
    p = "Latte."
    n = dict(pe_w=p + "x_embedder.proj.weight", pe_b=p + "x_embedder.proj.bias",
             pos=p + "pos_embedder.pos_embed_table", temp=p + "temp_embedder.temp_embed_table",
             t0_w=p + "t_embedder.mlp.0.weight", t0_b=p + "t_embedder.mlp.0.bias",
             t2_w=p + "t_embedder.mlp.2.weight", t2_b=p + "t_embedder.mlp.2.bias",
             fa_w=p + "final_layer.adaLN_modulation.1.weight", fa_b=p + "final_layer.adaLN_modulation.1.bias",
             fl_w=p + "final_layer.linear.weight", fl_b=p + "final_layer.linear.bias")
    blocks = []
    for i in range(depth):
        q = f"{p}blocks.{i}."
        blocks.append(dict(qkv_w=q + "attn.qkv.weight", qkv_b=q + "attn.qkv.bias",
                           proj_w=q + "attn.proj.weight", proj_b=q + "attn.proj.bias",
                           fc1_w=q + "mlp.fc1.weight", fc1_b=q + "mlp.fc1.bias",
                           fc2_w=q + "mlp.fc2.weight", fc2_b=q + "mlp.fc2.bias",
                           ada_w=q + "adaLN_modulation.1.weight", ada_b=q + "adaLN_modulation.1.bias"))
    n["blocks"] = blocks
    return n


# ---------------------------------------------------------------------------- TransformerBlock
def block_forward(P, nb, tok, sc, geo, heads, hd, temporal, fp8=False):
    """lat:311-316 on tokens tok [M, D] (spatial order); temporal: the attention
    runs over the frames of each patch position (lat:529-542)."""
    dev = tok.device
    D = tok.shape[1]
    M, Mb, B = geo.M, geo.Mb, geo.B
    scale = hd ** -0.5
    mod = _lin(fp8, sc, P[nb["ada_w"]], bias=P[nb["ada_b"]])               # [B, 6D] (lat:312)
    ch = lambda k: mod[:, k * D:(k + 1) * D].contiguous()                  # noqa: E731
    sh_a, g_a, sh_m, g_m = ch(0), ch(2), ch(3), ch(5)
    gam_a, gam_m = _vec(2, ch(1)), _vec(2, ch(4))
    Wqkv, bqkv, Wp, bp = P[nb["qkv_w"]], P[nb["qkv_b"]], P[nb["proj_w"]], P[nb["proj_b"]]
    W1, b1, W2, b2 = P[nb["fc1_w"]], P[nb["fc1_b"]], P[nb["fc2_w"]], P[nb["fc2_b"]]
    hq, h1p = (None, None) if fp8 else _packs((Wqkv, False), (W1, False))
    # attention branch: x1 = x + g_msa attn(modulate(norm1 x)) (lat:313)
    h1, m1, r1 = _empty((M, D), dev), _empty((M,), dev), _empty((M,), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        if temporal:
            h1[rs], m1[rs], r1[rs] = _ln(tok, gam_a[b], sh_a[b], Mb, src_map=geo.tim2tok[rs])
        else:
            h1[rs], m1[rs], r1[rs] = _ln(tok[rs], gam_a[b], sh_a[b], Mb)
    qkv = _lin(fp8, h1, Wqkv, bias=bqkv, hp=hq)
    nseq, N = (B * geo.Np, geo.F) if temporal else (B * geo.F, geo.Np)
    a, lse = _mhsa(qkv, nseq, N, heads, hd, scale)
    x1 = _empty((M, D), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        Wg, bg = _scale_rows(Wp, bp, g_a[b])
        hg = _gated_pack(fp8, Wg)
        if temporal:
            _lin(fp8, a[rs], Wg, bias=bg, out=x1, res=tok, row_map=geo.tim2tok[rs], hp=hg)
        else:
            _lin(fp8, a[rs], Wg, bias=bg, out=x1[rs], res=tok[rs], hp=hg)
    # Mlp branch: x2 = x1 + g_mlp mlp(modulate(norm2 x1)) (lat:314)
    h2, m2, r2 = _empty((M, D), dev), _empty((M,), dev), _empty((M,), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        h2[rs], m2[rs], r2[rs] = _ln(x1[rs], gam_m[b], sh_m[b], Mb)
    upre = _empty((M, W1.shape[0]), dev)
    v = _lin(fp8, h2, W1, bias=b1, act=4, aux_out=upre, hp=h1p)
    x2 = _empty((M, D), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        Wg, bg = _scale_rows(W2, b2, g_m[b])
        _lin(fp8, v[rs], Wg, bias=bg, out=x2[rs], res=x1[rs], hp=_gated_pack(fp8, Wg))
    sv = dict(mod=mod, gam_a=gam_a, gam_m=gam_m, x0=tok, x1=x1, h1=h1, h2=h2, m1=m1, r1=r1, m2=m2, r2=r2,
              qkv=qkv, a=a, lse=lse, upre=upre, v=v, temporal=temporal)
    return x2, sv


def block_backward(P, G, nb, sv, dy, sc, dsc, geo, heads, hd):
    """Backward of block_forward: returns d tokens; accumulates parameter grads into
    G and d SiLU(c) into dsc."""
    dev = dy.device
    D = dy.shape[1]
    M, Mb, B = geo.M, geo.Mb, geo.B
    scale = hd ** -0.5
    temporal = sv["temporal"]
    mod = sv["mod"]
    ch = lambda k: mod[:, k * D:(k + 1) * D].contiguous()                  # noqa: E731
    g_a, g_m = ch(2), ch(5)
    Wqkv, Wp, bp = P[nb["qkv_w"]], P[nb["proj_w"]], P[nb["proj_b"]]
    W1, W2, b2 = P[nb["fc1_w"]], P[nb["fc2_w"]], P[nb["fc2_b"]]
    dmod = _zeros((B, 6 * D), dev)
    dch = lambda k: dmod[:, k * D:(k + 1) * D]                              # noqa: E731
    dgam = {k: _zeros((B, D), dev) for k in ("a", "m")}
    dbet = {k: _zeros((B, D), dev) for k in ("a", "m")}
    dgate = {k: _zeros((B, D), dev) for k in ("a", "m")}
    hqT, h1T = _packs((Wqkv, True), (W1, True))
    # Mlp: x2 = x1 + g_m (v W2^T + b2)
    du = _empty((M, W1.shape[0]), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        Wg, _ = _scale_rows(W2, b2, g_m[b])
        _dx(dy[rs], Wg, _gated_pack(False, Wg, True), out=du[rs], act=5, aux=sv["upre"][rs])
        G2, cs = _zeros(W2.shape, dev), _zeros((D,), dev)
        _lin_grads(dy[rs], sv["v"][rs], G2, cs)
        _gated_grad(W2, b2, G2, cs, g_m[b], G[nb["fc2_w"]], G[nb["fc2_b"]], dgate["m"][b])
    dh2 = _dx(du, W1, h1T)
    _lin_grads(du, sv["h2"], G[nb["fc1_w"]], G[nb["fc1_b"]])
    dx1 = _empty((M, D), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        K.layernorm_bwd(dh2[rs], sv["x1"][rs], sv["gam_m"][b], sv["m2"][rs], sv["r2"][rs], dx1[rs],
                        dgam["m"][b], dbet["m"][b], dx_in=dy[rs])
    # attention: x1[row(j)] = x0[row(j)] + g_a (a[j] Wp^T + bp), row = tim2tok (temporal) or j
    dx1_s = K.gather_rows(dx1, geo.tim2tok, M, torch.float32) if temporal else dx1
    da = _empty((M, D), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        Wg, _ = _scale_rows(Wp, bp, g_a[b])
        _dx(dx1_s[rs], Wg, _gated_pack(False, Wg, True), out=da[rs])
        Gp, cs = _zeros(Wp.shape, dev), _zeros((D,), dev)
        _lin_grads(dx1_s[rs], sv["a"][rs], Gp, cs)
        _gated_grad(Wp, bp, Gp, cs, g_a[b], G[nb["proj_w"]], G[nb["proj_b"]], dgate["a"][b])
    nseq, N = (B * geo.Np, geo.F) if temporal else (B * geo.F, geo.Np)
    dqkv = _mhsa_bwd(sv["qkv"], sv["a"], da, sv["lse"], nseq, N, heads, hd, scale)
    dh1 = _dx(dqkv, Wqkv, hqT)
    _lin_grads(dqkv, sv["h1"], G[nb["qkv_w"]], G[nb["qkv_b"]])
    dx0 = _empty((M, D), dev)
    for b in range(B):
        rs = slice(b * Mb, (b + 1) * Mb)
        if temporal:
            K.layernorm_bwd(dh1[rs], sv["x0"], sv["gam_a"][b], sv["m1"][rs], sv["r1"][rs], dx0, dgam["a"][b],
                            dbet["a"][b], src_map=geo.tim2tok[rs], dx_in=dx1)
        else:
            K.layernorm_bwd(dh1[rs], sv["x0"][rs], sv["gam_a"][b], sv["m1"][rs], sv["r1"][rs], dx0[rs],
                            dgam["a"][b], dbet["a"][b], dx_in=dx1[rs])
    # adaLN: mod = SiLU(c) W^T + b, chunks (shift_msa, scale_msa, gate_msa, shift_mlp, scale_mlp, gate_mlp)
    for k, src in ((0, dbet["a"]), (1, dgam["a"]), (2, dgate["a"]), (3, dbet["m"]), (4, dgam["m"]), (5, dgate["m"])):
        dch(k).copy_(src)
    _lin_grads(dmod, sc, G[nb["ada_w"]], G[nb["ada_b"]])
    K.linear_dx(dmod, P[nb["ada_w"]], out=dsc, accumulate=1)
    return dx0


# ---------------------------------------------------------------------------- whole network
def _patch_weights(P, n, D, cin):
    """GEMM layouts of the per-frame patch embed [D][(kh, kw)][c at stride PAD_CIN]
    and of the final Linear [(p, q)][c at stride PAD_CIN][D] (lat:128, :449-475)."""
    Wpe = P[n["pe_w"]]                                          # [D, C, 4, 4]
    g = _zeros((D, 16, PAD_CIN), Wpe.device)
    g[:, :, :cin].copy_(K.permute(Wpe, (D, 16, cin), (cin * 16, 1, 16)).view(D, 16, cin))
    Wl, bl = P[n["fl_w"]], P[n["fl_b"]]                         # [16 C, D], [16 C]
    Wlp = _zeros((16, PAD_CIN, Wl.shape[1]), Wl.device)
    Wlp[:, :cin].copy_(Wl.view(16, cin, -1))
    blp = _zeros((16, PAD_CIN), Wl.device)
    blp[:, :cin].copy_(bl.view(16, cin))
    return g.view(D, 16 * PAD_CIN), Wlp.view(16 * PAD_CIN, -1), blp.view(-1)


def network_forward(P, n, x, t, meta):
    """LatteNet forward (lat:926-937 with Latte.forward lat:477-560): x complex
    [B, E, T, Y, X] -> same."""
    B, E, T, Y, X = x.shape
    pad, depth, heads = meta["pad"], meta["depth"], meta["heads"]
    F = T + 2 * pad
    if F % 4 or Y % 4 or X % 4:
        raise NotImplementedError("dl_cs HIP Latte: T + 2 pad, Y and X must be multiples of 4")
    dev = x.device
    geo = LGeo.get(B, F, Y, X, dev)
    cin = 2 * E
    D = P[n["pe_w"]].shape[0]
    hd = D // heads
    if hd > 32 or hd % 4 or D % heads:
        raise NotImplementedError(f"dl_cs HIP Latte: head dim {D}/{heads} must be <= 32 and a multiple of 4")
    if F > P[n["temp"]].shape[1]:
        raise ValueError(f"{F} frames exceed the TempEmbed table ({P[n['temp']].shape[1]})")
    u = K.swin_pre(x.contiguous(), torch.float32, pad, PAD_CIN)                 # [V, 8]  (lat:882-894)
    Wpe, Wlp, blp = _patch_weights(P, n, D, cin)
    # patch embed + position table (lat:513-516), token order via the row map
    pos = K.gather_rows(P[n["pos"]].view(-1, D), meta["pos_index"](geo), geo.M, torch.float32)
    tok = _empty((geo.M, D), dev)
    if _h3_ok(Wpe):
        _gemm_h3(u.view(geo.M, 16 * PAD_CIN), Wpe, D, out=tok, bias=P[n["pe_b"]], res=pos, row_map=geo.sub2tok)
    else:
        K.gemm(u.view(geo.M, 16 * PAD_CIN), Wpe, tok, geo.M, D, 16 * PAD_CIN, 16 * PAD_CIN, 16 * PAD_CIN, D,
               bias=P[n["pe_b"]], res=pos, ldr=D, row_map=geo.sub2tok)
    # conditioning c = t_embedder(t) (lat:521-523; extras = 1: no label / text term)
    tf = _empty((B, 256), dev)
    _lib.call("dlcs_timestep_embedding", K.p(t), B, 256, 10000.0, K.p(tf), K.S())
    th = K.linear(tf, P[n["t0_w"]], bias=P[n["t0_b"]])
    ts = _vec(0, th)
    c = K.linear(ts, P[n["t2_w"]], bias=P[n["t2_b"]])
    scv = _vec(0, c)
    fp8 = meta.get("fp8", False)
    svb = []
    for i in range(depth):
        if i == 1:                                                # + temp_embed before the first temporal block
            temp = K.gather_rows(P[n["temp"]].view(-1, D), geo.frame, geo.M, torch.float32)
            tok = _vec(3, tok, temp)
        tok, s_ = block_forward(P, n["blocks"][i], tok, scv, geo, heads, hd, temporal=(i % 2 == 1), fp8=fp8)
        svb.append(s_)
    # final layer (lat:331-336) + unpatchify2 (lat:450-475) into the blocked layout
    mod = K.linear(scv, P[n["fa_w"]], bias=P[n["fa_b"]])                       # [B, 2D]: shift | scale
    gam_f = _vec(2, mod[:, D:].contiguous())
    sh_f = mod[:, :D].contiguous()
    hf, mf, rf = _empty((geo.M, D), dev), _empty((geo.M,), dev), _empty((geo.M,), dev)
    for b in range(B):
        rs = slice(b * geo.Mb, (b + 1) * geo.Mb)
        hf[rs], mf[rs], rf[rs] = _ln(tok[rs], gam_f[b], sh_f[b], geo.Mb)
    o = _empty((geo.V, PAD_CIN), dev)
    if _h3_ok(Wlp):
        _gemm_h3(hf, Wlp, 16 * PAD_CIN, out=o.view(geo.M, 16 * PAD_CIN), bias=blp, row_map=geo.tok2sub)
    else:
        K.gemm(hf, Wlp, o.view(geo.M, 16 * PAD_CIN), geo.M, 16 * PAD_CIN, D, D, D, 16 * PAD_CIN, bias=blp,
               row_map=geo.tok2sub)
    out = K.swin_post(o, (B, E, T, Y, X), pad)                                 # lat:896-907
    sv = dict(u=u, geo=geo, shape=(B, E, T, Y, X), Wpe=Wpe, Wlp=Wlp, tf=tf, th=th, ts=ts, c=c, sc=scv,
              blocks=svb, tok_last=tok, gam_f=gam_f, hf=hf, mf=mf, rf=rf)
    return out, sv


def network_backward(P, n, sv, gout, meta, G):
    B, E, T, Y, X = sv["shape"]
    pad, depth, heads = meta["pad"], meta["depth"], meta["heads"]
    geo = sv["geo"]
    dev = gout.device
    D = P[n["pe_w"]].shape[0]
    hd = D // heads
    cin = 2 * E
    go = K.swin_post_bwd(gout.contiguous(), torch.float32, pad, PAD_CIN)       # [V, 8]
    dsub = go.view(geo.M, 16 * PAD_CIN)
    # final Linear (row-mapped into the 2-D patches): o[tok2sub[m]] = hf[m] Wlp^T + blp
    Wlp = sv["Wlp"]
    Cw = Wlp.shape[0]
    dhf = _empty((geo.M, D), dev)
    if _h3_ok(Wlp, True):
        _gemm_h3(dsub, Wlp, D, trans=True, out=dhf, row_map=geo.sub2tok)
    else:
        K.gemm(dsub, Wlp, dhf, geo.M, D, Cw, Cw, D, D, b_trans=1, row_map=geo.sub2tok)
    hf_sub = K.gather_rows(sv["hf"], geo.sub2tok, geo.M, torch.float32)
    dWp_, dbp_ = _zeros((Cw, D), dev), _zeros((Cw,), dev)
    _lin_grads(dsub, hf_sub, dWp_, dbp_)
    G[n["fl_w"]].view(16, cin, D).add_(dWp_.view(16, PAD_CIN, D)[:, :cin])
    G[n["fl_b"]].view(16, cin).add_(dbp_.view(16, PAD_CIN)[:, :cin])
    dmodf = _zeros((B, 2 * D), dev)
    dtok = _zeros((geo.M, D), dev)
    for b in range(B):
        rs = slice(b * geo.Mb, (b + 1) * geo.Mb)
        K.layernorm_bwd(dhf[rs], sv["tok_last"][rs], sv["gam_f"][b], sv["mf"][rs], sv["rf"][rs], dtok[rs],
                        dmodf[b, D:], dmodf[b, :D])
    dsc = _zeros((B, D), dev)
    _lin_grads(dmodf, sv["sc"], G[n["fa_w"]], G[n["fa_b"]])
    K.linear_dx(dmodf, P[n["fa_w"]], out=dsc, accumulate=1)
    for i in reversed(range(depth)):                          # the frame-table add has an identity gradient
        dtok = block_backward(P, G, n["blocks"][i], sv["blocks"][i], dtok, sv["sc"], dsc, geo, heads, hd)
    # conditioning: sc = SiLU(c), c = SiLU(th) W2^T + b2, th = tf W0^T + b0
    dc = _vec(1, dsc, sv["c"])
    _lin_grads(dc, sv["ts"], G[n["t2_w"]], G[n["t2_b"]])
    dts = K.linear_dx(dc, P[n["t2_w"]])
    dth = _vec(1, dts, sv["th"])
    _lin_grads(dth, sv["tf"], G[n["t0_w"]], G[n["t0_b"]])
    # patch embed: tok[sub2tok[j]] = u_patch[j] Wpe^T + b + pos
    dtok_sub = K.gather_rows(dtok, geo.sub2tok, geo.M, torch.float32)
    K.colsum(dtok, G[n["pe_b"]])
    dWpe = _zeros((D, 16 * PAD_CIN), dev)
    _lin_grads(dtok_sub, sv["u"].view(geo.M, 16 * PAD_CIN), dWpe, None)
    K.permute(dWpe.view(D, 16, PAD_CIN)[:, :, :cin].contiguous(), (D, cin, 16), (16 * cin, 1, cin),
              out=G[n["pe_w"]].view(D, cin, 16), accumulate=1)
    du = _empty((geo.V, PAD_CIN), dev)
    if _h3_ok(sv["Wpe"], True):
        _gemm_h3(dtok_sub, sv["Wpe"], 16 * PAD_CIN, trans=True, out=du.view(geo.M, 16 * PAD_CIN))
    else:
        K.gemm(dtok_sub, sv["Wpe"], du.view(geo.M, 16 * PAD_CIN), geo.M, 16 * PAD_CIN, D, D, 16 * PAD_CIN,
               16 * PAD_CIN, b_trans=1)
    return K.swin_pre_bwd(du, (B, E, T, Y, X), pad)


class _LatteFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, t, meta, *plist):
        P = dict(zip(meta["order"], plist))
        out, sv = network_forward(P, meta["names"], x.to(torch.complex64), t, meta)
        ctx.state = (P, sv, meta)
        return out

    @staticmethod
    def backward(ctx, gout):
        P, sv, meta = ctx.state
        ctx.state = None
        n = meta["names"]
        used = {v for k, v in n.items() if k != "blocks"} | {v for b in n["blocks"] for v in b.values()}
        # parameters the forward never reads (LatteNet's SFE / final ConvBlocks) get no gradient
        G = {k: (torch.zeros_like(v) if meta["trainable"][k] and k in used else None) for k, v in P.items()}
        Gz = {k: (g if g is not None else _zeros(P[k].shape, gout.device)) for k, g in G.items()}
        gx = network_backward(P, n, sv, gout.to(torch.complex64), meta, Gz)
        return (gx, None, None) + tuple(G[k] for k in meta["order"])


_POS = {}


def _pos_index(pe, geo):
    """Rows of the 2-D position table in token order (PosEmbed.index, lat:183), tiled over (b, f)."""
    key = (tuple(pe.max_grid_size), geo.B, geo.F, geo.Hp, geo.Wp, str(geo.sub2tok.device))
    idx = _POS.get(key)
    if idx is None:
        one = pe.index((geo.Hp, geo.Wp))
        idx = _POS[key] = _dev_i32(np.tile(one, geo.B * geo.F), geo.sub2tok.device)
    return idx


def latte_forward(mod, x, t, c):
    """LatteNet.forward (lat:926-937) through the HIP engine; c (the class label) is
    unused, as in the reference (Latte extras = 1)."""
    from .swin3D import get_compute_dtype
    from . import dit_engine
    if get_compute_dtype() != torch.float32:
        raise NotImplementedError("dl_cs HIP Latte: fp32 compute dtype")
    if not x.is_cuda:
        raise RuntimeError("dl_cs HIP Latte needs GPU tensors (no CPU fallback in the product path)")
    lat = mod.Latte
    if lat.extras != 1:
        raise NotImplementedError("dl_cs HIP Latte: extras = 1 (LatteNet builds Latte with the default)")
    depth, heads = len(lat.blocks), lat.num_heads
    if depth % 2:
        raise NotImplementedError("dl_cs HIP Latte: spatial / temporal block pairs (an even NUM_LAYERS)")
    params = dict(mod.named_parameters())
    order = list(params.keys())
    trainable = {k: p.requires_grad for k, p in params.items()}
    t = torch.as_tensor(t, device=x.device).reshape(-1).float().contiguous()
    if t.numel() == 1 and x.shape[0] > 1:
        t = t.expand(x.shape[0]).contiguous()
    pe = lat.pos_embedder
    grad = torch.is_grad_enabled() and (x.requires_grad or any(trainable.values()))
    meta = dict(order=order, names=names(depth), depth=depth, heads=heads, pad=mod.pad_size, trainable=trainable,
                pos_index=lambda geo: _pos_index(pe, geo), fp8=dit_engine.FP8 and not grad)
    return _LatteFn.apply(x, t, meta, *[params[k] for k in order])
