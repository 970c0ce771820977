"""Kernel-level forward / backward of the Swin regularizer (s3d:371-435 with the
video-Swin backbone vst:534-761) on libdlcs_hip.

Data layout on the GPU:
  * 160-channel volumes [B, Tp, Y, X, C] in the patch-blocked channels-last
    layout (T = storage dtype) -- every 3x3x3 conv reads / writes it, and the
    k4s4 patch embed / unembed are plain GEMMs on it ([tokens, 64*C] rows);
  * Swin tokens: fp32 residual stream [tokens, C]; GEMM operands in T;
  * windowed rows [nwin*N, C] are produced by the LayerNorm gather and
    scattered back by the proj GEMM epilogue (window_partition / reverse and
    the cyclic shift never materialise separately).
Backward is hand-scheduled (no autograd inside): every saved activation and
every gradient kernel is explicit.
"""
import ctypes
import math
import weakref


import torch

from .. import diag as _diag
from . import _ops as K
from ._window import get_window_size as get_window_size_tuple


class BlockWeights:
    """Compute-dtype views of one SwinTransformerBlock3D's parameters."""

    NAMES = ("norm1.weight", "norm1.bias", "attn.relative_position_bias_table", "attn.qkv.weight",
             "attn.qkv.bias", "attn.proj.weight", "attn.proj.bias", "norm2.weight", "norm2.bias",
             "mlp.fc1.weight", "mlp.fc1.bias", "mlp.fc2.weight", "mlp.fc2.bias")

    LINEARS = ("attn.qkv.weight", "attn.proj.weight", "mlp.fc1.weight", "mlp.fc2.weight")

    def __init__(self, params, dtype, cast=None, hr=None):
        self.p = params                       # name -> fp32 parameter tensor
        # cast: the four Linear weights already in the compute dtype (one batched
        # cast per network, NetWeights), else cast here
        w = cast if cast is not None else [K.cast(params[n], dtype) for n in self.LINEARS]
        self.wqkv, self.wproj, self.wfc1, self.wfc2 = w
        # fp32 build: the eight Linear GEMMs (four forwards, four input gradients) on
        # the row-scaled f16x3 split (dlcs_gemm_h3r): packed W / W^T operands, one
        # pack launch per network (NetWeights), else packed here
        self.hr = None
        if h3r_ok(dtype, self.wqkv, self.wproj, self.wfc1, self.wfc2):
            if hr is None:
                hr = K.h3r_pack([(params[n], t) for t in (False, True) for n in self.LINEARS])
            self.hr = dict(zip(("qkv", "proj", "fc1", "fc2", "qkvT", "projT", "fc1T", "fc2T"), hr))


def h3r_ok(dtype, wqkv, wproj, wfc1, wfc2):
    """True when the block's Linears run on dlcs_gemm_h3r (fp32, N % 160 == 0 and
    K in {160, 480, 640} for every forward and input-gradient product)."""
    if dtype != torch.float32 or not H3R:
        return False
    ks = (160, 480, 640)
    return all(w.dim() == 2 and w.shape[0] % 160 == 0 and w.shape[1] % 160 == 0 and w.shape[0] in ks and
               w.shape[1] in ks for w in (wqkv, wproj, wfc1, wfc2))


class SwinGeometry:
    """Token grid, window / shift clamping and cached index tables (vst:417-431)."""

    def __init__(self, B, D, H, W, window, shift_enabled, device):
        self.B, self.D, self.H, self.W = B, D, H, W
        self.window0 = tuple(window)
        shift = tuple(i // 2 for i in window) if shift_enabled else (0, 0, 0)
        self.ws, self.ss = get_window_size_tuple((D, H, W), window, shift)
        self.shifted = any(s > 0 for s in self.ss)
        self.N = self.ws[0] * self.ws[1] * self.ws[2]
        self.part, self.rev, self.labels, self.nrows = K.window_tables(
            B, D, H, W, self.ws, self.ss if self.shifted else (0, 0, 0), device, self.shifted)
        self.nwin = self.nrows // self.N
        self.ntok = B * D * H * W


def block_forward(bw, geo, x, dtype, heads, drop_scale=(1.0, 1.0), mask=None, mask_nw=0):
    """SwinTransformerBlock3D (vst:254-273) on fp32 tokens x [ntok, C].
    drop_scale: DropPath factors (0 = branch dropped, 1/keep otherwise).
    mask: explicit additive mask (standalone API) instead of region labels."""
    P = bw.p
    C = x.shape[1]
    hd = C // heads
    scale = hd ** -0.5
    s = {}
    # LN1 fused with pad + cyclic shift + window_partition (vst:219-235)
    ln1, m1, r1 = K.layernorm_fwd(x, P["norm1.weight"], P["norm1.bias"], geo.nrows, src_map=geo.part,
                                  out_dtype=dtype)
    hr = bw.hr
    if hr is not None:
        qkv = K.linear_h3r(ln1, hr["qkv"], bw.wqkv.shape[0], bias=P["attn.qkv.bias"])       # vst:146
    else:
        qkv = K.linear(ln1, bw.wqkv, P["attn.qkv.bias"])
    labels = geo.labels if (geo.shifted and mask is None) else None
    if ATTN_PROFILE is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    att, lse = K.attn_fwd(qkv, P["attn.relative_position_bias_table"], labels, geo.nwin, geo.N, heads, hd,
                          geo.window0, scale, mask=mask if geo.shifted else None, mask_nw=mask_nw)
    if ATTN_PROFILE is not None:
        e1.record()
        ATTN_PROFILE.append((e0, e1, 4.0 * geo.nwin * geo.N * geo.N * hd * heads))   # Q K^T + P V
    # proj + window_reverse + roll back + crop + DropPath + residual (vst:168, :239-266)
    x1 = torch.empty_like(x)
    if drop_scale[0] == 0.0:
        x1.copy_(x)
    elif hr is not None:
        K.linear_h3r(att, hr["proj"], C, out=x1, bias=P["attn.proj.bias"], alpha=drop_scale[0], res=x,
                     row_map=geo.part)
    else:
        K.linear(att, bw.wproj, P["attn.proj.bias"], out=x1, alpha=drop_scale[0], res=x, row_map=geo.part)
    # LN2 -> fc1 + GELU -> fc2 + DropPath + residual (vst:251-252, :270-271)
    ln2, m2, r2 = K.layernorm_fwd(x1, P["norm2.weight"], P["norm2.bias"], geo.ntok, out_dtype=dtype)
    h1 = K.empty((geo.ntok, bw.wfc1.shape[0]), dtype, x.device)
    if hr is not None:
        a1 = K.linear_h3r(ln2, hr["fc1"], bw.wfc1.shape[0], bias=P["mlp.fc1.bias"], act=1, aux_out=h1)
    else:
        a1 = K.linear(ln2, bw.wfc1, P["mlp.fc1.bias"], act=1, aux_out=h1)
    x2 = torch.empty_like(x)
    if drop_scale[1] == 0.0:
        x2.copy_(x1)
    elif hr is not None:
        K.linear_h3r(a1, hr["fc2"], C, out=x2, bias=P["mlp.fc2.bias"], alpha=drop_scale[1], res=x1)
    else:
        K.linear(a1, bw.wfc2, P["mlp.fc2.bias"], out=x2, alpha=drop_scale[1], res=x1)
    s.update(x=x, ln1=ln1, m1=m1, r1=r1, qkv=qkv, att=att, lse=lse, x1=x1, ln2=ln2, m2=m2, r2=r2,
             h1=h1, a1=a1, drop=drop_scale, mask=mask, mask_nw=mask_nw)
    return x2, s


def block_backward(bw, geo, s, g2, grads, dtype, heads):
    """Backward of block_forward.  g2 fp32 [ntok, C]; accumulates parameter
    gradients into grads[name] (fp32) and returns dL/dx (fp32)."""
    P = bw.p
    C = g2.shape[1]
    hd = C // heads
    scale = hd ** -0.5
    d0, d1 = s["drop"]
    # weight / bias gradients of the block's four Linears: one grouped launch per
    # token count (bf16 path), else per-Linear split-K GEMM + column sum
    dw_jobs = []

    def weight_grad(gout, act, wname, bname, T):
        if K.dw_grouped_ok(T, [(gout, act)]):
            dw_jobs.append((T, (gout, act, grads[wname], grads[bname], 0)))
        else:
            K.linear_dw(gout, act, grads[wname])
            K.colsum(gout, grads[bname])

    # ---- MLP branch (g1 = g2 + LN2 backward, written out of place)
    g1 = g2
    if d1 != 0.0:
        g2s = K.scaled_copy(g2, dtype, d1) if d1 != 1.0 else K.cast(g2, dtype)
        hr = bw.hr
        if hr is not None:
            dh = K.linear_h3r(g2s, hr["fc2T"], bw.wfc2.shape[1], act=2, aux=s["h1"])
        else:
            dh = K.linear_dx(g2s, bw.wfc2, out_dtype=dtype, act=2, aux=s["h1"])  # d fc1 out (post-GELU')
        weight_grad(g2s, s["a1"], "mlp.fc2.weight", "mlp.fc2.bias", geo.ntok)
        if hr is not None:
            dln2 = K.linear_h3r(dh, hr["fc1T"], bw.wfc1.shape[1])
        else:
            dln2 = K.linear_dx(dh, bw.wfc1, out_dtype=torch.float32)
        weight_grad(dh, s["ln2"], "mlp.fc1.weight", "mlp.fc1.bias", geo.ntok)
        g1 = torch.empty_like(g2)
        K.layernorm_bwd(dln2, s["x1"], P["norm2.weight"], s["m2"], s["r2"], g1,
                        grads["norm2.weight"], grads["norm2.bias"], dx_in=g2)
    # ---- attention branch (g0 = g1 + LN1 backward through the window map)
    g0 = g1
    if d0 != 0.0:
        gw = K.gather_rows(g1, geo.part, geo.nrows, dtype)                        # window_partition of dL/dx1
        if d0 != 1.0:
            K.axpby(gw, gw, d0, 0.0)
        if bw.hr is not None:
            datt = K.linear_h3r(gw, bw.hr["projT"], bw.wproj.shape[1])
        else:
            datt = K.linear_dx(gw, bw.wproj, out_dtype=dtype)
        weight_grad(gw, s["att"], "attn.proj.weight", "attn.proj.bias", geo.nrows)
        labels = geo.labels if (geo.shifted and s["mask"] is None) else None
        if ATTN_BWD_PROFILE is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        dqkv = K.attn_bwd(s["qkv"], s["att"], datt, s["lse"], P["attn.relative_position_bias_table"], labels,
                          grads["attn.relative_position_bias_table"], geo.nwin, geo.N, heads, hd, geo.window0,
                          scale, mask=s["mask"] if geo.shifted else None, mask_nw=s["mask_nw"])
        if ATTN_BWD_PROFILE is not None:
            e1.record()
            # dV = P^T dO, dP = dO V^T, dQ = dS K, dK = dS^T Q (the kernels' recomputation of P not counted)
            ATTN_BWD_PROFILE.append((e0, e1, 8.0 * geo.nwin * geo.N * geo.N * hd * heads))
        dqkv_t = K.cast(dqkv, dtype)
        if bw.hr is not None:
            dln1 = K.linear_h3r(dqkv_t, bw.hr["qkvT"], bw.wqkv.shape[1])
        else:
            dln1 = K.linear_dx(dqkv_t, bw.wqkv, out_dtype=torch.float32)
        if K.dw_grouped_ok(geo.nrows, [(dqkv_t, s["ln1"])]):
            dw_jobs.append((geo.nrows, (dqkv_t, s["ln1"], grads["attn.qkv.weight"], grads["attn.qkv.bias"], 0)))
        else:
            K.linear_dw(dqkv_t, s["ln1"], grads["attn.qkv.weight"])
            K.colsum(dqkv, grads["attn.qkv.bias"])
        g0 = torch.empty_like(g1)
        K.layernorm_bwd(dln1, s["x"], P["norm1.weight"], s["m1"], s["r1"], g0,
                        grads["norm1.weight"], grads["norm1.bias"], src_map=geo.part, dx_in=g1)
    for T in sorted({t for t, _ in dw_jobs}):
        K.gemm_dw_grouped(T, [job for t, job in dw_jobs if t == T])
    return g0


# --------------------------------------------------------------------------- regularizer
PAD_CIN = 8

# Optional live profiling of the dominant kernels (bench.py): when PROFILE is a
# dict, every 160->160 conv3d_k3 forward / dgrad / wgrad launch appends
# (start_event, end_event, algorithmic flops) to PROFILE["conv_fwd" | "conv_dgrad"
# | "conv_wgrad"], events recorded on the launching stream (torch's current
# stream, which every dlcs launch uses); ATTN_PROFILE likewise (a list) for the
# fused window attention forward (algorithmic flops of Q K^T and P V).
PROFILE = None
ATTN_PROFILE = None
ATTN_BWD_PROFILE = None         # the same for the attention backward (dK / dV / table + dQ kernels)
# Test hook: when a list, every swinnet_forward appends its post-ReLU activations
# (the ReLU decisions the backward uses) and grid (tests/test_gpu_swin.py).
CAPTURE = None
# Diagnostic hook (tools/dgrad_diag.py): when a list, the split path's 160 -> 160 input
# gradients append (fp32 input gradient, ReLU mask, torch weight, output).
DGRAD_CAPTURE = None


def _timed(role, flops, fn, *args, **kw):
    if PROFILE is None:
        return fn(*args, **kw)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    out = fn(*args, **kw)
    e1.record()
    PROFILE.setdefault(role, []).append((e0, e1, flops))
    return out


def _conv_flops(grid, cin, cout):
    return 2.0 * grid[0] * grid[1] * grid[2] * grid[3] * cout * cin * 27


def _timed_conv(*args, **kw):
    return _timed("conv_fwd", _conv_flops(args[5], args[1], args[3]), K.conv3d, *args, **kw)


# The DLCS_* switches below select superseded kernels for A/B runs; they are read
# only under DLCS_DIAG=1 (dl_cs/diag.py), otherwise the defaults hold.
#
# fp32 Conv3d 160 -> 160 on fp16 matrix cores at fp32 accuracy
# (tests/test_gpu_kernels.py::test_conv3d_f16x3): "f16x3" (default) = fp16 2-plane
# split with a power-of-two scale per tensor, three plane products
# (dlcs_conv3d_k3_f16x3 / _wgrad_f16x3, with the K = 160 patch GEMMs and the thin
# ends on the same split); "f32" = the f32-MFMA kernels (v_mfma_f32_16x16x4_f32).
FP32_CONV = _diag.knob("DLCS_FP32_CONV", "f32" if _diag.knob("DLCS_CONV_X6", "") == "0" else "f16x3")
if FP32_CONV not in ("f16x3", "f32"):
    raise ValueError(f"DLCS_FP32_CONV={FP32_CONV!r}: 'f16x3' (default) or 'f32'")
X6 = FP32_CONV != "f32"          # the split-plane kernels are in use (bench.py reads this)
# The Swin block's fp32 Linears on the row-scaled f16x3 split (dlcs_gemm_h3r;
# tests/test_gpu_kernels.py::test_gemm_h3r); DLCS_H3R=0 keeps them on f32 MFMAs.
H3R = _diag.knob("DLCS_H3R", "1") != "0"
# The fp32 patch-embed forward (13440 x 10240 -> 160) and the unembed input gradient
# (13440 x 10240 -> 160) on the row-scaled f16 split (dlcs_gemm_h3r, K = 10240 in eight
# XCD-group K ranges summed in a fixed order) by default; DLCS_EMBED_X6 = f: the
# forward on the bf16 3-plane NT GEMM (dlcs_gemm_nt_x6), b: the input gradient, 1: both.
_EX6 = _diag.knob("DLCS_EMBED_X6", "0")
EMBED_X6 = _EX6 in ("1", "f")          # the patch-embed forward on dlcs_gemm_nt_x6
UNEMBED_X6 = _EX6 in ("1", "b")        # the unembed input gradient on dlcs_gemm_nt_x6


# DLCS_THIN_F32=1 keeps the thin ends (SFE 2E -> C, final C -> 2E: forward, input
# and weight gradients) on the f32 kernels while the 160-channel convs take the split.
THIN_F32 = _diag.knob("DLCS_THIN_F32", "0") == "1"
# DLCS_K160_F32=1 (diagnostic): the k4s4 GEMMs with K = 160 (unembed forward, embed
# input gradient) on the f32 GEMM while the convs take the split.
K160_F32 = _diag.knob("DLCS_K160_F32", "0") == "1"
# The thin ends' 160-channel operand (relu(h) of the final conv, g_s of the SFE conv)
# split once into planes that the forward / input-gradient and the weight-gradient
# kernels DMA (conv3d_thin_planes.inc); DLCS_THIN_PLANES=0: the in-register split kernels.
THIN_PLANES = _diag.knob("DLCS_THIN_PLANES", "1") != "0"
# DLCS_FWD_PLANES_ONLY=0 (diagnostic): the forward keeps the fp32 a_k / relu(out) / relu(h)
# beside their planes and the input gradients read those as masks
FWD_PLANES_ONLY = _diag.knob("DLCS_FWD_PLANES_ONLY", "1") != "0"


_CONV_NORMS = []        # [(weakref to the weight, version, layout, ||W||_inf word)], most recent first


def clear_norm_cache():
    """Forget the cached weight norms (swin3D.clear_weight_cache: a parameter changed
    through .data keeps its version counter, so the cache cannot see the change)."""
    del _CONV_NORMS[:]


def _conv_norm(w, C, dgrad=False):
    """||W||_inf of a 160 -> 160 conv weight [co][ci][3][3][3] for planes_bound -- the max
    over co of sum |W[co]| (forward), or over ci of sum |W[:, ci]| (input gradient) --
    cached by the parameter tensor, its in-place version counter and the layout: the
    NetWeights of every unroll of a training step share one launch per weight."""
    for t, ver, dg, nrm in _CONV_NORMS:
        if t() is w and ver == w._version and dg == dgrad:
            return nrm
    if dgrad == "patch":
        # k4s4 patch weight [a][b][4][4][4] -> max over (b, k) of sum_a |W[a][b][k]|: the rows
        # (kd, kh, kw, b) of the unembed B operand (a = ci) and of the transposed embed
        # operand (a = co), read in the parameter's own layout
        nrm = K.abs_row_sum_max(w, C * 64, 1, 1, n_outer=w.shape[0], outer_stride=C * 64)
    elif dgrad:
        nrm = K.abs_row_sum_max(w, C, 27, 27, n_outer=w.shape[0], outer_stride=27 * C)
    else:
        nrm = K.abs_row_sum_max(w, C, 27 * C, 27 * C)
    _CONV_NORMS.insert(0, (weakref.ref(w), w._version, dgrad, nrm))
    del _CONV_NORMS[12:]
    return nrm


def _use_split(dtype, C):
    return X6 and dtype == torch.float32 and C == 160


class StageWeights:
    """Compute-dtype copies / packings of one ResSwinTransformer3DBlock (s3d:327-340):
    its SwinTransformer3D (patch embed, blocks, patch unembed) and its ConvBlock
    tail.  Engine parameter names carry the stage prefix `pre` ("rs<k>.")."""

    def __init__(self, params, pre, dtype, depth, split):
        self.pre = pre
        P = lambda n: params[pre + n]                 # noqa: E731
        tail = P("swin_tail.weight")
        self.tail = K.conv_pack_f16x3(tail, 0) if split else K.conv_pack(tail, dtype, 0)
        we = P("patch_embed.proj.weight")             # [co, ci, 4, 4, 4]
        C = we.shape[0]
        # embed B operand [co][(kd,kh,kw,ci)]
        self.emb = K.permute(we, (C, 4, 4, 4, C), (C * 64, 16, 4, 1, 64), dst_dtype=dtype)
        wu = P("patch_unembed.proj.weight")           # [ci, co, 4, 4, 4]
        # unembed B operand [(kd,kh,kw,co)][ci]
        self.unemb = K.permute(wu, (4, 4, 4, C, C), (16, 4, 1, 64, C * 64), dst_dtype=dtype)
        self.unemb_bias = K.fill_bias(K.empty((64 * C,), torch.float32, we.device), P("patch_unembed.proj.bias"),
                                      1, 64 * C, C)
        # fp32 unembed input gradient: on the row-scaled f16 split (dlcs_gemm_h3r, K = 64 C in
        # 160-wide segments; B = unemb^T packed) by default, or the x6 NT GEMM (DLCS_EMBED_X6=1|b):
        # the latter is as accurate per launch (tools/split_diag.py) but left the Swin blocks'
        # gradients at 1.3e-5 of float64 where h3r / f32 give <= 0.9e-5 (tools/grad_attrib.py)
        self.unembT = self.unemb.reshape(64 * C, C).t().contiguous() if split and UNEMBED_X6 else None
        # the patch-embed forward's B = emb [C][64 C] on the same split, packed in the same launch
        jobs = []
        if split and H3R and not UNEMBED_X6:
            jobs.append((self.unemb.reshape(64 * C, C), True))
        if split and H3R and not EMBED_X6:
            jobs.append((self.emb.reshape(C, 64 * C), False))
        packs = K.h3r_pack(jobs) if jobs else []
        self.unemb_dx = packs.pop(0) if split and H3R and not UNEMBED_X6 else None
        self.emb_h3r = packs.pop(0) if split and H3R and not EMBED_X6 else None
        if split:
            # the k4s4 GEMMs with K = 160 (unembed forward, embed input gradient) on fp16
            # matrix cores: B operands as [N = 10240][K = 160] plane pairs
            self.unemb_h3 = K.split2(self.unemb.reshape(64 * C, C))
            self.embT_h3 = K.split2(self.emb.reshape(C, 64 * C).t().contiguous())
            self.embT_norm = _conv_norm(we, C, dgrad="patch")
            # ||W||_inf of the producers that write their output's planes (planes_bound)
            self.unemb_norm = _conv_norm(wu, C, dgrad="patch")
            self.tail_norm = _conv_norm(tail, C)
        bp = [{n: P(f"blocks.{i}.{n}") for n in BlockWeights.NAMES} for i in range(depth)]
        casts = [None] * depth
        hrs = [None] * depth
        if depth and h3r_ok(dtype, *[bp[0][n] for n in BlockWeights.LINEARS]):
            flat = K.h3r_pack([(b[n], t) for b in bp for t in (False, True) for n in BlockWeights.LINEARS])
            hrs = [flat[8 * i:8 * i + 8] for i in range(depth)]
        if dtype == torch.bfloat16:
            flat = K.cast_multi_bf16([b[n] for b in bp for n in BlockWeights.LINEARS])
            casts = [flat[4 * i:4 * i + 4] for i in range(depth)]
        self.blocks = [BlockWeights(bp[i], dtype, casts[i], hrs[i]) for i in range(depth)]


class NetWeights:
    """Per-call compute-dtype copies / packings of one SwinTransformer3DNet's
    parameters: the SFE / DFE-tail / final convs and one StageWeights per
    ResSwin block (NUM_SWINBLOCKS, s3d:347-357)."""

    def __init__(self, params, dtype, depth, nstages=1):
        self.p = params
        self.dtype = dtype
        C = params["SFE.layers.2.conv.bias"].shape[0]
        self.split = _use_split(dtype, C)
        self.x6 = self.h3_patch = self.split            # older names (tools)
        self.sfe = K.conv_pack(params["SFE.layers.2.conv.weight"], dtype, 0)
        self.fin = K.conv_pack(params["final_layer.layers.2.conv.weight"], dtype, 0)
        dfe = params["dfe_tail.weight"]
        self.dfe = K.conv_pack_f16x3(dfe, 0) if self.split else K.conv_pack(dfe, dtype, 0)
        self.dfe_norm = _conv_norm(dfe, C) if self.split else None
        self.thin_h3 = self.split and not THIN_F32
        if self.thin_h3:
            # the thin ends (SFE 2E -> C, final C -> 2E) on the f16x3 split too
            cin = params["SFE.layers.2.conv.weight"].shape[1]
            self.sfe_h3 = K.thin_pack_f16x3(self.sfe, C, cin, 0)
            self.fin_h3 = K.thin_pack_f16x3(self.fin, cin, C, 1)
        self.stages = [StageWeights(params, f"rs{k}.", dtype, depth, self.split) for k in range(nstages)]


def _stage_swin_forward(W, st, inp, geos, ntok, heads, drops):
    """SwinTransformer3D (vst:735-756) of one stage on the patch grid: patch embed
    of the stage input (patch-blocked rows, vst:455), the blocks; -> the final
    tokens in the compute dtype and the blocks' saved state."""
    dtype, P = W.dtype, W.p
    C = st.emb.shape[0]
    # No split-K with float atomics in the forward: a 1-ulp change of a pre-activation
    # near 0 flips a downstream ReLU mask (3e-4 on some gradients, tests/test_gpu_dist.py)
    # -- the forward stays run-to-run deterministic (the split-K paths sum their K
    # ranges in a fixed order).
    if dtype == torch.float32 and st.emb_h3r is not None:
        tok = K.linear_h3r(inp.view(ntok, 64 * C), st.emb_h3r, C, bias=P[st.pre + "patch_embed.proj.bias"])
    else:
        tok = K.fill_bias(K.empty((ntok, C), torch.float32, inp.device), P[st.pre + "patch_embed.proj.bias"],
                          ntok, C, C)
        if dtype == torch.float32 and W.split and EMBED_X6:
            # fp32 on bf16 matrix cores, 3-plane split; split-K over partial slabs summed in a fixed order
            K.gemm_nt_x6(inp, st.emb, tok, ntok, C, 64 * C, 64 * C, 64 * C)
        elif dtype == torch.float32:
            K.gemm_f32_splitk_det(inp, st.emb, tok, ntok, C, 64 * C, 64 * C, 64 * C)
        else:
            K.gemm(inp, st.emb, tok, ntok, C, 64 * C, 64 * C, 64 * C, C, accumulate=1, splitk=1)
    bsaved = []
    for i, bw in enumerate(st.blocks):
        ds = drops[i] if drops is not None else (1.0, 1.0)
        tok, sv = block_forward(bw, geos[i], tok, dtype, heads, drop_scale=ds)
        bsaved.append(sv)
    return K.cast(tok, dtype), bsaved


def swinnet_forward(W, x, heads=8, window=(7, 8, 8), pad=4, drop_scales=None):
    """SwinTransformer3DNet.forward (s3d:420-435) with len(W.stages) ResSwin blocks.
    x complex64 [B, E, T, Y, X] -> (out complex64, saved dict).

        s = SFE(u);  in_0 = s
        out_k = conv_k(relu(Swin_k(in_k))) + in_k,  in_{k+1} = out_k   (s3d:339-340)
        h = conv_d(relu(out_last)) + 2 s                                 (s3d:368, :425-427)
        o = final(relu(h))                                               (s3d:391)
    """
    dtype = W.dtype
    P = W.p
    B, E, T, Y, X = x.shape
    Tp = T + 2 * pad
    if Tp % 4 or Y % 4 or X % 4:
        raise NotImplementedError("dl_cs HIP path: T+2*pad, Y and X must be multiples of 4")
    grid = (B, Tp, Y, X)
    C = P["SFE.layers.2.conv.bias"].shape[0]
    cin = 2 * E
    dev = x.device
    rows = B * Tp * Y * X
    flops = _conv_flops(grid, C, C)
    u = K.swin_pre(x.contiguous(), dtype, pad, PAD_CIN)                              # s3d:394-406
    # max |.| words of the forward's 160-channel tensors (s, a_k, out_k), inputs of the
    # planes bounds of the producers that split their own output
    mx = K.zeros((2 * len(W.stages) + 2,), torch.int32, dev) if W.split else None
    word = (lambda i: ctypes.c_void_p(mx.data_ptr() + 4 * i)) if W.split else None
    if W.thin_h3:                                                                    # s3d:384 (SFE)
        umax = K.absmax(u)
        s = K.conv3d_thin_f16x3(u, cin, umax, W.sfe_h3, C, C, grid, bias=P["SFE.layers.2.conv.bias"],
                                out_max=word(0) if W.split else None)
    else:
        umax = None
        s = K.conv3d(u, cin, W.sfe, C, C, grid, bias=P["SFE.layers.2.conv.bias"])
        if W.split:
            K.absmax(s, out=mx[0:1])
    nT, nY, nX = Tp // 4, Y // 4, X // 4
    ntok = B * nT * nY * nX
    depth = len(W.stages[0].blocks)
    geos = [SwinGeometry(B, nT, nY, nX, window, i % 2 == 1, dev) for i in range(depth)]
    nst = len(W.stages)
    stages = []
    inp, pout = s, None
    inp_max = word(0) if W.split else None
    # a_k, relu(out_last) and relu(h) are read later only through their ReLU signs (the
    # input gradients' masks) and their planes: written as planes only (the masks read
    # from the planes), unless a diagnostic captures the fp32 tensors
    fwd_po = (W.split and not K160_F32 and W.thin_h3 and THIN_PLANES and CAPTURE is None and
              DGRAD_CAPTURE is None and FWD_PLANES_ONLY)
    for k, st in enumerate(W.stages):
        last = k == nst - 1
        tok_t, bsaved = _stage_swin_forward(W, st, inp, geos, ntok, heads,
                                            drop_scales[k] if drop_scales is not None else None)
        # the unembed output a_k is only ever consumed through the tail ConvBlock's
        # ReLU (s3d:256-259) and, in backward, through its sign: stored post-ReLU
        # straight from the producing epilogue (vst:517, k4s4 convT)
        a = None if fwd_po else K.empty((rows, C), dtype, dev)
        ss = dict(inp=inp, tok_t=tok_t, bsaved=bsaved, a=a)
        tb = P[st.pre + "swin_tail.bias"]
        if W.split:
            # the producers write their output's planes from the epilogue (no split pass over
            # the fp32 tensor), scaled by a bound of max|out| set before they run (planes_bound:
            # |relu(W x + b + r)| <= ||W||_inf max|x| + max|b| + max|r|)
            pa = K.planes_alloc(rows, dev)
            amax, omax = word(1 + 2 * k), word(2 + 2 * k)
            if K160_F32:
                K.gemm(tok_t, st.unemb, a, ntok, 64 * C, C, C, C, 64 * C, bias=st.unemb_bias, act=3)
                K.split2(a, out=pa)
                K.absmax(a, out=mx[1 + 2 * k:2 + 2 * k])
            else:
                tp = K.split2(tok_t)
                K.planes_bound(pa, rows, m0=K.planes_max(tp, ntok), n0=st.unemb_norm, vec=st.unemb_bias)
                K.gemm_k160_f16x3(tp, ntok, st.unemb_h3, 64 * C, a.view(ntok, 64 * C) if a is not None else None,
                                  bias=st.unemb_bias, act=3, out_max=amax, out_planes=pa)
            # the input planes are kept for the weight gradient (0.8 GB per stage at BASELINE size)
            ss["planes"] = pa
            if last:
                # out_last feeds only the DFE tail's ReLU: stored post-ReLU, with its planes
                pb = K.planes_alloc(rows, dev)
                K.planes_bound(pb, rows, m0=amax, n0=st.tail_norm, m1=inp_max, vec=tb)
                out = _timed("conv_fwd", flops, K.conv3d_f16x3, ss["planes"], st.tail, grid, bias=tb, res=inp,
                             relu_out=1, out_max=omax, out_planes=pb, planes_only=fwd_po)
                pout = pb
            else:
                # an inner stage's output is the next stage's input and residual: raw
                out = _timed("conv_fwd", flops, K.conv3d_f16x3, ss["planes"], st.tail, grid, bias=tb, res=inp,
                             out_max=omax)
            inp_max = omax
        else:
            K.gemm(tok_t, st.unemb, a, ntok, 64 * C, C, C, C, 64 * C, bias=st.unemb_bias, act=3)
            out = _timed_conv(a, C, st.tail, C, C, grid, bias=tb, res=inp, relu_out=int(last))
        ss["out"] = out
        stages.append(ss)
        inp = out
    b = inp                                                                          # relu(out_last)
    ph = None
    if W.split:                                                                      # s3d:356, :391
        hmax = mx[-1:]
        if W.thin_h3 and THIN_PLANES:
            # relu(h) written with its planes: the final conv's forward and weight gradient DMA them
            ph = K.planes_alloc(rows, dev)
            K.planes_bound(ph, rows, m0=inp_max, n0=W.dfe_norm, m1=word(0), c1=2.0, vec=P["dfe_tail.bias"])
        h = _timed("conv_fwd", flops, K.conv3d_f16x3, pout, W.dfe, grid, bias=P["dfe_tail.bias"], res=s,
                   res_scale=2.0, relu_out=1, out_max=K.p(hmax), out_planes=ph, planes_only=fwd_po)
        if ph is not None:
            o = K.conv3d_thin_out_planes(ph, W.fin_h3, cin, PAD_CIN, grid, bias=P["final_layer.layers.2.conv.bias"])
        elif W.thin_h3:
            o = K.conv3d_thin_f16x3(h, C, hmax, W.fin_h3, cin, PAD_CIN, grid,
                                    bias=P["final_layer.layers.2.conv.bias"])
        else:
            o = K.conv3d(h, C, W.fin, cin, PAD_CIN, grid, bias=P["final_layer.layers.2.conv.bias"],
                         out_dtype=torch.float32)
    else:
        hmax = None
        h = _timed_conv(b, C, W.dfe, C, C, grid, bias=P["dfe_tail.bias"], res=s, res_scale=2.0, relu_out=1)
        o = K.conv3d(h, C, W.fin, cin, PAD_CIN, grid, bias=P["final_layer.layers.2.conv.bias"],
                     out_dtype=torch.float32)
    out = K.swin_post(o, (B, E, T, Y, X), pad)                                       # s3d:408-418
    saved = dict(u=u, s=s, b=b, pout=pout, h=h, ph=ph, stages=stages, geos=geos, shape=(B, E, T, Y, X), grid=grid,
                 pad=pad, heads=heads, cin=cin, C=C, ntok=ntok, umax=umax, hmax=hmax)
    if CAPTURE is not None:
        # the oracle's ReLU call order: each stage's tail ConvBlock, the DFE tail, the final conv
        CAPTURE.append(dict(relu_inputs=[ss["a"] for ss in stages] + [b, h], grid=grid, C=C))
    return out, saved


def swinnet_backward(W, sv, gout, grads):
    """Backward of swinnet_forward.  gout complex64 [B,E,T,Y,X]; accumulates into
    grads[name] (fp32, torch layouts; patch GEMM weights into grads["rs<k>.emb_packed"
    / "rs<k>.unemb_packed"]) and returns dL/dx complex64."""
    dtype = W.dtype
    P = W.p
    grid, pad, C, cin, ntok = sv["grid"], sv["pad"], sv["C"], sv["cin"], sv["ntok"]
    dev = gout.device
    rows = grid[0] * grid[1] * grid[2] * grid[3]
    flops = _conv_flops(grid, C, C)
    go = K.swin_post_bwd(gout.contiguous(), dtype, pad, PAD_CIN)
    # the DFE input gradient g_out as planes only (no fp32 tensor, no split pass); the
    # diagnostics that capture the fp32 gradients keep the fp32 path
    gout_planes = W.split and not K160_F32 and DGRAD_CAPTURE is None

    def conv_grads(x_in, cin_, g, cout, wname, bname):
        dwp = torch.zeros((27, K.pad32(cout), K.pad32(cin_)), dtype=torch.float32, device=dev)
        # the bias gradient (column sums of g) comes with the weight gradient: the 160-channel
        # and SFE kernels sum the g tiles they already hold, other shapes add a column-sum launch
        if cin_ == C and cout == C:
            _timed("conv_wgrad", flops, K.conv3d_wgrad, x_in, cin_, 0, g, cout, grid, dwp, dbias=grads[bname])
        else:
            K.conv3d_wgrad(x_in, cin_, 0, g, cout, grid, dwp, dbias=grads[bname])
        K.conv_unpack_grad(dwp, grads[wname], cout, cin_)

    def split_wgrad(x_planes, g_planes, wname):
        # the bias gradient came with the split of g (colsum)
        dwp = torch.zeros((27, C, C), dtype=torch.float32, device=dev)
        _timed("conv_wgrad", flops, K.conv3d_wgrad_f16x3, x_planes, g_planes, grid, dwp)
        K.conv_unpack_grad(dwp, grads[wname], C, C)

    # final conv (s3d:391):  o = conv(relu(h))
    wf = K.conv_pack(P["final_layer.layers.2.conv.weight"], dtype, 1)
    if W.split:
        pg = K.planes_alloc(rows, dev)
        if W.thin_h3:
            # thin ends on the f16x3 split: g_h's max goes straight into its split trailer
            gomax = K.absmax(go)
            if gout_planes:
                # g_h written as planes only (the DFE dgrad and weight gradient DMA them, the embed
                # gradient reads its residual from them) with the DFE bias gradient's column sums;
                # scale from |g_h| <= ||W_fin^T||_inf max|go|
                ghm = K.zeros((1,), torch.int32, dev)
                K.planes_bound(pg, rows, m0=gomax, n0=_conv_norm(P["final_layer.layers.2.conv.weight"], C, dgrad=True))
                K.conv3d_thin_f16x3(go, cin, gomax, K.thin_pack_f16x3(wf, C, cin, 0), C, C, grid, mask=sv["h"],
                                    mask_planes=sv["ph"] if sv["h"] is None else None, out_max=K.p(ghm),
                                    out_planes=pg, planes_only=True, colsum=grads["dfe_tail.bias"])
                g_h = None
            else:
                g_h = K.conv3d_thin_f16x3(go, cin, gomax, K.thin_pack_f16x3(wf, C, cin, 0), C, C, grid, mask=sv["h"],
                                          out_max=K.planes_max(pg, rows))
            dwp = torch.zeros((27, K.pad32(cin), C), dtype=torch.float32, device=dev)
            if sv["ph"] is not None:
                K.conv3d_thin_wgrad_planes(sv["ph"], go, cin, gomax, 0, grid, dwp)
            else:
                K.conv3d_thin_wgrad_f16x3(sv["h"], C, sv["hmax"], go, cin, gomax, grid, dwp)
            K.conv_unpack_grad(dwp, grads["final_layer.layers.2.conv.weight"], cin, C)
            K.colsum(go, grads["final_layer.layers.2.conv.bias"], rows=rows, C=cin, ld=go.shape[-1])
        else:
            g_h = K.conv3d(go, cin, wf, C, C, grid, relu_in=0, mask=sv["h"])
            conv_grads(sv["h"], C, go, cin, "final_layer.layers.2.conv.weight", "final_layer.layers.2.conv.bias")
        # DFE tail (s3d:356):  h = conv_d(relu(out_last)) + 2 s
        if g_h is None:                            # planes and bias gradient already written
            gp = gh_pl = pg
            ghmax = ghm
        else:
            gh_pl = None
            gp = K.split2(g_h, out=pg, have_max=W.thin_h3, colsum=grads["dfe_tail.bias"])
            ghmax = gp[rows * 640:rows * 640 + 4].view(torch.int32).clone()   # max|g_h| (bounds below)
        pg = K.planes_alloc(rows, dev)
        if gout_planes:
            # g_out written as planes only (the stage tail's dgrad and weight gradient DMA them,
            # the embed gradient reads its residual from them) with its column sums (the stage
            # tail's bias gradient); scale from |g_out| <= ||W_dfe^T||_inf max|g_h|
            gom = K.zeros((1,), torch.int32, dev)
            K.planes_bound(pg, rows, m0=ghmax, n0=_conv_norm(P["dfe_tail.weight"], C, dgrad=True))
            _timed("conv_dgrad", flops, K.conv3d_f16x3, gp, K.conv_pack_f16x3(P["dfe_tail.weight"], 1), grid,
                   mask=sv["b"], mask_planes=sv["pout"] if sv["b"] is None else None, out_max=K.p(gom),
                   out_planes=pg, planes_only=True,
                   colsum=grads[W.stages[-1].pre + "swin_tail.bias"])
            g_out = None
        else:
            g_out = _timed("conv_dgrad", flops, K.conv3d_f16x3, gp, K.conv_pack_f16x3(P["dfe_tail.weight"], 1), grid,
                           mask=sv["b"], out_max=K.planes_max(pg, rows))
        split_wgrad(sv["pout"], gp, "dfe_tail.weight")
        del gp
        if DGRAD_CAPTURE is not None:
            DGRAD_CAPTURE.append(("dfe_tail", g_h, sv["b"], P["dfe_tail.weight"], g_out))
    else:
        g_h = K.conv3d(go, cin, wf, C, C, grid, relu_in=0, mask=sv["h"])
        conv_grads(sv["h"], C, go, cin, "final_layer.layers.2.conv.weight", "final_layer.layers.2.conv.bias")
        w2 = K.conv_pack(P["dfe_tail.weight"], dtype, 1)
        g_out = _timed("conv_dgrad", flops, K.conv3d, g_h, C, w2, C, C, grid, mask=sv["b"])
        conv_grads(sv["b"], C, g_h, C, "dfe_tail.weight", "dfe_tail.bias")
    gsmax = None
    pgs = None                                     # planes of g_s (thin-end planes path)
    gout_pl = None                                 # g_out as planes only (the DFE input gradient's)
    for k in reversed(range(len(W.stages))):
        st, ss = W.stages[k], sv["stages"][k]
        pre = st.pre
        # tail ConvBlock (s3d:336):  out_k = conv_k(relu(a_k)) + in_k
        if W.split:
            if g_out is None:                      # planes and bias gradient already written
                gp = gout_pl = pg
                gomax = gom
            else:
                gout_pl = None
                gp = K.split2(g_out, out=pg, have_max=True, colsum=grads[pre + "swin_tail.bias"])
                gomax = gp[rows * 640:rows * 640 + 4].view(torch.int32).clone()
            g_a = _timed("conv_dgrad", flops, K.conv3d_f16x3, gp, K.conv_pack_f16x3(P[pre + "swin_tail.weight"], 1),
                         grid, mask=ss["a"], mask_planes=ss["planes"] if ss["a"] is None else None)
            split_wgrad(ss["planes"], gp, pre + "swin_tail.weight")
            del gp
            if DGRAD_CAPTURE is not None:
                DGRAD_CAPTURE.append((pre + "swin_tail", g_out, ss["a"], P[pre + "swin_tail.weight"], g_a))
        else:
            w1 = K.conv_pack(P[pre + "swin_tail.weight"], dtype, 1)
            g_a = _timed("conv_dgrad", flops, K.conv3d, g_out, C, w1, C, C, grid, mask=ss["a"])
            conv_grads(ss["a"], C, g_out, C, pre + "swin_tail.weight", pre + "swin_tail.bias")
        # ---- Swin backward: unembed (K = 64 C)
        # h3r writes d_tok; the other two accumulate into it
        d_tok = (K.empty if st.unemb_dx is not None else K.zeros)((ntok, C), torch.float32, dev)
        if st.unemb_dx is not None:
            K.linear_h3r(g_a.view(ntok, 64 * C), st.unemb_dx, C, out=d_tok)
        elif st.unembT is not None:
            # fp32 on bf16 matrix cores (3-plane split), fixed-order split-K: run-to-run deterministic
            K.gemm_nt_x6(g_a, st.unembT, d_tok, ntok, C, 64 * C, 64 * C, 64 * C)
        else:
            K.gemm(g_a, st.unemb, d_tok, ntok, C, 64 * C, 64 * C, C, C, b_trans=1, accumulate=1, splitk=16)
        if DGRAD_CAPTURE is not None:
            DGRAD_CAPTURE.append((pre + "unembed_dx", g_a, None, st.unemb, d_tok))
        g_a_tok = g_a.view(ntok, 64 * C)                   # patch-blocked rows: one token = 64 consecutive rows
        if K.dw_grouped_ok(ntok, [(g_a_tok, ss["tok_t"])]):
            K.gemm_dw_grouped(ntok, [(g_a_tok, ss["tok_t"], grads[pre + "unemb_packed"],
                                      grads[pre + "patch_unembed.proj.bias"], C)])
        else:
            K.gemm(g_a, ss["tok_t"], grads[pre + "unemb_packed"], 64 * C, C, ntok, 64 * C, C, C, a_trans=1,
                   b_trans=1, accumulate=1, splitk=max(1, min(16, ntok // 256)))
            K.colsum(g_a, grads[pre + "patch_unembed.proj.bias"], rows=rows, C=C, ld=C)
        del g_a, g_a_tok
        for i in reversed(range(len(st.blocks))):
            bg = {n: grads[f"{pre}blocks.{i}.{n}"] for n in BlockWeights.NAMES}
            d_tok = block_backward(st.blocks[i], sv["geos"][i], ss["bsaved"][i], d_tok, bg, dtype, sv["heads"])
        # embed (k4s4 conv) backward: dL/d in_k = (embed backward) + g_out_k (the ResSwin
        # residual); in_0 = s also feeds the DFE residual twice (h = conv_d(.) + 2 s): + 2 g_h.
        # Summed in the GEMM epilogue in fp32 and rounded once to the compute dtype.
        d_tok_t = K.cast(d_tok, dtype)
        first = k == 0
        # (the split path's first stage writes g_s as planes only, below)
        planes_only = W.split and not K160_F32 and first and W.thin_h3 and THIN_PLANES
        g_in = None if planes_only else K.empty((rows, C), dtype, dev)
        if W.split and K160_F32:
            pg = K.planes_alloc(rows, dev)
            if first:
                K.gemm(d_tok_t, st.emb, g_in, ntok, 64 * C, C, C, 64 * C, 64 * C, b_trans=1,
                       res=g_h, ldr=64 * C, res_scale=2.0, res2=g_out, ldr2=64 * C)
                gsmax = K.absmax(g_in)
            else:
                K.gemm(d_tok_t, st.emb, g_in, ntok, 64 * C, C, C, 64 * C, 64 * C, b_trans=1, res=g_out, ldr=64 * C)
                K.absmax(g_in, out=pg[rows * 640:rows * 640 + 4].view(torch.int32))
        elif W.split:
            if first:
                dtp = K.split2(d_tok_t)
                if planes_only:
                    # g_s is only read through its planes (the SFE conv's input and weight
                    # gradients): the GEMM writes them and the SFE bias gradient (column sums),
                    # no fp32 g_s; scale from |g_s| <= max|d_tok| ||emb^T||_inf + 2 max|g_h| + max|g_out|
                    pgs = K.planes_alloc(rows, dev)
                    gsmax = None
                    K.planes_bound(pgs, rows, m0=K.planes_max(dtp, ntok), n0=st.embT_norm, m1=ghmax, c1=2.0,
                                   vec=gomax.view(torch.float32))
                    K.gemm_k160_f16x3(dtp, ntok, st.embT_h3, 64 * C, None,
                                      res=g_h.view(ntok, 64 * C) if g_h is not None else None, res_planes=gh_pl,
                                      res_scale=2.0, res2=g_out.view(ntok, 64 * C) if g_out is not None else None,
                                      res2_planes=gout_pl, out_planes=pgs, colsum=grads["SFE.layers.2.conv.bias"])
                else:
                    gsmax = K.zeros((1,), torch.int32, dev)
                    K.gemm_k160_f16x3(dtp, ntok, st.embT_h3, 64 * C, g_in.view(ntok, 64 * C),
                                      res=g_h.view(ntok, 64 * C) if g_h is not None else None, res_planes=gh_pl,
                                      res_scale=2.0, res2=g_out.view(ntok, 64 * C) if g_out is not None else None,
                                      res2_planes=gout_pl, out_max=K.p(gsmax))
            else:
                pg = K.planes_alloc(rows, dev)
                K.gemm_k160_f16x3(K.split2(d_tok_t), ntok, st.embT_h3, 64 * C, g_in.view(ntok, 64 * C),
                                  res=g_out.view(ntok, 64 * C) if g_out is not None else None, res_planes=gout_pl,
                                  out_max=K.planes_max(pg, rows))
        elif first:
            K.gemm(d_tok_t, st.emb, g_in, ntok, 64 * C, C, C, 64 * C, 64 * C, b_trans=1,
                   res=g_h, ldr=64 * C, res_scale=2.0, res2=g_out, ldr2=64 * C)
        else:
            K.gemm(d_tok_t, st.emb, g_in, ntok, 64 * C, C, C, 64 * C, 64 * C, b_trans=1, res=g_out, ldr=64 * C)
        in_tok = ss["inp"].view(ntok, 64 * C)
        if K.dw_grouped_ok(ntok, [(d_tok_t, in_tok)]):
            K.gemm_dw_grouped(ntok, [(d_tok_t, in_tok, grads[pre + "emb_packed"], grads[pre + "patch_embed.proj.bias"],
                                      0)])
        else:
            K.gemm(d_tok_t, ss["inp"], grads[pre + "emb_packed"], C, 64 * C, ntok, C, 64 * C, 64 * C, a_trans=1,
                   b_trans=1, accumulate=1, splitk=max(1, min(16, ntok // 256)))
            K.colsum(d_tok, grads[pre + "patch_embed.proj.bias"])
        g_out = g_in
    g_s_t = g_out
    # ---- SFE (s3d:384), no activation
    wsfe = K.conv_pack(P["SFE.layers.2.conv.weight"], dtype, 1)
    if pgs is not None:
        # g_s as planes (its column sums = the SFE bias gradient): the SFE input gradient and
        # weight gradient DMA them
        if g_s_t is not None:
            K.split2(g_s_t, out=pgs, have_max=True, colsum=grads["SFE.layers.2.conv.bias"])
        g_u = K.conv3d_thin_out_planes(pgs, K.thin_pack_f16x3(wsfe, cin, C, 1), cin, PAD_CIN, grid)
        dwp = torch.zeros((27, C, K.pad32(cin)), dtype=torch.float32, device=dev)
        K.conv3d_thin_wgrad_planes(pgs, sv["u"], cin, sv["umax"], 1, grid, dwp)
        K.conv_unpack_grad(dwp, grads["SFE.layers.2.conv.weight"], C, cin)
    elif W.thin_h3:
        g_u = K.conv3d_thin_f16x3(g_s_t, C, gsmax, K.thin_pack_f16x3(wsfe, cin, C, 1), cin, PAD_CIN, grid)
        dwp = torch.zeros((27, C, K.pad32(cin)), dtype=torch.float32, device=dev)
        K.conv3d_thin_wgrad_f16x3(sv["u"], cin, sv["umax"], g_s_t, C, gsmax, grid, dwp,
                                  colsum=grads["SFE.layers.2.conv.bias"])
        K.conv_unpack_grad(dwp, grads["SFE.layers.2.conv.weight"], C, cin)
    else:
        g_u = K.conv3d(g_s_t, C, wsfe, cin, PAD_CIN, grid)
        conv_grads(sv["u"], cin, g_s_t, C, "SFE.layers.2.conv.weight", "SFE.layers.2.conv.bias")
    return K.swin_pre_bwd(g_u, sv["shape"], pad)


def unpack_patch_grads(grads, C, nstages=1):
    """rs<k>.emb_packed [co][(kd,kh,kw,ci)] -> [co][ci][kd][kh][kw];
    rs<k>.unemb_packed [(kd,kh,kw,co)][ci] -> [ci][co][kd][kh][kw]."""
    for k in range(nstages):
        pre = f"rs{k}."
        K.permute(grads[pre + "emb_packed"], (C, C, 4, 4, 4), (64 * C, 1, 16 * C, 4 * C, C),
                  out=grads[pre + "patch_embed.proj.weight"], accumulate=1)
        K.permute(grads[pre + "unemb_packed"], (C, C, 4, 4, 4), (1, C, 16 * C * C, 4 * C * C, C * C),
                  out=grads[pre + "patch_unembed.proj.weight"], accumulate=1)
