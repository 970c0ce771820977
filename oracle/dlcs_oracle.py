"""Plain PyTorch-CPU (fp32 / complex64) restatement of the reference hot path.

TEST INFRASTRUCTURE ONLY (see oracle/__init__): the checker for the HIP path and
the timed CPU baseline in bench.py.  Functional style: every function takes a
flat parameter dict keyed by the reference's own state_dict names, so the same
weights (oracle/recipe.py) drive the reference, this oracle and the HIP build.

Reference files (under /root/reference):
  tr   = dl_cs/mri/transforms.py
  s3d  = dl_cs/models/swin3D.py
  vst  = dl_cs/models/video_swin_transformer_mri_downsample.py
  urs  = dl_cs/models/unrolledswin.py
  ur   = dl_cs/models/unrolled.py
  r3d  = dl_cs/models/resnet3d.py
  alg  = dl_cs/mri/algorithms.py
  met  = dl_cs/utils/metrics.py
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import windex

# ----------------------------------------------------------------------------
# SENSE operator (tr:12-110)
# ----------------------------------------------------------------------------


def fft2c(x, adjoint=False):
    """tr:31-46 -- uncentered orthonormal FFT over the last two dims."""
    if adjoint:
        return torch.fft.ifftn(x, dim=(-1, -2), norm="ortho")
    return torch.fft.fftn(x, dim=(-1, -2), norm="ortho")


def sense_forward(x, maps, weights):
    """tr:92-98 -- y[b,c,t] = W * F( sum_e S[b,e,c] x[b,e,t] ).
    x c64 [B,E,T,Y,X], maps c64 [B,E,C,1,Y,X], weights f32 [B,1,T,Y,X] or None."""
    d = (x.unsqueeze(2) * maps).sum(1)
    d = fft2c(d)
    return d if weights is None else weights * d


def sense_adjoint(y, maps, weights):
    """tr:84-90 -- x[b,e,t] = sum_c conj(S[b,e,c]) F^-1( W * y[b,c,t] )."""
    d = y if weights is None else weights * y
    d = fft2c(d, adjoint=True)
    return (d.unsqueeze(1) * torch.conj(maps)).sum(2)


# ----------------------------------------------------------------------------
# Swin window attention (vst:88-170) and block (vst:173-273)
# ----------------------------------------------------------------------------

_RPI_CACHE = {}


def _rpi(ws):
    if ws not in _RPI_CACHE:
        _RPI_CACHE[ws] = torch.from_numpy(windex.relative_position_index(ws))
    return _RPI_CACHE[ws]


def window_attention(P, pre, x, mask, num_heads, window_size):
    """vst:139-170.  x [B_, N, C]; mask [nW, N, N] or None.
    window_size is the *constructed* window: the bias index is sliced [:N, :N]."""
    B_, N, C = x.shape
    hd = C // num_heads
    scale = hd ** -0.5
    qkv = F.linear(x, P[pre + "qkv.weight"], P[pre + "qkv.bias"])
    qkv = qkv.reshape(B_, N, 3, num_heads, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    q = q * scale
    attn = q @ k.transpose(-2, -1)
    idx = _rpi(tuple(window_size))[:N, :N].reshape(-1)
    bias = P[pre + "relative_position_bias_table"][idx].reshape(N, N, -1).permute(2, 0, 1)
    attn = attn + bias.unsqueeze(0)
    if mask is not None:
        nW = mask.shape[0]
        attn = attn.view(B_ // nW, nW, num_heads, N, N) + mask.unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, num_heads, N, N)
    attn = torch.softmax(attn, dim=-1)
    out = (attn @ v).transpose(1, 2).reshape(B_, N, C)
    return F.linear(out, P[pre + "proj.weight"], P[pre + "proj.bias"])


def mlp(P, pre, x):
    """vst:20-38 -- fc2(GELU_erf(fc1 x)); dropout 0."""
    h = F.gelu(F.linear(x, P[pre + "fc1.weight"], P[pre + "fc1.bias"]))
    return F.linear(h, P[pre + "fc2.weight"], P[pre + "fc2.bias"])


def _partition(x, ws):
    """vst:41-52"""
    B, D, H, W, C = x.shape
    x = x.view(B, D // ws[0], ws[0], H // ws[1], ws[1], W // ws[2], ws[2], C)
    return x.permute(0, 1, 3, 5, 2, 4, 6, 7).reshape(-1, ws[0] * ws[1] * ws[2], C)


def _reverse(win, ws, B, D, H, W):
    """vst:55-67"""
    x = win.view(B, D // ws[0], H // ws[1], W // ws[2], ws[0], ws[1], ws[2], -1)
    return x.permute(0, 1, 4, 2, 5, 3, 6, 7).reshape(B, D, H, W, -1)


def swin_block(P, pre, x, shift, mask, num_heads, window_size, drop=(1.0, 1.0)):
    """vst:215-273.  x [B,D,H,W,C].  drop = the two DropPath factors of this block
    (vst:252, :266; timm DropPath: 0 for a dropped branch, 1/keep for a kept one,
    one decision per sample -- B = 1 here); (1, 1) = eval mode / p = 0."""
    B, D, H, W, C = x.shape
    ws, ss = windex.get_window_size((D, H, W), window_size, shift)
    h = F.layer_norm(x, (C,), P[pre + "norm1.weight"], P[pre + "norm1.bias"], eps=1e-5)
    pd = (ws[0] - D % ws[0]) % ws[0]
    pb = (ws[1] - H % ws[1]) % ws[1]
    pr = (ws[2] - W % ws[2]) % ws[2]
    h = F.pad(h, (0, 0, 0, pr, 0, pb, 0, pd))
    _, Dp, Hp, Wp, _ = h.shape
    shifted = any(s > 0 for s in ss)
    if shifted:
        h = torch.roll(h, shifts=(-ss[0], -ss[1], -ss[2]), dims=(1, 2, 3))
    win = _partition(h, ws)
    a = window_attention(P, pre + "attn.", win, mask if shifted else None, num_heads, window_size)
    a = _reverse(a.view(-1, *(ws + (C,))), ws, B, Dp, Hp, Wp)
    if shifted:
        a = torch.roll(a, shifts=ss, dims=(1, 2, 3))
    a = a[:, :D, :H, :W, :]
    x = x + drop[0] * a
    return x + drop[1] * mlp(P, pre + "mlp.", F.layer_norm(x, (C,), P[pre + "norm2.weight"],
                                                           P[pre + "norm2.bias"], eps=1e-5))


def swin3d(P, pre, x, depth=6, num_heads=8, window_size=(7, 8, 8), patch=(4, 4, 4), drops=None):
    """vst:735-756 with depths=[6] (single BasicLayer, no PatchMerging/Expand).
    x [B, C, D, H, W] -> same shape.  drops: per block (d0, d1) DropPath factors."""
    pre_size = x.shape
    _, _, D, H, W = x.shape
    x = F.pad(x, (0, (-W) % patch[2], 0, (-H) % patch[1], 0, (-D) % patch[0]))     # vst:464-470
    x = F.conv3d(x, P[pre + "patch_embed.proj.weight"], P[pre + "patch_embed.proj.bias"],
                 stride=patch)                                                      # vst:472
    B, C, d, h, w = x.shape
    shift = tuple(i // 2 for i in window_size)                                      # vst:391
    ws, ss = windex.get_window_size((d, h, w), window_size, shift)                  # vst:424
    Dp, Hp, Wp = windex.padded_grid(d, h, w, ws)
    mask = torch.from_numpy(windex.compute_mask(Dp, Hp, Wp, ws, ss))                # vst:429
    t = x.permute(0, 2, 3, 4, 1).contiguous()
    lp = pre + "layers.0.blocks."
    for i in range(depth):
        t = swin_block(P, f"{lp}{i}.", t, (0, 0, 0) if i % 2 == 0 else shift, mask,
                       num_heads, window_size, drop=drops[i] if drops is not None else (1.0, 1.0))
    x = t.permute(0, 4, 1, 2, 3)
    x = F.conv_transpose3d(x, P[pre + "patch_unembed.proj.weight"],
                           P[pre + "patch_unembed.proj.bias"], stride=patch)        # vst:517
    cs = x.shape
    diff = [cs[j] - pre_size[j] for j in range(5)]                                 # vst:520-524
    return x[:, :, math.ceil(diff[2] / 2):cs[2] - math.floor(diff[2] / 2),
             math.ceil(diff[3] / 2):cs[3] - math.floor(diff[3] / 2),
             math.ceil(diff[4] / 2):cs[4] - math.floor(diff[4] / 2)]


def conv_block(P, pre, x, act=True, relu=F.relu):
    """s3d:225-270 -- Identity norm -> (ReLU) -> Conv3d(k3, p1).
    `relu` replaces the ReLU (tests: a ReLU whose mask is given, see MaskedRelu)."""
    if act:
        x = relu(x)
    return F.conv3d(x, P[pre + "layers.2.conv.weight"], P[pre + "layers.2.conv.bias"], padding=1)


class MaskedRelu:
    """A ReLU whose 0/1 decisions are supplied (TEST INFRASTRUCTURE): called in the
    network's ReLU order, the i-th call returns v * masks[i].  Evaluating the
    oracle (fp32 or float64) with the masks another implementation took in its
    forward removes the one chaotic element of a ReLU network's gradient -- a
    pre-activation within rounding of 0 flips its mask between summation orders
    -- so the gradients can be compared at arithmetic precision.  Records, per
    call, the number of masks that disagree with v > 0 and the largest |v| among
    them (relative to the RMS of v)."""

    def __init__(self, masks):
        self.masks, self.i, self.stats = list(masks), 0, []

    def __call__(self, v):
        m = self.masks[self.i].to(device=v.device)
        self.i += 1
        own = v.detach() > 0
        dis = own != m
        n = int(dis.sum())
        rel = float(v.detach()[dis].abs().max() / v.detach().pow(2).mean().sqrt()) if n else 0.0
        self.stats.append((n, rel))
        return v * m.to(v.dtype)


def swinnet(P, x, num_swinblocks=1, kernel_size=3, relu=F.relu, drops=None, amp_dtype=None):
    """s3d:394-435 -- SwinTransformer3DNet.forward (use_complex_layers=False,
    circular_pad=True).  x c64 [B,E,T,Y,X] -> c64 [B,E,T,Y,X].  drops: per ResSwin
    block, the per-Swin-block DropPath factors (train mode; None = eval).
    amp_dtype (TEST INFRASTRUCTURE, e.g. torch.bfloat16): the real-valued body under
    CPU torch.autocast with the complex boundary kept in fp32 -- the reference itself
    cannot run bf16 (torch.complex refuses bf16 halves at s3d:416), so
    its output is upcast before torch.complex; the bf16 build's error yardstick."""
    pad = (2 * num_swinblocks + 2) * (kernel_size - 1) // 2                        # s3d:380
    u = torch.cat((x.real, x.imag), dim=1)                                         # s3d:399
    u = F.pad(u, (0, 0, 0, 0, pad, pad), mode="circular")                          # s3d:402-404
    with torch.autocast("cpu", dtype=amp_dtype or torch.bfloat16, enabled=amp_dtype is not None):
        s = conv_block(P, "SFE.", u, act=False)                                    # s3d:384
        y = s
        for i in range(num_swinblocks):                                            # s3d:339-340
            pre = f"DFE.resswin_blocks.{i}.layers."
            a = swin3d(P, pre + "0.transformer.", y, drops=drops[i] if drops is not None else None)
            y = conv_block(P, pre + "1.", a, relu=relu) + y
        d = conv_block(P, f"DFE.layers.{num_swinblocks}.", y, relu=relu) + s       # s3d:354-368
        h = s + d                                                                  # s3d:427
        o = conv_block(P, "final_layer.", h, relu=relu)                            # s3d:391
    o = o[:, :, pad:o.shape[2] - pad].to(x.real.dtype)                             # s3d:410
    E = o.shape[1] // 2
    return torch.complex(o[:, :E].contiguous(), o[:, E:].contiguous())             # s3d:416


def pgd(Ps, y, maps, weights, x0=None, step_size=-2.0, reg=None):
    """urs:91-122 (also ur:91-122 with reg = resnet) -- unrolled proximal gradient
    descent.  Ps: list of per-unroll parameter dicts (cnn_update.{i}.* with the
    prefix stripped)."""
    reg = swinnet if reg is None else reg
    ATy = sense_adjoint(y, maps, weights)
    x = ATy if x0 is None else x0
    for P in Ps:
        x = x + step_size * (sense_adjoint(sense_forward(x, maps, weights), maps, weights) - ATy)
        x = reg(P, x)
    return x


def resnet(P, x, num_resblocks=2, kernel_size=3, relu=F.relu):
    """r3d:243-317 (r3d = dl_cs/models/resnet3d.py) -- the ResNet regularizer of the
    "dlespirit" unrolled network.  The pre-activation ReLUs are in place
    (r3d:44, :200-208), so a ResBlock's residual and the final layer see relu(o)."""
    pad = (2 * num_resblocks + 2) * (kernel_size - 1) // 2                          # r3d:253
    E = x.shape[1]
    u = torch.cat((x.real, x.imag), dim=1)                                           # r3d:273-276
    u = F.pad(u, (0, 0, 0, 0, pad, pad), mode="circular")                            # r3d:279-280
    conv = lambda h, pre: F.conv3d(h, P[pre + ".layers.2.conv.weight"], P[pre + ".layers.2.conv.bias"], padding=1)
    o = conv(u, "init_layer")                                                        # act 'none'
    for k in range(num_resblocks):
        r = relu(o)                                                                  # in-place ReLU on the block input
        o = conv(relu(conv(r, f"res_blocks.{k}.layers.0")), f"res_blocks.{k}.layers.1") + r
    o = conv(relu(o), "final_layer") + u                                             # r3d:308
    o = o[:, :, pad:o.shape[2] - pad]                                                # r3d:286
    return torch.complex(o[:, :E].contiguous(), o[:, E:].contiguous())               # r3d:288-292


def _zdot(a, b):
    """alg:38-42 -- sum(conj(a) * b) over the whole batch."""
    return torch.sum(a.conj() * b)


def conjugate_gradient(normal, x, b, num_iter):
    """alg:50-73 -- num_iter CG steps on normal(x) = b from x (no early exit)."""
    r = b - normal(x)
    rsold = _zdot(r, r).real
    p = r
    for _ in range(num_iter):
        Ap = normal(p)
        alpha = rsold / _zdot(p, Ap)
        x = x + alpha * p
        r = r - alpha * Ap
        rsnew = _zdot(r, r).real
        p = (rsnew / rsold) * p + r
        rsold = rsnew
    return x


def hqs(Ps, y, maps, weights, x0=None, lamda=0.1, num_cg=10, reg=None):
    """urs:139-172 -- half-quadratic splitting / MoDL: z = R_i(x);
    x <- CG(A^H A + lamda I, A^H y + lamda z) started from x."""
    reg = swinnet if reg is None else reg
    ATy = sense_adjoint(y, maps, weights)
    x = ATy if x0 is None else x0
    normal = lambda m: sense_adjoint(sense_forward(m, maps, weights), maps, weights) + lamda * m
    for P in Ps:
        z = reg(P, x)
        x = conjugate_gradient(normal, x, ATy + lamda * z, num_cg)
    return x


def split_unrolls(sd, n):
    """Split a ProximalGradientDescent state_dict into per-unroll dicts."""
    out = []
    for i in range(n):
        p = f"cnn_update.{i}."
        out.append({k[len(p):]: v for k, v in sd.items() if k.startswith(p)})
    return out


# ----------------------------------------------------------------------------
# Metrics (met:20-39, met:121-125; LOSS_WEIGHT False)
# ----------------------------------------------------------------------------



# ----------------------------------------------------------------------------
# Conv PatchGAN discriminator (BASELINE config 3).  Not in the reference
# (SURVEY 8a row a22): restates the build-defined network of
# dl_cs/models/patchgan.py, so its parity is pinned to this spec only.
# ----------------------------------------------------------------------------


def patchgan(P, x, relu=F.relu):
    """x c64 [B,E,T,Y,X] -> logits [B,1,T/4,Y/4,X/4]; channels cat(re, im) as s3d:394-406."""
    h = torch.cat((x.real, x.imag), dim=1).to(P["conv1.weight"].dtype)
    h = F.conv3d(h, P["conv1.weight"], P["conv1.bias"], padding=1)
    h = F.conv3d(relu(h), P["conv2.weight"], P["conv2.bias"], padding=1)
    h = F.conv3d(relu(h), P["patch.weight"], P["patch.bias"], stride=4)
    return F.conv3d(relu(h), P["head.weight"], P["head.bias"])

def l2(ref, pred):
    return torch.sqrt(torch.mean(torch.abs(ref - pred) ** 2))


def l1(ref, pred):
    return torch.mean(torch.abs(ref - pred))


def psnr(ref, pred):
    return 20 * torch.log10(torch.abs(ref).max() / l2(ref, pred))


def nrmse(ref, x):
    ref = torch.as_tensor(ref).to(torch.complex128 if torch.is_complex(torch.as_tensor(ref)) else torch.float64)
    x = torch.as_tensor(x).to(ref.dtype)
    return float(torch.linalg.vector_norm(x - ref) / torch.linalg.vector_norm(ref))


def nrmse_np(ref, x):
    ref = np.asarray(ref).astype(np.complex128)
    x = np.asarray(x).astype(np.complex128)
    return float(np.linalg.norm(x - ref) / np.linalg.norm(ref))
