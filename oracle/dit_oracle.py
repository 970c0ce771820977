"""Plain PyTorch-CPU restatement of the reference's DiT denoiser path (BASELINE
config 5).

TEST INFRASTRUCTURE ONLY (see oracle/__init__): the checker of the HIP DiT path
(dl-swin-gan_amd/dl_cs/models/DiT.py, unrolledDiT.py, dl_cs/diffusion) and the
CPU baseline of its bench key.  Functional style, parameters keyed by the
reference's own state_dict names.  Works in any float dtype (float32 for the
fp32 oracle, float64 for the float64 floor).

Reference files (under /root/reference):
  dit  = dl_cs/models/DiT.py
  lat  = dl_cs/models/Latte.py, ulat = dl_cs/models/unrolledLatte.py
  udit = dl_cs/models/unrolledDiT.py
  gd   = dl_cs/diffusion/gaussian_diffusion.py, dl_cs/diffusion/__init__.py
timm (not installed; unpinned) -- the reference imports
timm.models.vision_transformer.{Attention, Mlp} (dit:18).  Restated here from
timm's published module (qkv Linear -> [3, heads, hd] split -> softmax(q k^T *
hd^-0.5) v -> proj; Mlp fc1 -> act -> fc2, dropout 0): PARITY UNPINNED AGAINST
TIMM ITSELF; pinned against the reference run with the same restatement
(tests/golden/make_golden.py --only dit).
"""
import itertools
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import dlcs_oracle as O

PATCH = (2, 4, 4)
MAX_GRID = (128, 128, 15)          # dit:257 PosEmbed(max_grid_size)


# ----------------------------------------------------------------------------
# embeddings
# ----------------------------------------------------------------------------


def timestep_embedding(t, dim=256, max_period=10000):
    """dit:198-216 -- [cos(t f), sin(t f)], f = exp(-ln(max_period) k / half)."""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(start=0, end=half, dtype=torch.float32) / half)
    args = t[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


def t_embedder(P, pre, t, dtype):
    """dit:218-221 -- Linear(256, D) -> SiLU -> Linear(D, D)."""
    f = timestep_embedding(t).to(dtype)
    h = F.silu(F.linear(f, P[pre + "mlp.0.weight"], P[pre + "mlp.0.bias"]))
    return F.linear(h, P[pre + "mlp.2.weight"], P[pre + "mlp.2.bias"])


def y_embedder(P, pre, labels):
    """dit:246-251 in eval mode (no label dropout) -- table lookup."""
    return P[pre + "embedding_table.weight"][labels]


def _sincos_1d(embed_dim, pos):
    """dit:771-789"""
    omega = np.arange(embed_dim // 2, dtype=np.float64)
    omega /= embed_dim / 2.
    omega = 1. / 10000 ** omega
    out = np.einsum('m,d->md', pos.reshape(-1), omega)
    return np.concatenate([np.sin(out), np.cos(out)], axis=1)


def pos_embed_table(hidden, max_grid=MAX_GRID):
    """dit:711-741 (get_3d_sincos_pos_embed over the max grid) -> float32 [prod(max_grid), hidden].
    meshgrid's default 'xy' indexing makes the grid (g1, g0, g2)-shaped."""
    g0 = np.arange(max_grid[0], dtype=np.float32)
    g1 = np.arange(max_grid[1], dtype=np.float32)
    g2 = np.arange(max_grid[2], dtype=np.float32)
    grid = np.stack(np.meshgrid(g0, g1, g2), axis=0).reshape(3, 1, max_grid[0], max_grid[1], max_grid[2])
    d3 = hidden // 3
    emb = np.concatenate([_sincos_1d(d3, grid[0]), _sincos_1d(d3, grid[1]), _sincos_1d(d3, grid[2])], axis=1)
    return torch.from_numpy(emb).float()


def pos_index(grid, max_grid=MAX_GRID):
    """dit:268-305 -- rows of the table used for a (F, H, W) token grid, in token
    order.  The reference's loop `for w, h, f in product(range(F), range(H),
    range(W))` binds w to the frame index and f to the width index:
    index = f + h * max_F + w * max_F * max_H."""
    Fd, H, W = grid
    mF, mH, _ = max_grid
    return np.array([f + h * mF + w * mF * mH for w, h, f in itertools.product(range(Fd), range(H), range(W))],
                    dtype=np.int64)


# ----------------------------------------------------------------------------
# DiT block (dit:311-350) with timm Attention / Mlp
# ----------------------------------------------------------------------------


def modulate(x, shift, scale):
    """dit:22-23"""
    return x * (1 + scale.unsqueeze(1)) + shift.unsqueeze(1)


def attention(P, pre, x, heads):
    """timm vision_transformer.Attention (qkv_bias=True, no qk-norm, dropout 0)."""
    B, N, C = x.shape
    hd = C // heads
    qkv = F.linear(x, P[pre + "qkv.weight"], P[pre + "qkv.bias"]).reshape(B, N, 3, heads, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    attn = torch.softmax((q * hd ** -0.5) @ k.transpose(-2, -1), dim=-1)
    out = (attn @ v).transpose(1, 2).reshape(B, N, C)
    return F.linear(out, P[pre + "proj.weight"], P[pre + "proj.bias"])


def mlp(P, pre, x):
    """timm Mlp with act_layer GELU(approximate='tanh') (dit:322-323), drop 0."""
    h = F.gelu(F.linear(x, P[pre + "fc1.weight"], P[pre + "fc1.bias"]), approximate="tanh")
    return F.linear(h, P[pre + "fc2.weight"], P[pre + "fc2.bias"])


def factorize(x, ps, flag):
    """dit:55-65 -- flag 0: sequences over the H*W tokens of a frame; flag 1:
    sequences over the frames of a spatial position."""
    b, d, f, h, w = ps
    if flag == 0:
        return x.reshape(b * f, h * w, d)
    return x.reshape(b, f, h, w, d).permute(0, 2, 3, 1, 4).reshape(b * h * w, f, d)


def unfactorize(x, ps, flag):
    """dit:67-76"""
    b, d, f, h, w = ps
    if flag == 0:
        return x.reshape(b, f * h * w, d)
    return x.reshape(b, h, w, f, d).permute(0, 3, 1, 2, 4).reshape(b, f * h * w, d)


def _ln(x):
    return F.layer_norm(x, (x.shape[-1],), eps=1e-6)


def dit_block_factor(P, pre, x, c, ps, heads):
    """dit:329-350.  Both attentions share self.attn; the second one is
    modulated with the *spatial* shift / scale (dit:342), so shift/scale_msa_temporal
    are unused; norm1 / norm2 / norm3 have no affine parameters, eps 1e-6."""
    mod = F.linear(F.silu(c), P[pre + "adaLN_modulation.1.weight"], P[pre + "adaLN_modulation.1.bias"])
    sh_s, sc_s, g_s, _sh_t, _sc_t, g_t, sh_m, sc_m, g_m = mod.chunk(9, dim=1)
    r = x
    h = attention(P, pre + "attn.", factorize(modulate(_ln(x), sh_s, sc_s), ps, 1), heads)
    x = g_s.unsqueeze(1) * unfactorize(h, ps, 1) + r
    r = x
    h = attention(P, pre + "attn.", factorize(modulate(_ln(x), sh_s, sc_s), ps, 0), heads)
    x = g_t.unsqueeze(1) * unfactorize(h, ps, 0) + r
    return x + g_m.unsqueeze(1) * mlp(P, pre + "mlp.", modulate(_ln(x), sh_m, sc_m))


def final_layer(P, pre, x, c):
    """dit:404-408"""
    mod = F.linear(F.silu(c), P[pre + "adaLN_modulation.1.weight"], P[pre + "adaLN_modulation.1.bias"])
    shift, scale = mod.chunk(2, dim=1)
    return F.linear(modulate(_ln(x), shift, scale), P[pre + "linear.weight"], P[pre + "linear.bias"])


def calc_num_patch(shape, patch=PATCH):
    """dit:30-53 -> (grid, pad)"""
    _, _, D, H, W = shape
    pad = [(p - n % p) % p for n, p in zip((D, H, W), patch)]
    grid = [(n + q) // p for n, q, p in zip((D, H, W), pad, patch)]
    return grid, pad


def dit(P, pre, x, t, y, depth, heads, patch=PATCH, pos_table=None):
    """dit:546-579 -- DiT.forward with DiTBlockFactor blocks; x [N, C, F, H, W]."""
    N, Cin, D, H, W = x.shape
    grid, pad = calc_num_patch(x.shape, patch)
    xp = F.pad(x, (0, pad[2], 0, pad[1], 0, pad[0]))                               # dit:117-122
    e = F.conv3d(xp, P[pre + "x_embedder.proj.weight"], P[pre + "x_embedder.proj.bias"], stride=patch)
    ps = e.shape                                                                   # dit:125
    tok = e.reshape(e.shape[0], e.shape[1], -1).permute(0, 2, 1)                   # dit:135-136
    hidden = tok.shape[-1]
    if pos_table is None:
        pos_table = pos_embed_table(hidden)
    tok = tok + pos_table.to(tok.dtype)[torch.from_numpy(pos_index(grid))].unsqueeze(0)   # dit:571
    c = t_embedder(P, pre + "t_embedder.", t, tok.dtype) + y_embedder(P, pre + "y_embedder.", y)   # dit:572-574
    for i in range(depth):
        tok = dit_block_factor(P, f"{pre}blocks.{i}.", tok, c, ps, heads)
    out = final_layer(P, pre + "final_layer.", tok, c)
    # unpatchify2 (dit:515-543)
    Cout = out.shape[-1] // (patch[0] * patch[1] * patch[2])
    f, h, w = D + pad[0], H + pad[1], W + pad[2]
    out = out.reshape(N, f // patch[0], h // patch[1], w // patch[2], patch[0], patch[1], patch[2], Cout)
    out = torch.einsum('nfhwpqrc->ncfphqwr', out).reshape(N, Cout, f, h, w)
    return out[:, :, math.ceil(pad[0] / 2):f - math.floor(pad[0] / 2),
               math.ceil(pad[1] / 2):h - math.floor(pad[1] / 2),
               math.ceil(pad[2] / 2):w - math.floor(pad[2] / 2)]


def _pre(x, pad):
    """dit:1307-1319 (== s3d:394-406): cat(re, im), circular pad in T."""
    u = torch.cat((x.real, x.imag), dim=1)
    return F.pad(u, (0, 0, 0, 0, pad, pad), mode="circular")


def _post(o, pad):
    """dit:1321-1331"""
    o = o[:, :, pad:o.shape[2] - pad]
    E = o.shape[1] // 2
    return torch.complex(o[:, :E].contiguous(), o[:, E:].contiguous())


def dit_resnet(P, x, t, c, depth, heads, num_blocks=0, kernel_size=3, pos_table=None, relu=F.relu):
    """dit:1284-1350 -- DiTResNet.forward: SFE conv -> DiT (in_channels = chans)
    -> ReLU + conv(x + res) -> crop, complex.  (`relu`: see dlcs_oracle.MaskedRelu.)"""
    pad = (2 * num_blocks + 2) * (kernel_size - 1) // 2                            # dit:1293
    u = _pre(x, pad)
    res = O.conv_block(P, "SFE.", u, act=False)                                    # dit:1339
    o = dit(P, "DiT.", res, t, c, depth, heads, pos_table=pos_table)               # dit:1341
    o = O.conv_block(P, "final_layer.", o + res, relu=relu)                        # dit:1344
    return _post(o, pad)


def dit_net(P, x, t, c, depth, heads, num_blocks=0, kernel_size=3, pos_table=None):
    """dit:1199-1282 -- DiTNet.forward: the DiT straight on the 2E channels."""
    pad = (2 * num_blocks + 2) * (kernel_size - 1) // 2
    return _post(dit(P, "DiT.", _pre(x, pad), t, c, depth, heads, pos_table=pos_table), pad)


# ----------------------------------------------------------------------------
# Latte (lat = dl_cs/models/Latte.py; ulat = dl_cs/models/unrolledLatte.py)
# ----------------------------------------------------------------------------

LATTE_MAX_GRID = (128, 128)        # lat:165 PosEmbed(max_grid_size)


def latte_pos_table(hidden, max_grid=LATTE_MAX_GRID):
    """lat:593-619 -- 2-D sin-cos table (meshgrid 'xy': w goes first): row
    i * max_W + j = [sincos(D/2, j), sincos(D/2, i)]."""
    g = np.meshgrid(np.arange(max_grid[1], dtype=np.float32), np.arange(max_grid[0], dtype=np.float32))
    grid = np.stack(g, axis=0).reshape(2, 1, max_grid[0], max_grid[1])
    emb = np.concatenate([_sincos_1d(hidden // 2, grid[0]), _sincos_1d(hidden // 2, grid[1])], axis=1)
    return torch.from_numpy(emb).float()


def latte_temp_table(hidden, max_frames=100):
    """lat:149-159, :589-591 -- 1-D sin-cos table over frames."""
    return torch.from_numpy(_sincos_1d(hidden, np.arange(max_frames, dtype=np.float64))).float()


def latte_pos_index(H, W, max_grid=LATTE_MAX_GRID):
    """lat:179-191 -- [h + w * max_H for w, h in product(range(H), range(W))]."""
    return np.array([h + w * max_grid[0] for w, h in itertools.product(range(H), range(W))], dtype=np.int64)


def latte_block(P, pre, x, c, heads):
    """lat:311-316 -- adaLN-Zero TransformerBlock on x [nseq, N, D] with c [nseq, D]."""
    mod = F.linear(F.silu(c), P[pre + "adaLN_modulation.1.weight"], P[pre + "adaLN_modulation.1.bias"])
    sh_a, sc_a, g_a, sh_m, sc_m, g_m = mod.chunk(6, dim=1)
    x = x + g_a.unsqueeze(1) * attention(P, pre + "attn.", modulate(_ln(x), sh_a, sc_a), heads)
    return x + g_m.unsqueeze(1) * mlp(P, pre + "mlp.", modulate(_ln(x), sh_m, sc_m))


def latte(P, pre, x, t, depth, heads, patch=(4, 4), pos_table=None, temp_table=None):
    """lat:477-560 -- Latte.forward (extras = 1) on x [B, C, F, H, W]."""
    B, C, Fr, H, W = x.shape
    pad = [(p - n % p) % p for n, p in zip((H, W), patch)]                        # lat:193-214
    grid = [(n + q) // p for n, q, p in zip((H, W), pad, patch)]
    xf = x.permute(0, 2, 1, 3, 4).reshape(B * Fr, C, H, W)                        # lat:503-504
    xf = F.pad(xf, (0, pad[1], 0, pad[0]))                                         # lat:126-129
    e = F.conv2d(xf, P[pre + "x_embedder.proj.weight"], P[pre + "x_embedder.proj.bias"], stride=patch)
    tok = e.reshape(e.shape[0], e.shape[1], -1).permute(0, 2, 1)                   # lat:142-145
    D = tok.shape[-1]
    if pos_table is None:
        pos_table = latte_pos_table(D)
    if temp_table is None:
        temp_table = latte_temp_table(D)
    tok = tok + pos_table.to(tok.dtype)[torch.from_numpy(latte_pos_index(*grid))].unsqueeze(0)   # lat:514-516
    temp = temp_table.to(tok.dtype)[:Fr].unsqueeze(0)                              # lat:518
    te = t_embedder(P, pre + "t_embedder.", t, tok.dtype)                          # lat:521
    c_s = te.repeat_interleave(Fr, dim=0)                                          # lat:522 repeat '(n c) d'
    Np = tok.shape[1]
    c_t = te.repeat_interleave(Np, dim=0)                                          # lat:523
    for i in range(0, depth, 2):                                                   # lat:533-550
        tok = latte_block(P, f"{pre}blocks.{i}.", tok, c_s, heads)
        tok = tok.reshape(B, Fr, Np, D).permute(0, 2, 1, 3).reshape(B * Np, Fr, D)  # '(b f) t d -> (b t) f d'
        if i == 0:
            tok = tok + temp
        tok = latte_block(P, f"{pre}blocks.{i + 1}.", tok, c_t, heads)
        tok = tok.reshape(B, Np, Fr, D).permute(0, 2, 1, 3).reshape(B * Fr, Np, D)  # '(b t) f d -> (b f) t d'
    out = final_layer(P, pre + "final_layer.", tok, c_s)                           # lat:556
    # unpatchify2 (lat:450-475)
    Cout = out.shape[-1] // (patch[0] * patch[1])
    h, w = H + pad[0], W + pad[1]
    out = out.reshape(B * Fr, h // patch[0], w // patch[1], patch[0], patch[1], Cout)
    out = torch.einsum('nhwpqc->nchpwq', out).reshape(B * Fr, Cout, h, w)
    out = out[:, :, math.ceil(pad[0] / 2):h - math.floor(pad[0] / 2), math.ceil(pad[1] / 2):w - math.floor(pad[1] / 2)]
    out = out.reshape(B, Fr, Cout, out.shape[-2], out.shape[-1])                   # lat:559-560
    return out.permute(0, 2, 1, 3, 4)


def latte_net(P, x, t, depth, heads, num_blocks=0, kernel_size=3, pos_table=None, temp_table=None):
    """lat:926-937 -- LatteNet.forward: pre-process, Latte, post-process (the SFE /
    final ConvBlocks are constructed but not called)."""
    pad = (2 * num_blocks + 2) * (kernel_size - 1) // 2                            # lat:870
    o = latte(P, "Latte.", _pre(x, pad), t, depth, heads, pos_table=pos_table, temp_table=temp_table)
    return _post(o, pad)


def latte_pgd(Ps, x0, t, maps, weights, depth, heads, step_size=-2.0, pos_table=None, temp_table=None):
    """ulat:233-265 (= udit:198-231 with LatteNet)."""
    x = x0
    for P in Ps:
        x = x + step_size * (O.sense_adjoint(O.sense_forward(x, maps, weights), maps, weights) - x0)
        x = latte_net(P, x, t, depth, heads, pos_table=pos_table, temp_table=temp_table)
    return x


# ----------------------------------------------------------------------------
# unrolled drivers (udit) and the diffusion training loss (gd)
# ----------------------------------------------------------------------------


def split_unrolls(sd, n, prefix="nn_update"):
    out = []
    for i in range(n):
        p = f"{prefix}.{i}."
        out.append({k[len(p):]: v for k, v in sd.items() if k.startswith(p)})
    return out


def _relu(relus):
    return F.relu if relus is None else relus()


def pgd(Ps, x0, t, c, maps, weights, depth, heads, step_size=-2.0, pos_table=None, relus=None):
    """udit:198-231 -- x <- R_i(x + s (A^H A x - x0)), ATy = x0.  (`relus`: a
    callable handing out one ReLU per network call, tests' HipMasks.relu.)"""
    x = x0
    for P in Ps:
        x = x + step_size * (O.sense_adjoint(O.sense_forward(x, maps, weights), maps, weights) - x0)
        x = dit_resnet(P, x, t, c, depth, heads, pos_table=pos_table, relu=_relu(relus))
    return x


def data_consistency(Ps, x0, t, c, maps, mask_p, depth, heads, pos_table=None, relus=None):
    """udit:147-181 -- x <- A_F^H (A_1 R_i(x) + A x0), A = S(maps, mask_p),
    A_1 = S(maps, 1 - mask_p), A_F = S(maps) (train_DiT.py:249-254)."""
    x = x0
    for P in Ps:
        z = dit_resnet(P, x, t, c, depth, heads, pos_table=pos_table, relu=_relu(relus))
        k = O.sense_forward(z, maps, 1 - mask_p) + O.sense_forward(x0, maps, mask_p)
        x = O.sense_adjoint(k, maps, None)
    return x


def ddpm(Ps, x0, t, c, depth, heads, pos_table=None):
    """udit:111-135 -- the DiTs chained, no data consistency."""
    x = x0
    for P in Ps:
        x = dit_resnet(P, x, t, c, depth, heads, pos_table=pos_table)
    return x


def betas(schedule, n=1000):
    """gd:106-133 (note beta_end = scale * 0.0008 for 'linear', gd:117) and
    gd:135-152; float64."""
    if schedule == "linear":
        scale = 1000 / n
        return np.linspace(scale * 0.0001, scale * 0.0008, n, dtype=np.float64)
    if schedule == "squaredcos_cap_v2":
        ab = lambda s: math.cos((s + 0.008) / 1.008 * math.pi / 2) ** 2
        return np.array([min(1 - ab((i + 1) / n) / ab(i / n), 0.999) for i in range(n)])
    raise NotImplementedError(schedule)


def alphas_cumprod(schedule="linear", n=1000):
    """gd:185-187 as built by create_diffusion (diffusion/__init__.py:10-46):
    SpacedDiffusion with every step kept re-derives the betas from the base
    cumulative product (respace.py:73-86) before the cumulative product."""
    ab0 = np.cumprod(1.0 - betas(schedule, n))
    nb, last = [], 1.0
    for a in ab0:
        nb.append(1 - a / last)
        last = a
    return np.cumprod(1.0 - np.array(nb))


def q_sample(x_start_ri, t, noise, schedule="linear", n=1000):
    """gd:226-241 with gd:1039-1051 (_extract_into_tensor: float64 table ->
    float32 per-sample coefficient)."""
    ab = alphas_cumprod(schedule, n)
    a = torch.from_numpy(np.sqrt(ab))[t].float()
    b = torch.from_numpy(np.sqrt(1.0 - ab))[t].float()
    sh = (-1,) + (1,) * (x_start_ri.ndim - 1)
    return a.view(sh).to(x_start_ri.dtype) * x_start_ri + b.view(sh).to(x_start_ri.dtype) * noise


def ri(x):
    """gd:15-17"""
    return torch.cat((x.real, x.imag), dim=1)


def cplx(x):
    """gd:19-22"""
    c = x.shape[1]
    return torch.complex(x[:, :c // 2], x[:, c // 2:])


def training_kspace_loss(model_fn, x_start, t, maps, target, noise, schedule="linear"):
    """gd:837-873 -- x_t = q_sample(x_start); out = model(x_t, t, ...);
    loss = mean |A_F out - A_F target| (A_F = SENSE without a mask)."""
    x_t = cplx(q_sample(ri(x_start), t, noise, schedule))
    out = model_fn(x_t)
    return torch.mean(torch.abs(O.sense_forward(out, maps, None) - O.sense_forward(target, maps, None))), out, x_t
