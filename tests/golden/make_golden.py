"""Generate the golden vectors by importing the REFERENCE itself.

Runs only in the survey container, where /root/reference exists:

    python tests/golden/make_golden.py [--only NAME]

The reference imports unchanged except for ``timm.models.layers.{DropPath,
trunc_normal_}`` (vst:11), which is not installed here; the two symbols are
restated below in-process (timm is unpinned in environment_swin.yaml:21;
DropPath is the identity in eval mode, trunc_normal_ only affects init and every
fixture overwrites init with oracle/recipe.py).  Nothing from /root/reference is
copied into the repository: the outputs are data (inputs are regenerated from
recipe seeds, expected outputs are stored).
"""
import argparse
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import recipe  # noqa: E402

REF = "/root/reference"


def _install_timm_standin():
    timm = types.ModuleType("timm")
    models = types.ModuleType("timm.models")
    layers = types.ModuleType("timm.models.layers")

    class DropPath(torch.nn.Module):
        """Per-sample stochastic depth (identity in eval mode / p == 0)."""

        def __init__(self, drop_prob=0.0):
            super().__init__()
            self.drop_prob = drop_prob

        def forward(self, x):
            if self.drop_prob == 0.0 or not self.training:
                return x
            keep = 1.0 - self.drop_prob
            m = x.new_empty((x.shape[0],) + (1,) * (x.ndim - 1)).bernoulli_(keep)
            return x * m / keep

    def trunc_normal_(t, mean=0.0, std=1.0, a=-2.0, b=2.0):
        with torch.no_grad():
            return t.normal_(mean, std).clamp_(a, b)

    layers.DropPath = DropPath
    layers.trunc_normal_ = trunc_normal_
    timm.models = models
    models.layers = layers

    # timm.models.vision_transformer.{PatchEmbed, Attention, Mlp} (imported by the
    # DiT denoiser, dit:18), restated from timm's published modules: qkv Linear ->
    # [3, heads, head_dim] split -> softmax(q k^T * head_dim^-0.5) v -> proj;
    # Mlp fc1 -> act -> fc2 (dropout 0, no norm).  Parity unpinned against timm.
    vt = types.ModuleType("timm.models.vision_transformer")
    nn = torch.nn

    class Attention(nn.Module):
        def __init__(self, dim, num_heads=8, qkv_bias=False, qk_norm=False, attn_drop=0.0, proj_drop=0.0,
                     norm_layer=nn.LayerNorm):
            super().__init__()
            self.num_heads = num_heads
            self.head_dim = dim // num_heads
            self.scale = self.head_dim ** -0.5
            self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
            self.q_norm = norm_layer(self.head_dim) if qk_norm else nn.Identity()
            self.k_norm = norm_layer(self.head_dim) if qk_norm else nn.Identity()
            self.attn_drop = nn.Dropout(attn_drop)
            self.proj = nn.Linear(dim, dim)
            self.proj_drop = nn.Dropout(proj_drop)

        def forward(self, x):
            B, N, C = x.shape
            qkv = self.qkv(x).reshape(B, N, 3, self.num_heads, self.head_dim).permute(2, 0, 3, 1, 4)
            q, k, v = qkv.unbind(0)
            q, k = self.q_norm(q), self.k_norm(k)
            attn = (q * self.scale) @ k.transpose(-2, -1)
            attn = self.attn_drop(attn.softmax(dim=-1))
            x = (attn @ v).transpose(1, 2).reshape(B, N, C)
            return self.proj_drop(self.proj(x))

    class Mlp(nn.Module):
        def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU,
                     norm_layer=None, bias=True, drop=0.0, use_conv=False):
            super().__init__()
            out_features = out_features or in_features
            hidden_features = hidden_features or in_features
            self.fc1 = nn.Linear(in_features, hidden_features, bias=bias)
            self.act = act_layer()
            self.drop1 = nn.Dropout(drop)
            self.norm = norm_layer(hidden_features) if norm_layer is not None else nn.Identity()
            self.fc2 = nn.Linear(hidden_features, out_features, bias=bias)
            self.drop2 = nn.Dropout(drop)

        def forward(self, x):
            return self.drop2(self.fc2(self.norm(self.drop1(self.act(self.fc1(x))))))

    class PatchEmbed(nn.Module):     # imported by dit:18, never instantiated on the DiTResNet path
        def __init__(self, *a, **k):
            raise NotImplementedError("timm PatchEmbed stand-in")

    vt.Attention, vt.Mlp, vt.PatchEmbed = Attention, Mlp, PatchEmbed
    models.vision_transformer = vt
    sys.modules.update({"timm": timm, "timm.models": models, "timm.models.layers": layers,
                        "timm.models.vision_transformer": vt})


def _import_ref():
    _install_timm_standin()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import dl_cs.mri.transforms as T
    import dl_cs.models.video_swin_transformer_mri_downsample as vst
    import dl_cs.models.swin3D as s3d
    import dl_cs.models.unrolledswin as urs
    import dl_cs.mri.subsample as ss
    return T, vst, s3d, urs, ss


def _save(name, **arrs):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrs)
    print(f"wrote {path}: {os.path.getsize(path) / 1024:.1f} KiB")


NSAMPLE = 4096
FULL_MAX = 1 << 18          # outputs / input gradients up to 262,144 elements are stored whole
GRAD_FULL_MAX = 2 * NSAMPLE # parameter gradients: sampled above 8,192 elements


def sample_index(numel):
    """Fixed element sample used for large tensors (same function in tests)."""
    rng = np.random.default_rng(numel)
    return np.sort(rng.choice(numel, size=min(NSAMPLE, numel), replace=False))


def _c(x, full_max=FULL_MAX):
    """Tensors above full_max elements are stored as (norm, fixed sample); the rest whole."""
    a = x.detach().numpy()
    if a.size <= full_max:
        return a
    flat = a.reshape(-1)
    return {"norm": np.array(float(np.linalg.norm(flat.astype(np.complex128)))),
            "shape": np.array(a.shape), "sample": flat[sample_index(flat.size)]}


def _put(out, key, val):
    if isinstance(val, dict):
        for k, v in val.items():
            out[f"{key}@{k}"] = v
    else:
        out[key] = val


# grids (D, H, W) on the token lattice: the BASELINE grid, the X=64 training
# crop, a 2x2-window grid, a single-window grid, and a grid that needs padding.
GRIDS = [(7, 48, 40), (7, 48, 16), (7, 16, 16), (7, 8, 8), (7, 12, 10), (3, 16, 24), (8, 8, 8), (8, 48, 40)]
WINDOW = (7, 8, 8)


def gen_windex(vst):
    out = {}
    shift_c = tuple(i // 2 for i in WINDOW)
    for (D, H, W) in GRIDS:
        tag = f"{D}x{H}x{W}"
        ws, ss = vst.get_window_size((D, H, W), WINDOW, shift_c)
        out[f"ws_{tag}"] = np.array(ws)
        out[f"ss_{tag}"] = np.array(ss)
        Dp, Hp, Wp = [int(np.ceil(n / w)) * w for n, w in zip((D, H, W), ws)]
        for shifted in (0, 1):
            s = ss if shifted else (0, 0, 0)
            # partition: token ids (+1, 0 = pad) flow through pad -> roll -> window_partition
            ids = (torch.arange(D * H * W, dtype=torch.float64) + 1).view(1, D, H, W, 1)
            x = torch.nn.functional.pad(ids, (0, 0, 0, Wp - W, 0, Hp - H, 0, Dp - D))
            if any(i > 0 for i in s):
                x = torch.roll(x, shifts=(-s[0], -s[1], -s[2]), dims=(1, 2, 3))
            win = vst.window_partition(x, ws).reshape(-1)
            out[f"part_{tag}_s{shifted}"] = (win.numpy().astype(np.int64) - 1)
            # reverse: row ids flow through window_reverse -> roll back -> crop
            nrow = win.numel()
            rows = (torch.arange(nrow, dtype=torch.float64)).view(-1, *(ws + (1,)))
            y = vst.window_reverse(rows, ws, 1, Dp, Hp, Wp)
            if any(i > 0 for i in s):
                y = torch.roll(y, shifts=s, dims=(1, 2, 3))
            y = y[:, :D, :H, :W, :]
            out[f"rev_{tag}_s{shifted}"] = y.reshape(-1).numpy().astype(np.int64)
        m = vst.compute_mask(Dp, Hp, Wp, ws, ss, torch.device("cpu"))
        out[f"mask_{tag}"] = np.packbits((m.numpy() != 0).reshape(-1))
        out[f"maskshape_{tag}"] = np.array(m.shape)
        uniq = np.unique(m.numpy())
        out[f"maskvals_{tag}"] = uniq
    wa = vst.WindowAttention3D(160, WINDOW, 8, qkv_bias=True)
    out["rpi_7x8x8"] = wa.relative_position_index.numpy().astype(np.int16)
    cases = [((7, 48, 40), (7, 8, 8), (3, 4, 4)), ((7, 8, 8), (7, 8, 8), (3, 4, 4)),
             ((5, 3, 20), (7, 8, 8), (3, 4, 4)), ((8, 9, 9), (7, 8, 8), (0, 0, 0))]
    gws = []
    for xs, w, s in cases:
        a, b = vst.get_window_size(xs, w, s)
        gws.append(list(xs) + list(w) + list(s) + list(a) + list(b))
    out["get_window_size_cases"] = np.array(gws)
    _save("windex", **out)


def gen_sense(T):
    out = {}
    for tag, (B, E, C, Tt, Y, X) in {"small": (1, 2, 3, 2, 24, 20), "mid": (2, 2, 4, 2, 48, 40)}.items():
        maps = recipe.sense_maps(11, B, E, C, Y, X)
        w = recipe.binary_mask(12, (B, 1, Tt, Y, X))
        x = recipe.crandn(13, (B, E, Tt, Y, X))
        y = recipe.crandn(14, (B, C, Tt, Y, X))
        A = T.SenseModel(maps, weights=w)
        _put(out, f"fwd_{tag}", _c(A(x)))
        _put(out, f"adj_{tag}", _c(A(y, adjoint=True)))
        _put(out, f"fwd_nomask_{tag}", _c(T.SenseModel(maps)(x)))
        out[f"shape_{tag}"] = np.array([B, E, C, Tt, Y, X])
    _save("sense", **out)


def _grad_summary(prefix, named, out, full_limit=20000):
    for k, p in named:
        if p.grad is None:
            continue
        g = p.grad.detach().double()
        out[f"{prefix}norm::{k}"] = np.array(float(g.norm()))
        _put(out, f"{prefix}grad::{k}", _c(g.float(), GRAD_FULL_MAX))


def gen_blocks(vst):
    """WindowAttention3D / Mlp / SwinTransformerBlock3D forward + backward."""
    out = {}
    torch.manual_seed(0)
    # -- window attention with the shift mask of a 2x2-window grid
    wa = vst.WindowAttention3D(160, WINDOW, 8, qkv_bias=True)
    recipe.fill_module(wa, 21)
    mask = vst.compute_mask(7, 8, 16, (7, 8, 8), (0, 0, 4), torch.device("cpu"))
    for tag, m in (("mask", mask), ("nomask", None)):
        x = recipe.randn(22, (2, 448, 160)).requires_grad_()
        dy = recipe.randn(23, (2, 448, 160))
        wa.zero_grad()
        y = wa(x, m)
        (y * dy).sum().backward()
        _put(out, f"attn_{tag}_y", _c(y))
        _put(out, f"attn_{tag}_dx", _c(x.grad))
        _grad_summary(f"attn_{tag}_", wa.named_parameters(), out)
    # -- Mlp
    ml = vst.Mlp(160, 640)
    recipe.fill_module(ml, 24)
    x = recipe.randn(25, (896, 160)).requires_grad_()
    dy = recipe.randn(26, (896, 160))
    y = ml(x)
    (y * dy).sum().backward()
    _put(out, "mlp_y", _c(y))
    _put(out, "mlp_dx", _c(x.grad))
    _grad_summary("mlp_", ml.named_parameters(), out)
    # -- full Swin block, shifted, on a padded grid (7, 12, 10)
    for tag, grid in (("blk", (7, 16, 16)), ("blkpad", (7, 12, 10))):
        blk = vst.SwinTransformerBlock3D(160, 8, window_size=WINDOW, shift_size=(3, 4, 4),
                                         qkv_bias=True, drop_path=0.1)
        blk.eval()
        recipe.fill_module(blk, 27)
        D, H, W = grid
        ws, ss = vst.get_window_size(grid, WINDOW, (3, 4, 4))
        Dp, Hp, Wp = [int(np.ceil(n / w)) * w for n, w in zip(grid, ws)]
        m = vst.compute_mask(Dp, Hp, Wp, ws, ss, torch.device("cpu"))
        x = recipe.randn(28, (1, D, H, W, 160)).requires_grad_()
        dy = recipe.randn(29, (1, D, H, W, 160))
        y = blk(x, m)
        (y * dy).sum().backward()
        _put(out, f"{tag}_y", _c(y))
        _put(out, f"{tag}_dx", _c(x.grad))
        _grad_summary(f"{tag}_", blk.named_parameters(), out)
    _save("blocks", **out)


def gen_swinnet(s3d):
    out = {}
    torch.manual_seed(0)
    for tag, (Tt, Y, X) in (("net32", (20, 32, 32)), ("net4840", (20, 48, 40))):
        net = s3d.SwinTransformer3DNet(num_swinblocks=1, in_chans=4, chans=160, kernel_size=3,
                                       window_size=(4, 4))
        net.eval()
        recipe.fill_module(net, 31)
        x = recipe.crandn(32, (1, 2, Tt, Y, X)).requires_grad_()
        y = net(x)
        _put(out, f"{tag}_y", _c(y))
        if tag == "net32":
            g = recipe.crandn(33, y.shape)
            (y.real * g.real + y.imag * g.imag).sum().backward()
            _put(out, f"{tag}_dx", _c(x.grad))
            _grad_summary(f"{tag}_", net.named_parameters(), out)
        print(tag, "done")
    # NUM_SWINBLOCKS = 2 (the reference default, defaults.py:34): two ResSwin blocks
    # in the DFE (s3d:347-357), T pad 6 (s3d:380) -> token grid (8, 8, 8): windows
    # padded in D with the D shift active (vst:391, :424)
    net = s3d.SwinTransformer3DNet(num_swinblocks=2, in_chans=4, chans=160, kernel_size=3, window_size=(4, 4))
    net.eval()
    recipe.fill_module(net, 34)
    x = recipe.crandn(35, (1, 2, 20, 32, 32)).requires_grad_()
    y = net(x)
    g = recipe.crandn(36, y.shape)
    (y.real * g.real + y.imag * g.imag).sum().backward()
    _put(out, "nb2_y", _c(y))
    _put(out, "nb2_dx", _c(x.grad))
    _grad_summary("nb2_", net.named_parameters(), out)
    print("nb2 done")
    _save("swinnet", **out)


class _Cfg:
    """Attribute namespace with the MODEL.PARAMETERS keys urs:23-35 reads."""


def _pgd_cfg(n_unrolls):
    c = _Cfg()
    c.MODEL = _Cfg()
    p = c.MODEL.PARAMETERS = _Cfg()
    p.NUM_UNROLLS = n_unrolls
    p.NUM_SWINBLOCKS = 1
    p.NUM_FEATURES = 160
    p.CONV_BLOCK = _Cfg()
    p.CONV_BLOCK.KERNEL_SIZE = (3,)
    p.CONV_BLOCK.COMPLEX = False
    p.CONV_BLOCK.CIRCULAR_PAD = True
    p.NUM_EMAPS = 2
    p.SHARE_WEIGHTS = False
    p.FIX_STEP_SIZE = True
    p.GRAD_CHECKPOINT = False
    p.WINDOW_SIZE = (4, 4)
    p.NUM_HEAD = 4
    p.NUM_LAYERS = 4
    return c


def gen_pgd(T, urs):
    out = {}
    torch.manual_seed(0)
    # --- 2 unrolls, fwd + bwd of the training loss (complex L1, train_swin.py:134)
    B, E, C, Tt, Y, X = 1, 2, 8, 20, 32, 32
    model = urs.ProximalGradientDescent(_pgd_cfg(2))
    model.eval()
    recipe.fill_module(model, 41)
    maps = recipe.sense_maps(42, B, E, C, Y, X)
    mask = recipe.binary_mask(43, (B, 1, Tt, Y, X))
    y = recipe.crandn(44, (B, C, Tt, Y, X)) * mask
    target = recipe.crandn(45, (B, E, Tt, Y, X))
    A = T.SenseModel(maps, weights=mask)
    pred = model(y=y, A=A, x0=None)
    loss = torch.mean(torch.abs(target - pred))
    loss.backward()
    _put(out, "pgd2_pred", _c(pred))
    out["pgd2_loss"] = np.array(float(loss))
    _grad_summary("pgd2_", model.named_parameters(), out)
    print("pgd2 done")
    # --- 10 unrolls, eval forward at 64x64 (2x2 shifted windows)
    B, E, C, Tt, Y, X = 1, 2, 8, 20, 64, 64
    model = urs.ProximalGradientDescent(_pgd_cfg(10))
    model.eval()
    recipe.fill_module(model, 51)
    maps = recipe.sense_maps(52, B, E, C, Y, X)
    mask = recipe.binary_mask(53, (B, 1, Tt, Y, X))
    y = recipe.crandn(54, (B, C, Tt, Y, X)) * mask
    with torch.no_grad():
        pred = model(y=y, A=T.SenseModel(maps, weights=mask), x0=None)
    _put(out, "pgd10_pred", _c(pred))
    _save("pgd", **out)


def gen_hqs(T, urs):
    """HalfQuadraticSplitting (urs:125-172) + ConjugateGradient (alg:11-73):
    2 unrolls x 10 CG steps, fwd + bwd of the complex-L1 loss with a learnable
    lamda (FIX_STEP_SIZE False), and a 3-unroll eval forward at 48x40."""
    out = {}
    torch.manual_seed(0)
    B, E, C, Tt, Y, X = 1, 2, 8, 20, 32, 32
    cfg = _pgd_cfg(2)
    cfg.MODEL.PARAMETERS.FIX_STEP_SIZE = False
    cfg.MODEL.PARAMETERS.MODL = _Cfg()
    cfg.MODEL.PARAMETERS.MODL.NUM_CG_STEPS = 10
    model = urs.HalfQuadraticSplitting(cfg)
    model.eval()
    recipe.fill_module(model, 61)
    maps = recipe.sense_maps(62, B, E, C, Y, X)
    mask = recipe.binary_mask(63, (B, 1, Tt, Y, X))
    y = recipe.crandn(64, (B, C, Tt, Y, X)) * mask
    target = recipe.crandn(65, (B, E, Tt, Y, X))
    pred = model(y=y, A=T.SenseModel(maps, weights=mask), x0=None)
    loss = torch.mean(torch.abs(target - pred))
    loss.backward()
    _put(out, "hqs2_pred", _c(pred))
    out["hqs2_loss"] = np.array(float(loss))
    out["hqs2_lamda_grad"] = model.lamda.grad.detach().numpy()
    _grad_summary("hqs2_", model.named_parameters(), out)
    print("hqs2 done")
    B, E, C, Tt, Y, X = 1, 2, 8, 20, 48, 40
    cfg = _pgd_cfg(3)
    cfg.MODEL.PARAMETERS.MODL = _Cfg()
    cfg.MODEL.PARAMETERS.MODL.NUM_CG_STEPS = 10
    model = urs.HalfQuadraticSplitting(cfg)
    model.eval()
    recipe.fill_module(model, 71)
    maps = recipe.sense_maps(72, B, E, C, Y, X)
    mask = recipe.binary_mask(73, (B, 1, Tt, Y, X))
    y = recipe.crandn(74, (B, C, Tt, Y, X)) * mask
    with torch.no_grad():
        pred = model(y=y, A=T.SenseModel(maps, weights=mask), x0=None)
    _put(out, "hqs3_pred", _c(pred))
    _save("hqs", **out)


def gen_resnet(T):
    """The "dlespirit" unrolled ResNet (BASELINE config 1, configs/example.yaml:
    NUM_RESBLOCKS 2, NUM_FEATURES 64, NUM_EMAPS 1), dl_cs/models/unrolled.py
    ProximalGradientDescent with resnet3d.ResNet: 2 unrolls at 32 x 32, fwd + bwd
    of the complex-L1 loss."""
    import dl_cs.models.unrolled as ur
    out = {}
    torch.manual_seed(0)
    B, E, C, Tt, Y, X = 1, 1, 8, 20, 32, 32
    cfg = _pgd_cfg(2)
    cfg.MODEL.PARAMETERS.NUM_RESBLOCKS = 2
    cfg.MODEL.PARAMETERS.NUM_FEATURES = 64
    cfg.MODEL.PARAMETERS.NUM_EMAPS = 1
    model = ur.ProximalGradientDescent(cfg)
    model.eval()
    recipe.fill_module(model, 81)
    maps = recipe.sense_maps(82, B, E, C, Y, X)
    mask = recipe.binary_mask(83, (B, 1, Tt, Y, X))
    y = recipe.crandn(84, (B, C, Tt, Y, X)) * mask
    target = recipe.crandn(85, (B, E, Tt, Y, X))
    pred = model(y=y, A=T.SenseModel(maps, weights=mask), x0=None)
    loss = torch.mean(torch.abs(target - pred))
    loss.backward()
    _put(out, "res2_pred", _c(pred))
    out["res2_loss"] = np.array(float(loss))
    _grad_summary("res2_", model.named_parameters(), out)
    _save("resnet", **out)


def gen_misc(ss):
    out = {}
    mf = ss.VDktMaskFunc((10, 15), sim_partial_kx=0.25, sim_partial_ky=0.25)
    m = mf((1, 1, 20, 192, 160), seed=1000)
    out["vdkt_seed1000_bits"] = np.packbits((m.numpy() != 0).reshape(-1))
    out["vdkt_seed1000_shape"] = np.array(m.shape)
    out["vdkt_seed1000_sum"] = np.array(float(m.sum()))
    # metrics (met:20-39, met:121-125) on recipe tensors -- restated formulas
    ref = recipe.crandn(61, (1, 2, 4, 8, 8))
    pred = ref + 0.1 * recipe.crandn(62, (1, 2, 4, 8, 8))
    l2 = torch.sqrt(torch.mean(torch.abs(ref - pred) ** 2))
    out["metric_l1"] = np.array(float(torch.mean(torch.abs(ref - pred))))
    out["metric_l2"] = np.array(float(l2))
    out["metric_psnr"] = np.array(float(20 * torch.log10(torch.abs(ref).max() / l2)))
    _save("misc", **out)


# (accelerations, partial_kx, partial_ky, shape, seed) of the extra VDkt masks
VDKT_CASES = [((4, 6), 0.25, 0.0, (1, 1, 8, 32, 40), 7),
              ((10, 15), 0.25, 0.25, (1, 1, 20, 192, 64), 5),
              ((6, 8), 0.1, 0.25, (1, 1, 12, 96, 80), 123),
              ((10, 15), 0.25, 0.25, (1, 1, 20, 192, 160), None)]
# CinePreprocess cases: (C, T, Y, X, E, crop_readout, zpad_pe, slwin, fname)
PREP_CASES = [(4, 8, 32, 40, 2, 16, 0, True, "slice_a.h5"),
              (3, 6, 40, 24, 2, 0, 24, False, "slice_b.h5"),
              (4, 10, 32, 32, 1, 0, 0, True, "slice_c.h5")]


def prep_config(crop, zpad, slwin, accel=(4, 6), pkx=0.25, pky=0.25):
    """The config keys CinePreprocess reads (preprocess.py:37-52, :59, :84, :160)."""
    N = types.SimpleNamespace
    return N(AUG_TRAIN=N(UNDERSAMPLE=N(ACCELERATIONS=accel, PARTIAL_KX=pkx, PARTIAL_KY=pky),
                         CROP_READOUT=crop, ZPAD_PE=zpad),
             MODEL=N(PARAMETERS=N(SLWIN_INIT=slwin, DSLR=N(BLOCK_SIZE=8, NUM_BASIS=4, OVERLAPPING=False))))


def prep_inputs(i, C, T, Y, X, E):
    k = recipe.crandn(700 + i, (C, T, Y, X)).numpy()
    maps = recipe.sense_maps(710 + i, 1, E, C, Y, X)[0].numpy()
    target = recipe.crandn(720 + i, (E, T, Y, X)).numpy()
    return k, maps, target


def gen_prep(ss):
    """VDkt masks at more shapes / seeds, the k-t helpers (ut:29-49) and the full
    CinePreprocess (preprocess.py:128-180, use_seed=True so every random choice
    follows from the file name) on small recipe inputs -- full tensors."""
    import dl_cs.data.preprocess as pp
    import dl_cs.mri.utils as ut
    out = {}
    for i, (acc, pkx, pky, shape, seed) in enumerate(VDKT_CASES):
        m = ss.VDktMaskFunc(acc, sim_partial_kx=pkx, sim_partial_ky=pky)(shape, seed=seed if seed is not None else 0)
        out[f"vdkt{i}_bits"] = np.packbits((m.numpy() != 0).reshape(-1))
    kk = torch.from_numpy(recipe.crandn(730, (1, 3, 9, 12, 10)).numpy()) * \
        torch.from_numpy((recipe.binary_mask(731, (1, 1, 9, 12, 10)).numpy()))
    out["ta_in"] = kk.numpy()
    out["ta_out"] = ut.time_average(kk, dim=2).numpy()
    for w in (1, 3, 5, 9):
        out[f"slwin{w}_out"] = ut.sliding_window(kk, dim=2, window_size=w).numpy()
    for i, (C, T, Y, X, E, crop, zpad, slwin, fname) in enumerate(PREP_CASES):
        pre = pp.CinePreprocess(prep_config(crop, zpad, slwin), use_seed=True)
        res = pre(*prep_inputs(i, C, T, Y, X, E), fname)
        for name, v in zip(("kspace", "mask", "maps", "init", "scale", "target"), res):
            out[f"prep{i}_{name}"] = v.numpy() if torch.is_tensor(v) else np.asarray(v)
    _save("prep", **out)


def _dit_cfg(n_unrolls, layers=2, heads=16, feats=384):
    """The MODEL.PARAMETERS keys udit:20-36 reads (config_dit.yaml values except
    the unroll / layer counts)."""
    c = _pgd_cfg(n_unrolls)
    p = c.MODEL.PARAMETERS
    p.NUM_RESBLOCKS, p.NUM_FEATURES, p.NUM_LAYERS, p.NUM_HEADS = 0, feats, layers, heads
    p.LEARN_SIGMA = False
    return c


def gen_dit(T):
    """DiT denoiser path (BASELINE config 5): DiTResNet /
    DiTNet fwd + bwd, the unrolled PGD (udit:183-231) 2-unroll training step
    (complex L1), the DDPM_X DataConsistency step through the diffusion k-space
    loss (gd:837-873, fixed t / noise / mask), and the diffusion constants."""
    import dl_cs.models.DiT as dit
    import dl_cs.models.unrolledDiT as udit
    from dl_cs.diffusion import create_diffusion
    out = {}
    torch.manual_seed(0)
    B, E, C, Tt, Y, X = 1, 2, 8, 4, 32, 32
    t = torch.tensor([37])
    lab = torch.tensor([1])
    # --- DiTResNet / DiTNet, 2 layers, 384 features, 16 heads, fwd + bwd
    for tag, cls in (("ditres", dit.DiTResNet), ("ditnet", dit.DiTNet)):
        net = cls(num_blocks=0, in_chans=4, chans=384, kernel_size=3, num_heads=16, num_layers=2)
        net.eval()
        recipe.fill_module(net, 301)
        x = recipe.crandn(302, (B, E, Tt, Y, X)).requires_grad_()
        y = net(x, t, lab)
        g = recipe.crandn(303, y.shape)
        (y.real * g.real + y.imag * g.imag).sum().backward()
        _put(out, f"{tag}_y", _c(y))
        _put(out, f"{tag}_dx", _c(x.grad))
        _grad_summary(f"{tag}_", net.named_parameters(), out)
        print(tag, "done")
    # --- unrolled PGD, 2 unrolls: x0 = A^H y, complex-L1 training loss
    model = udit.ProximalGradientDescent(_dit_cfg(2))
    model.eval()
    recipe.fill_module(model, 311)
    maps = recipe.sense_maps(312, B, E, C, Y, X)
    mask = recipe.binary_mask(313, (B, 1, Tt, Y, X))
    yk = recipe.crandn(314, (B, C, Tt, Y, X)) * mask
    target = recipe.crandn(315, (B, E, Tt, Y, X))
    A = T.SenseModel(maps, weights=mask)
    x0 = A(yk, adjoint=True)
    pred = model(x0, t, A, lab)
    loss = torch.mean(torch.abs(target - pred))
    loss.backward()
    _put(out, "ditpgd2_pred", _c(pred))
    out["ditpgd2_loss"] = np.array(float(loss))
    _grad_summary("ditpgd2_", model.named_parameters(), out)
    print("ditpgd2 done")
    # --- DDPM_X: DataConsistency through GaussianDiffusion.training_kspace_loss
    model = udit.DataConsistency(_dit_cfg(2))
    model.eval()
    recipe.fill_module(model, 321)
    diff = create_diffusion(timestep_respacing="", noise_schedule="linear", diffusion_steps=1000,
                            learn_sigma=False, predict_xstart=True)
    mask_p = recipe.binary_mask(322, (B, 1, Tt, Y, X))
    target = recipe.crandn(323, (B, E, Tt, Y, X))
    noise = recipe.randn(324, (B, 2 * E, Tt, Y, X))
    td = torch.tensor([613])
    kw = dict(A=T.SenseModel(maps, weights=mask_p), A_1=T.SenseModel(maps, weights=1 - mask_p),
              A_F=T.SenseModel(maps), A_S=T.SenseModel(maps, weights=mask), fs=target, c=lab)
    terms, im_out, x_t = diff.training_kspace_loss(model, target, td, kw, noise=noise)
    terms["loss"].backward()
    _put(out, "ditdc2_pred", _c(im_out))
    _put(out, "ditdc2_xt", _c(x_t))
    out["ditdc2_loss"] = np.array(float(terms["loss"]))
    _grad_summary("ditdc2_", model.named_parameters(), out)
    print("ditdc2 done")
    # --- diffusion constants and embeddings
    for sched in ("linear", "squaredcos_cap_v2"):
        d = create_diffusion(timestep_respacing="", noise_schedule=sched, diffusion_steps=1000, learn_sigma=False)
        out[f"sqrt_ab_{sched}"] = d.sqrt_alphas_cumprod
        out[f"sqrt_1mab_{sched}"] = d.sqrt_one_minus_alphas_cumprod
    tt = torch.tensor([0, 1, 37, 613, 999])
    out["temb_t"] = tt.numpy()
    out["temb"] = dit.TimestepEmbedder.timestep_embedding(tt, 256).numpy()
    pe = dit.PosEmbed((2, 4, 4), 384)
    out["pos_index_12x48x40"] = np.asarray(
        [f + h * 128 + w * 128 * 128 for w, h, f in __import__("itertools").product(range(12), range(48), range(40))])
    rows = sample_index(pe.pos_embed_table.shape[1])
    out["pos_table_rows"] = rows
    out["pos_table_sample"] = pe.pos_embed_table[0, rows].detach().numpy()
    out["pos_12x48x40_norm"] = np.array(float(pe((12, 48, 40)).double().norm()))
    _save("dit", **out)


def _latte_cfg(n_unrolls, layers=2, heads=6, feats=192):
    """The MODEL.PARAMETERS keys ulat:20-36 reads (config_latte.yaml values except
    the unroll / layer counts)."""
    return _dit_cfg(n_unrolls, layers=layers, heads=heads, feats=feats)


def gen_latte(T):
    """Latte denoiser (BASELINE config 5, config_latte.yaml): LatteNet fwd + bwd
    (2 layers = one spatial / temporal pair, 192 features, 6 heads) and the
    unrolled PGD (ulat:233-265) 2-unroll training step; the 2-D position and
    frame tables and the position index."""
    import dl_cs.models.Latte as lat
    import dl_cs.models.unrolledLatte as ulat
    out = {}
    torch.manual_seed(0)
    B, E, C, Tt, Y, X = 1, 2, 8, 4, 32, 32
    t = torch.tensor([37])
    lab = torch.tensor([1])
    net = lat.LatteNet(num_blocks=0, in_chans=4, chans=192, kernel_size=3, num_heads=6, num_layers=2)
    net.eval()
    recipe.fill_module(net, 501)
    x = recipe.crandn(502, (B, E, Tt, Y, X)).requires_grad_()
    y = net(x, t, lab)
    g = recipe.crandn(503, y.shape)
    (y.real * g.real + y.imag * g.imag).sum().backward()
    _put(out, "latte_y", _c(y))
    _put(out, "latte_dx", _c(x.grad))
    _grad_summary("latte_", net.named_parameters(), out)
    print("latte done")
    # a non-square grid (Y != X): the position index's row / column binding
    net2 = lat.LatteNet(num_blocks=0, in_chans=4, chans=192, kernel_size=3, num_heads=6, num_layers=2)
    net2.eval()
    recipe.fill_module(net2, 504)
    x2 = recipe.crandn(505, (B, E, Tt, 24, 40))
    with torch.no_grad():
        _put(out, "latte_rect_y", _c(net2(x2, t, lab)))
    model = ulat.ProximalGradientDescent(_latte_cfg(2))
    model.eval()
    recipe.fill_module(model, 511)
    maps = recipe.sense_maps(512, B, E, C, Y, X)
    mask = recipe.binary_mask(513, (B, 1, Tt, Y, X))
    yk = recipe.crandn(514, (B, C, Tt, Y, X)) * mask
    target = recipe.crandn(515, (B, E, Tt, Y, X))
    A = T.SenseModel(maps, weights=mask)
    x0 = A(yk, adjoint=True)
    pred = model(x0, t, A, lab)
    loss = torch.mean(torch.abs(target - pred))
    loss.backward()
    _put(out, "lattepgd2_pred", _c(pred))
    out["lattepgd2_loss"] = np.array(float(loss))
    _grad_summary("lattepgd2_", model.named_parameters(), out)
    print("lattepgd2 done")
    pe = lat.PosEmbed((4, 4), 192)
    rows = sample_index(pe.pos_embed_table.shape[1])
    out["pos_table_rows"] = rows
    out["pos_table_sample"] = pe.pos_embed_table[0, rows].detach().numpy()
    out["pos_index_48x40"] = pe.forward((48, 40)).detach().numpy()[0, :, :4]
    te = lat.TempEmbed(192)
    out["temp_table"] = te.temp_embed_table[0].detach().numpy()
    _save("latte", **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count())
    T, vst, s3d, urs, ss = _import_ref()
    jobs = {"windex": lambda: gen_windex(vst), "sense": lambda: gen_sense(T),
            "blocks": lambda: gen_blocks(vst), "swinnet": lambda: gen_swinnet(s3d),
            "pgd": lambda: gen_pgd(T, urs), "hqs": lambda: gen_hqs(T, urs), "resnet": lambda: gen_resnet(T), "misc": lambda: gen_misc(ss), "prep": lambda: gen_prep(ss), "dit": lambda: gen_dit(T),
            "latte": lambda: gen_latte(T)}
    for name, fn in jobs.items():
        if args.only is None or args.only == name:
            fn()


if __name__ == "__main__":
    main()
