"""Dynamic range of the fp32-on-fp16 conv split (conv3d_f16x3.inc: one
power-of-two scale per tensor, two fp16 planes = 22 significant bits) on
heavy-tailed data, vs float64: one channel x 1e4, and a block of voxels at
2^-20 of the tensor's max (where the low plane runs into fp16 subnormals).

Bound, per region (the whole tensor, and the output voxels computed only from
the small block): NRMSE(HIP vs float64) <= max(1e-5, 4 x NRMSE(torch fp32 CPU
vs float64)) -- the kernel is held to PyTorch's own fp32 conv / the fp32 oracle.
Conv level (fwd, dgrad, wgrad) and SwinNet level (output and input gradient).
"""
import math

import pytest
import torch
import torch.nn.functional as F

from goldutil import nrmse
from oracle import dlcs_oracle as O
from oracle import recipe

pytestmark = pytest.mark.gpu
DEV = "cuda"
SMALL = 2.0 ** -20


def _K():
    from dl_cs.models import _ops as K
    return K


def _to_blocked(x):
    B, C, D, H, W = x.shape
    t = x.permute(0, 2, 3, 4, 1).reshape(B, D // 4, 4, H // 4, 4, W // 4, 4, C)
    return t.permute(0, 1, 3, 5, 2, 4, 6, 7).reshape(-1, C)


def _from_blocked(r, B, C, D, H, W):
    t = r.reshape(B, D // 4, H // 4, W // 4, 4, 4, 4, C).permute(0, 1, 4, 2, 5, 3, 6, 7)
    return t.reshape(B, D, H, W, C).permute(0, 4, 1, 2, 3)


def _heavy(shape, seed, chan):
    """N(0,1) with channel `chan` x 1e4 and the block [:, :, 0:4, 0:8, 0:8] at 2^-20 of the max."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(shape, generator=g)
    x[:, chan] *= 1e4
    mx = float(x.abs().max())
    x[:, :, 0:4, 0:8, 0:8] = torch.randn(x[:, :, 0:4, 0:8, 0:8].shape, generator=g) * (mx * SMALL)
    return x


def _check(label, ref64, ref32, got, regions):
    for name, sl in regions:
        floor = nrmse(ref64[sl].numpy(), ref32[sl].numpy())
        err = nrmse(ref64[sl].numpy(), got[sl].numpy())
        print(f"{label} [{name}]: HIP err vs f64 {err:.3g}, torch fp32 floor {floor:.3g}")
        assert err <= max(1e-5, 4 * floor), (label, name, err, floor)


INNER = (slice(None), slice(None), slice(1, 3), slice(1, 7), slice(1, 7))   # outputs fed only by the small block
ALL = (slice(None),) * 5


def test_conv_f16x3_heavy_tailed():
    K = _K()
    B, C, D, H, W = 1, 160, 8, 16, 16
    grid = (B, D, H, W)
    x = _heavy((B, C, D, H, W), 70, 7)
    g = _heavy((B, C, D, H, W), 71, 3) * 1e-6                  # gradient-sized, also heavy-tailed
    w = torch.randn((C, C, 3, 3, 3), generator=torch.Generator().manual_seed(72)) / (27 * C) ** 0.5
    xd, gd = _to_blocked(x).to(DEV), _to_blocked(g).to(DEV)
    # forward
    out = K.conv3d_f16x3(K.split2(xd), K.conv_pack_f16x3(w.to(DEV), 0), grid)
    got = _from_blocked(out.cpu(), B, C, D, H, W).double()
    ref64 = F.conv3d(x.double(), w.double(), None, padding=1)
    ref32 = F.conv3d(x, w, None, padding=1).double()
    _check("fwd", ref64, ref32, got, [("all", ALL), ("small block", INNER)])
    # dgrad (input gradient of the conv for the heavy-tailed g)
    dx = K.conv3d_f16x3(K.split2(gd), K.conv_pack_f16x3(w.to(DEV), 1), grid)
    got = _from_blocked(dx.cpu(), B, C, D, H, W).double()
    ref64 = torch.nn.grad.conv3d_input(x.shape, w.double(), g.double(), padding=1)
    ref32 = torch.nn.grad.conv3d_input(x.shape, w, g, padding=1).double()
    _check("dgrad", ref64, ref32, got, [("all", ALL), ("small block", INNER)])
    # wgrad from the heavy-tailed x and g
    dwp = torch.zeros((27, C, C), device=DEV)
    K.conv3d_wgrad_f16x3(K.split2(xd), K.split2(gd), grid, dwp)
    gw = torch.zeros((C, C, 3, 3, 3), device=DEV)
    K.conv_unpack_grad(dwp, gw, C, C)
    ref64 = torch.nn.grad.conv3d_weight(x.double(), w.shape, g.double(), padding=1)
    ref32 = torch.nn.grad.conv3d_weight(x, w.shape, g, padding=1).double()
    got = gw.cpu().double()
    rest_o = [i for i in range(C) if i != 3]
    rest_i = [i for i in range(C) if i != 7]
    _check("wgrad", ref64, ref32, got, [("all", (slice(None),) * 5)])
    _check("wgrad", ref64[rest_o][:, rest_i], ref32[rest_o][:, rest_i], got[rest_o][:, rest_i],
           [("channels off the heavy ones", (slice(None),) * 5)])


def test_swinnet_f16x3_heavy_tailed():
    """The fp32 SwinNet (every 160 -> 160 conv on the split) on an input whose
    real part of map 1 is x 1e4 and with a block at 2^-20 of the max: output and
    input gradient vs the float64 oracle, held to the fp32 oracle's floor."""
    from dl_cs.models import swin3D
    old = swin3D.get_compute_dtype()
    swin3D.set_compute_dtype(torch.float32)
    try:
        net = swin3D.SwinTransformer3DNet(num_swinblocks=1, in_chans=4, chans=160, kernel_size=3, window_size=(4, 4))
        net.eval()
        recipe.fill_module(net, 73)
        net = net.to(DEV)
        re = _heavy((1, 2, 20, 32, 32), 74, 1)
        im = _heavy((1, 2, 20, 32, 32), 75, 0) * 1e-4
        x = torch.complex(re, im)
        gy = recipe.crandn(76, (1, 2, 20, 32, 32))
        xg = x.to(DEV).requires_grad_()
        y = net(xg)
        (y.real * gy.real.to(DEV) + y.imag * gy.imag.to(DEV)).sum().backward()
        sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
        outs = {}
        for dt, cd in ((torch.float32, torch.complex64), (torch.float64, torch.complex128)):
            P = {k: (v.to(dt) if torch.is_floating_point(v) else v) for k, v in sd.items()}
            xo = x.detach().to(cd).requires_grad_()
            yo = O.swinnet(P, xo)
            gc = gy.to(cd)
            (yo.real * gc.real + yo.imag * gc.imag).sum().backward()
            outs[dt] = (yo.detach().to(torch.complex128), xo.grad.to(torch.complex128))
        regions = [("all", ALL), ("small block", (slice(None), slice(None), slice(1, 3), slice(1, 7), slice(1, 7)))]
        _check("swinnet out", outs[torch.float64][0], outs[torch.float32][0], y.detach().cpu().to(torch.complex128),
               regions)
        _check("swinnet dx", outs[torch.float64][1], outs[torch.float32][1], xg.grad.cpu().to(torch.complex128),
               regions)
    finally:
        swin3D.set_compute_dtype(old)


def test_conv_f16x3_dgrad_unbiased():
    """The masked input-gradient launch (the backward's default accumulation mode,
    conv3d_f16x3.inc): the matrix core's accumulate truncates toward -inf, an
    offset of one sign for every output that a per-element NRMSE does not see but a
    bias gradient's column sum over all voxels does (tools/dgrad_diag.py).  Bound:
    mean error / mean |ref| below 1e-8 (the uncancelled kernels sit at 5e-8 .. 1e-7),
    per-channel column sums within max(2e-6, 4 x PyTorch fp32's)."""
    K = _K()
    B, C, D, H, W = 1, 160, 8, 64, 64
    grid = (B, D, H, W)
    gen = torch.Generator().manual_seed(81)
    g = torch.randn((B, C, D, H, W), generator=gen)
    m = torch.relu(torch.randn((B, C, D, H, W), generator=gen))          # a post-ReLU mask, half zeros
    w = torch.randn((C, C, 3, 3, 3), generator=gen) / (27 * C) ** 0.5
    dx = K.conv3d_f16x3(K.split2(_to_blocked(g).to(DEV)), K.conv_pack_f16x3(w.to(DEV), 1), grid,
                        mask=_to_blocked(m).to(DEV))
    got = _from_blocked(dx.cpu(), B, C, D, H, W).double()
    keep = (m > 0).double()
    ref64 = torch.nn.grad.conv3d_input(g.shape, w.double(), g.double(), padding=1) * keep
    ref32 = (torch.nn.grad.conv3d_input(g.shape, w, g, padding=1) * (m > 0)).double()
    bias = float((got - ref64).sum() / ref64.abs().sum())
    cs64 = ref64.sum(dim=(0, 2, 3, 4)).numpy()
    cs_err = nrmse(cs64, got.sum(dim=(0, 2, 3, 4)).numpy())
    cs_floor = nrmse(cs64, ref32.sum(dim=(0, 2, 3, 4)).numpy())
    print(f"dgrad: mean err / mean |ref| {bias:+.3g}; column sums {cs_err:.3g} (torch fp32 {cs_floor:.3g}); "
          f"elements {nrmse(ref64.numpy(), got.numpy()):.3g} (torch fp32 {nrmse(ref64.numpy(), ref32.numpy()):.3g})")
    assert abs(bias) < 1e-8, bias
    assert cs_err <= max(2e-6, 4 * cs_floor), (cs_err, cs_floor)
