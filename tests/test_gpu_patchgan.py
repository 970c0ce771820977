"""HIP conv PatchGAN discriminator (Swin-GAN, BASELINE config 3) vs the oracle.

The discriminator is build-defined (the reference does not ship one, SURVEY 8a
row a22): parity is against oracle/dlcs_oracle.py::patchgan (torch fp32 CPU
autograd), "parity unpinned" with respect to the reference.  Tolerances: fp32
build NRMSE <= 1e-5 on logits and 1e-4 on gradients (parameters and the input
gradient the generator receives); bf16 build: the logits within 2e-2 of fp32 (SURVEY
8(c) bf16 budget); every tensor within 5e-3 of a float64 restatement rounded to
bf16 at the same storage points (_bf16_chain: isolates kernel error), and within
1.25x that restatement's own distance to fp32 (the quantisation floor, up to 0.07
on the first conv's gradients).
"""
import pytest
import torch
import torch.nn.functional as F

from goldutil import nrmse
from oracle import dlcs_oracle as O
from oracle import recipe

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _r(t):
    """Round to bf16 and back (the HIP bf16 path's storage points)."""
    return t.to(torch.bfloat16).double()


def _bf16_chain(P, x, glog):
    """Test-local float64 restatement of the discriminator's fwd + bwd that rounds
    operands to bf16 at exactly the points patchgan._forward/_backward store them
    (u, weights, a1, a2, a3, g, da3, da2, dc1); accumulation stays float64.  It
    separates kernel defects (HIP vs this chain) from bf16 quantisation (this
    chain vs the fp32 oracle).  Returns logits, x.grad, parameter grads."""
    cg = torch.nn.grad
    W = {k: v.detach().double() for k, v in P.items()}
    w1, w2, wp, wh = (_r(W[k]) for k in ("conv1.weight", "conv2.weight", "patch.weight", "head.weight"))
    u = _r(torch.cat((x.real, x.imag), dim=1).double())
    c1 = F.conv3d(u, w1, W["conv1.bias"], padding=1)
    a1 = _r(F.relu(c1))
    c2 = F.conv3d(a1, w2, W["conv2.bias"], padding=1)
    a2 = _r(F.relu(c2))
    p = F.conv3d(a2, wp, W["patch.bias"], stride=4)
    a3 = _r(F.relu(p))
    logits = F.conv3d(a3, wh, W["head.bias"])
    g = _r(glog.double())
    G = {"head.weight": cg.conv3d_weight(a3, wh.shape, g), "head.bias": g.sum((0, 2, 3, 4))}
    da3 = _r(cg.conv3d_input(a3.shape, wh, g)) * (a3 > 0)
    G["patch.weight"] = cg.conv3d_weight(a2, wp.shape, da3, stride=4)
    G["patch.bias"] = da3.sum((0, 2, 3, 4))
    da2 = _r(cg.conv3d_input(a2.shape, wp, da3, stride=4)) * (a2 > 0)
    G["conv2.weight"] = cg.conv3d_weight(a1, w2.shape, da2, padding=1)
    G["conv2.bias"] = da2.sum((0, 2, 3, 4))
    dc1 = _r(cg.conv3d_input(a1.shape, w2, da2, padding=1) * (a1 > 0))
    G["conv1.weight"] = cg.conv3d_weight(u, w1.shape, dc1, padding=1)
    G["conv1.bias"] = dc1.sum((0, 2, 3, 4))
    du = _r(cg.conv3d_input(u.shape, w1, dc1, padding=1))
    E = x.shape[1]
    gx = torch.complex(du[:, :E], du[:, E:])
    return logits, gx, G


def _run(dtype, shape, chans, seed=11, emulate=False):
    from dl_cs.models import patchgan, swin3D
    old = swin3D.get_compute_dtype()
    swin3D.set_compute_dtype(dtype)
    try:
        B, E, T, Y, X = shape
        D = patchgan.PatchGANDiscriminator3D(in_chans=2 * E, chans=chans)
        recipe.fill_module(D, seed)
        for p in D.parameters():          # keep pre-activations away from 0 / saturation
            p.data.mul_(0.5)
        x = recipe.crandn(seed + 1, shape)
        glog = recipe.randn(seed + 2, (B, 1, T // 4, Y // 4, X // 4))
        # oracle (CPU fp32 autograd)
        P = {k: v.detach().clone().requires_grad_() for k, v in D.state_dict().items()}
        xr = x.clone().requires_grad_()
        ref = O.patchgan(P, xr)
        ref.backward(glog)
        # HIP
        Dg = D.to(DEV)
        xg = x.to(DEV).requires_grad_()
        out = Dg(xg)
        out.backward(glog.to(DEV))
        torch.cuda.synchronize()
        errs = {"logits": nrmse(ref.detach(), out.detach().cpu()),
                "x.grad": nrmse(xr.grad, xg.grad.cpu())}
        for n, p in Dg.named_parameters():
            errs[n] = nrmse(P[n].grad, p.grad.cpu())
        if not emulate:
            return errs
        # bf16-rounded restatement: kernel error (hip_vs_emu) vs quantisation floor (emu_vs_fp32)
        el, egx, eG = _bf16_chain(P, x, glog)
        hip_vs_emu = {"logits": nrmse(el, out.detach().cpu()), "x.grad": nrmse(egx, xg.grad.cpu())}
        emu_vs_fp32 = {"logits": nrmse(ref.detach(), el), "x.grad": nrmse(xr.grad, egx)}
        for n, p in Dg.named_parameters():
            hip_vs_emu[n] = nrmse(eG[n], p.grad.cpu())
            emu_vs_fp32[n] = nrmse(P[n].grad, eG[n])
        return errs, hip_vs_emu, emu_vs_fp32
    finally:
        swin3D.set_compute_dtype(old)


@pytest.mark.parametrize("shape", [(1, 2, 4, 16, 16), (1, 2, 8, 24, 16), (2, 2, 4, 8, 12)])
def test_patchgan_fp32(shape):
    errs = _run(torch.float32, shape, 160)
    assert errs["logits"] <= 1e-5, errs
    bad = {k: v for k, v in errs.items() if v > 1e-4}
    assert not bad, errs


@pytest.mark.parametrize("chans", [32, 64])
def test_patchgan_fp32_narrow(chans):
    errs = _run(torch.float32, (1, 2, 4, 16, 16), chans)
    bad = {k: v for k, v in errs.items() if v > 1e-4}
    assert not bad, errs


def test_patchgan_bf16():
    errs, hip_vs_emu, floor = _run(torch.bfloat16, (1, 2, 8, 32, 32), 160, emulate=True)
    print("hip_vs_fp32", errs)
    print("hip_vs_bf16emu", hip_vs_emu)
    print("bf16emu_vs_fp32", floor)
    # Kernel parity: the HIP bf16 chain vs the same chain rounded at the same
    # points in float64 (measured on MI355X: <= 1.6e-3, accumulation order only).
    bad = {k: v for k, v in hip_vs_emu.items() if v > 5e-3}
    assert not bad, hip_vs_emu
    # Against the fp32 oracle the budget is the bf16 quantisation floor itself
    # (measured: 0.072 on conv1.weight -- the deepest gradient passes four bf16
    # roundings, a3/da3/da2/dc1), plus 25 %: the 2e-2 SURVEY budget holds only for
    # outputs and the shallow layers (logits 8.9e-4, head 1.4e-3).
    bad = {k: v for k, v in errs.items() if v > max(2e-2, 1.25 * floor[k])}
    assert not bad, (errs, floor)


def test_patchgan_gan_step_grads_reach_generator():
    """One Swin-GAN generator step: L1 + adversarial BCE; the adversarial term's
    gradient reaches the generator through dlcs kernels only (finite, nonzero)."""
    from dl_cs.config import get_cfg
    from dl_cs.models import patchgan, swin3D, unrolledswin
    from dl_cs.mri import transforms as T
    swin3D.set_compute_dtype(torch.float32)
    cfg = get_cfg()
    Pm = cfg.MODEL.PARAMETERS
    Pm.NUM_UNROLLS, Pm.NUM_SWINBLOCKS, Pm.NUM_FEATURES = 1, 1, 160
    Pm.CONV_BLOCK.COMPLEX, Pm.FIX_STEP_SIZE = False, True
    G = unrolledswin.ProximalGradientDescent(cfg)
    recipe.fill_module(G, 3)
    G = G.to(DEV)
    D = patchgan.PatchGANDiscriminator3D(4, 160)
    recipe.fill_module(D, 4)
    D = D.to(DEV)
    B, E, C, Tt, Y, X = 1, 2, 8, 4, 32, 32
    maps = recipe.sense_maps(1, B, E, C, Y, X).to(DEV)
    mask = recipe.binary_mask(2, (B, 1, Tt, Y, X)).to(DEV)
    target = recipe.crandn(5, (B, E, Tt, Y, X)).to(DEV)
    A = T.SenseModel(maps, weights=mask)
    y = A(target)
    pred = G(y=y, A=A)
    d_fake = D(pred)
    loss = torch.mean(torch.abs(target - pred)) + 0.01 * patchgan.g_adv_loss(d_fake)
    loss.backward()
    g = G.cnn_update[0].SFE.layers[2].conv.weight.grad
    assert g is not None and torch.isfinite(g).all() and g.abs().sum() > 0
    dl = patchgan.d_loss(D(target), D(pred.detach()))
    D.zero_grad()
    dl.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in D.parameters())
