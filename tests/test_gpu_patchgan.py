"""HIP conv PatchGAN discriminator (Swin-GAN, BASELINE config 3) vs the oracle.

The discriminator is build-defined (the reference does not ship one, SURVEY 8a
row a22): parity is against oracle/dlcs_oracle.py::patchgan (torch fp32 CPU
autograd), "parity unpinned" with respect to the reference.  Tolerances: fp32
build NRMSE <= 1e-5 on logits and 1e-4 on gradients (parameters and the input
gradient the generator receives); bf16 build NRMSE <= 2e-2 (SURVEY 8(c) bf16
budget; the gradients pass three bf16-rounded activations).
"""
import pytest
import torch

from goldutil import nrmse
from oracle import dlcs_oracle as O
from oracle import recipe

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(dtype, shape, chans, seed=11):
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
        return errs
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
    errs = _run(torch.bfloat16, (1, 2, 8, 32, 32), 160)
    bad = {k: v for k, v in errs.items() if v > 2e-2}
    assert not bad, errs


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
