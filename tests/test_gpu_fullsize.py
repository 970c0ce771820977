"""Parity at the BASELINE shapes: the full 8-coil x 20-frame x
192 x 160 slice (token grid 7 x 48 x 40, 30 windows of 448) and the
config_swin training crop X = 64, against the fp32 PyTorch-CPU oracle (pinned
to the reference's goldens by tests/test_oracle_*.py), full tensors compared.

Tolerances (fp32 build): outputs NRMSE <= 1e-5; input and parameter gradients
held to the float64 floor, per tensor: NRMSE vs a float64 oracle evaluation <=
max(1e-5, 4 x the fp32 oracle's own NRMSE vs float64) (goldutil.H3_GRAD_TOL /
H3_FACTOR, also for the f16x3 split's 22-bit operands), the parameter gradients
with the oracle's ReLU decisions fixed to the HIP forward's (goldutil.
assert_masked_f64: pre-activations within fp32 rounding of 0 flip a ReLU mask
between summation orders; test_gpu_swin.py).
bf16 build (config_swin's 5-unroll bf16 configuration): NRMSE <= 1e-2.
The Swin-GAN step (BASELINE config 3; discriminator build-defined, parity
pinned to the oracle's restatement only) at a reduced slice.
"""
import pytest
import torch

from goldutil import H3_FACTOR, H3_GRAD_TOL, HipMasks, assert_f64_floor, assert_masked_f64, nrmse, oracle_grads
from oracle import dlcs_oracle as O
from oracle import recipe

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _setup():
    from dl_cs.models import swin3D
    old = swin3D.get_compute_dtype()
    swin3D.set_compute_dtype(torch.float32)
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    yield
    swin3D.set_compute_dtype(old)


def _net(seed):
    from dl_cs.models import swin3D
    net = swin3D.SwinTransformer3DNet(num_swinblocks=1, in_chans=4, chans=160, kernel_size=3, window_size=(4, 4))
    net.eval()
    recipe.fill_module(net, seed)
    return net.to(DEV)


def swinnet_grads_f64(sd, x, g):
    """Input and parameter gradients of <swinnet(x), g> evaluated by the oracle in float64."""
    P = {k: (v.detach().cpu().double().requires_grad_("relative_position_index" not in k)
             if torch.is_floating_point(v) else v.detach().cpu()) for k, v in sd.items()}
    xo = x.to(torch.complex128).requires_grad_()
    yo = O.swinnet(P, xo)
    g = g.to(torch.complex128)
    (yo.real * g.real + yo.imag * g.imag).sum().backward()
    return xo.grad.numpy(), {k: v.grad.numpy() for k, v in P.items() if torch.is_tensor(v) and v.grad is not None}


def swinnet_dx_f64(sd, x, g):
    """Input gradient of <swinnet(x), g> evaluated by the oracle in float64."""
    return swinnet_grads_f64(sd, x, g)[0]


def _pgd(n, seed):
    from dl_cs.config import get_cfg
    from dl_cs.models import unrolledswin
    cfg = get_cfg()
    P = cfg.MODEL.PARAMETERS
    P.NUM_UNROLLS, P.NUM_SWINBLOCKS, P.NUM_FEATURES = n, 1, 160
    P.CONV_BLOCK.COMPLEX, P.FIX_STEP_SIZE = False, True
    m = unrolledswin.ProximalGradientDescent(cfg)
    m.eval()
    recipe.fill_module(m, seed)
    return m.to(DEV)


def _slice(X, seed=60):
    B, E, C, Tt, Y = 1, 2, 8, 20, 192
    maps = recipe.sense_maps(seed, B, E, C, Y, X)
    mask = recipe.binary_mask(seed + 1, (B, 1, Tt, Y, X), density=0.08)
    y = recipe.crandn(seed + 2, (B, C, Tt, Y, X)) * mask
    return maps, mask, y


@pytest.mark.parametrize("X", [160, 64])
def test_swinnet_full_size_fwd_bwd(X):
    from dl_cs.models import engine
    net = _net(71)
    x = recipe.crandn(72, (1, 2, 20, 192, X))
    xg = x.to(DEV).requires_grad_()
    engine.CAPTURE = []
    try:
        y = net(xg)
    finally:
        caps, engine.CAPTURE = engine.CAPTURE, None
    g = recipe.crandn(73, y.shape)
    (y.real * g.real.to(DEV) + y.imag * g.imag.to(DEV)).sum().backward()
    P = {k: v.detach().cpu().clone().requires_grad_(torch.is_floating_point(v) and "relative_position_index" not in k)
         for k, v in net.state_dict().items()}
    xo = x.clone().requires_grad_()
    yo = O.swinnet(P, xo)
    (yo.real * g.real + yo.imag * g.imag).sum().backward()
    assert nrmse(yo.detach().numpy(), y.detach().cpu().numpy()) < 1e-5
    # the input gradient crosses four ReLU masks: its floor is the fp32 oracle's own
    # distance from a float64 evaluation (mask flips at |pre-activation| ~ fp32 ulp)
    dx64, pg64 = swinnet_grads_f64(net.state_dict(), x, g)
    floor = nrmse(dx64, xo.grad.numpy())
    err = nrmse(dx64, xg.grad.cpu().numpy())
    print(f"X={X} dx err vs f64 {err:.3g}, oracle32 floor {floor:.3g}")
    assert err < max(1e-5, 4 * floor), (err, floor)
    named = dict(net.named_parameters())
    o32 = {n: v.grad.numpy() for n, v in P.items() if torch.is_tensor(v) and v.grad is not None}
    hip = {n: p.grad for n, p in named.items() if p.grad is not None}
    assert_f64_floor(hip, o32, pg64, f"full-size swinnet X={X} (own masks)")

    def lf(Pm, c, mk):
        yo, gc = O.swinnet(Pm, c(x), relu=mk.relu()), c(g)
        return (yo.real * gc.real + yo.imag * gc.imag).sum()
    assert_masked_f64(hip, lf, net.state_dict(), lambda k: "relative_position_index" not in k, HipMasks(caps),
                      f"full-size swinnet X={X}", min_tol=H3_GRAD_TOL, factor=H3_FACTOR)


def test_pgd_unroll_full_size():
    """One unroll (fused SENSE normal operator + DC + SwinNet, urs:106-120) at
    the BASELINE slice."""
    from dl_cs.mri import transforms as T
    model = _pgd(1, 81)
    maps, mask, y = _slice(160)
    with torch.no_grad():
        out = model(y=y.to(DEV), A=T.SenseModel(maps.to(DEV), weights=mask.to(DEV))).cpu()
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        ref = O.pgd(O.split_unrolls(sd, 1), y, maps, mask)
    assert nrmse(ref.numpy(), out.numpy()) < 1e-5


def test_pgd5_bf16_config_swin():
    """BASELINE config 2: config_swin's 5-iteration unroll in bf16 (fp32 complex
    boundary) vs the fp32 oracle at the BASELINE slice, NRMSE <= 1e-2."""
    from dl_cs.models import swin3D
    from dl_cs.mri import transforms as T
    model = _pgd(5, 91)
    maps, mask, y = _slice(160, 95)
    swin3D.set_compute_dtype(torch.bfloat16)
    with torch.no_grad():
        out = model(y=y.to(DEV), A=T.SenseModel(maps.to(DEV), weights=mask.to(DEV))).cpu()
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        ref = O.pgd(O.split_unrolls(sd, 5), y, maps, mask)
    err = nrmse(ref.numpy(), out.numpy())
    assert err < 1e-2, err


@pytest.mark.parametrize("grid", [(4, 32, 32), (20, 192, 160)])
def test_swin_gan_step_vs_oracle(grid):
    """BASELINE config 3: one generator step of Swin-GAN -- L1 + 0.01 x
    adversarial BCE through the PatchGAN -- and the discriminator's step, both
    vs oracle autograd on the same weights (fp32); a toy grid and the BASELINE
    slice (8 coils x 20 frames x 192 x 160, the 160-feature discriminator at full
    resolution)."""
    import torch.nn.functional as F
    from dl_cs.models import patchgan
    from dl_cs.mri import transforms as T
    B, E, C = 1, 2, 8
    Tt, Y, X = grid
    G = _pgd(1, 101)
    D = patchgan.PatchGANDiscriminator3D(4, 160)
    recipe.fill_module(D, 102)
    D = D.to(DEV)
    maps = recipe.sense_maps(103, B, E, C, Y, X)
    mask = recipe.binary_mask(104, (B, 1, Tt, Y, X))
    target = recipe.crandn(105, (B, E, Tt, Y, X))
    y = O.sense_forward(target, maps, mask)
    # HIP (the ReLU decisions of G and of D(pred) captured for the masked float64 check)
    from dl_cs.models import engine
    engine.CAPTURE = []
    try:
        pred = G(y=y.to(DEV), A=T.SenseModel(maps.to(DEV), weights=mask.to(DEV)))
        loss = torch.mean(torch.abs(target.to(DEV) - pred)) + 0.01 * patchgan.g_adv_loss(D(pred))
    finally:
        caps, engine.CAPTURE = engine.CAPTURE, None
    loss.backward()
    d_loss = patchgan.d_loss(D(target.to(DEV)), D(pred.detach()))
    D.zero_grad()
    d_loss.backward()
    # oracle
    sd = {k: v.detach().cpu().clone().requires_grad_(torch.is_floating_point(v) and
                                                     "relative_position_index" not in k and "step_size" not in k)
          for k, v in G.state_dict().items()}
    Pd = {k: v.detach().cpu().clone().requires_grad_() for k, v in D.state_dict().items()}
    po = O.pgd(O.split_unrolls(sd, 1), y, maps, mask)
    lo_adv = F.binary_cross_entropy_with_logits(O.patchgan(Pd, po), torch.ones_like(O.patchgan(Pd, po)))
    lo = torch.mean(torch.abs(target - po)) + 0.01 * lo_adv
    lo.backward()
    assert abs(float(loss) - float(lo)) < 1e-5 * abs(float(lo))
    gnamed = dict(G.named_parameters())
    sdG, sdD = G.state_dict(), D.state_dict()

    def lf(Pg, c, mk):
        Pdc = {k: c(v) for k, v in sdD.items()}
        reg = lambda Pu, xu: O.swinnet(Pu, xu, relu=mk.relu())                # noqa: E731
        po_ = O.pgd(O.split_unrolls(Pg, 1), c(y), c(maps), c(mask), reg=reg)
        lg = O.patchgan(Pdc, po_, relu=mk.relu())
        return torch.mean(torch.abs(c(target) - po_)) + 0.01 * F.binary_cross_entropy_with_logits(
            lg, torch.ones_like(lg))
    tr = lambda k: "relative_position_index" not in k and "step_size" not in k    # noqa: E731
    assert_masked_f64({n: p.grad for n, p in gnamed.items() if p.grad is not None}, lf, sdG, tr, HipMasks(caps),
                      "swin-gan G step", min_tol=H3_GRAD_TOL, factor=H3_FACTOR)
    for v in Pd.values():
        v.grad = None
    lr_, lf_ = O.patchgan(Pd, target), O.patchgan(Pd, po.detach())
    do = (F.binary_cross_entropy_with_logits(lr_, torch.ones_like(lr_)) +
          F.binary_cross_entropy_with_logits(lf_, torch.zeros_like(lf_)))
    do.backward()
    assert abs(float(d_loss) - float(do)) < 1e-5 * abs(float(do))
    # D's parameter gradients held to the fp32 oracle's own distance from a float64
    # evaluation (ReLU decisions within fp32 rounding of 0 flip between summation
    # orders; at the BASELINE slice the first conv's weight gradient sums 0.6 M voxels)
    Pd64 = {k: v.detach().double().requires_grad_() for k, v in Pd.items()}
    c128 = torch.complex128
    l64r, l64f = O.patchgan(Pd64, target.to(c128)), O.patchgan(Pd64, po.detach().to(c128))
    (F.binary_cross_entropy_with_logits(l64r, torch.ones_like(l64r)) +
     F.binary_cross_entropy_with_logits(l64f, torch.zeros_like(l64f))).backward()
    assert_f64_floor({n: p.grad for n, p in D.named_parameters()}, {n: v.grad.double() for n, v in Pd.items()},
                     {n: v.grad for n, v in Pd64.items()}, "swin-gan D step")
