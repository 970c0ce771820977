"""HIP Latte denoiser path (BASELINE config 5, config_latte.yaml; lat =
dl_cs/models/Latte.py, ulat = dl_cs/models/unrolledLatte.py) vs the reference
goldens (tests/golden/latte.npz) and the fp32 / float64 oracle
(oracle/dit_oracle.py latte_*).

Tolerances (fp32 build): outputs vs the reference goldens <= 1e-5; input and
parameter gradients held to the float64 floor (goldutil.assert_f64_floor: NRMSE
vs a float64 oracle <= max(1e-5, 4 x the fp32 oracle's own NRMSE vs float64) --
LatteNet's forward has no ReLU, so no decisions need pinning); the fp8
inference path within its stated budget."""
import pytest
import torch

from goldutil import assert_f64_floor, golden_err, grad_keys, nrmse, oracle_grads
from oracle import dit_oracle as DO
from oracle import dlcs_oracle as O
from oracle import recipe

pytestmark = pytest.mark.gpu
DEV = "cuda"
B, E, C, Tt, Y, X = 1, 2, 8, 4, 32, 32
FROZEN = ("pos_embed_table", "temp_embed_table", "step_size")


def _tr(k):
    return not any(f in k for f in FROZEN)


@pytest.fixture(scope="module")
def tables():
    return DO.latte_pos_table(192), DO.latte_temp_table(192)


def _net(seed, D=192, heads=6, layers=2):
    from dl_cs.models import Latte
    net = Latte.LatteNet(num_blocks=0, in_chans=4, chans=D, kernel_size=3, num_heads=heads, num_layers=layers)
    net.eval()
    recipe.fill_module(net, seed)
    return net.to(DEV)


def test_latte_vs_reference(golden, tables):
    """LatteNet (one spatial / temporal pair, 192 features, 6 heads) fwd + bwd:
    output vs the reference; input and parameter gradients at the float64 floor."""
    g = golden("latte")
    pos, temp = tables
    net = _net(501)
    x = recipe.crandn(502, (B, E, Tt, Y, X))
    xg = x.to(DEV).requires_grad_()
    t, lab = torch.tensor([37]), torch.tensor([1])
    y = net(xg, t.to(DEV), lab.to(DEV))
    gr = recipe.crandn(503, y.shape)
    (y.real * gr.real.to(DEV) + y.imag * gr.imag.to(DEV)).sum().backward()
    assert golden_err(g, "latte_y", y) < 1e-5
    assert golden_err(g, "latte_dx", xg.grad) < 1e-5
    named = dict(net.named_parameters())
    keys = grad_keys(g, "latte_")
    assert set(keys) <= set(named)
    for k in keys:
        assert golden_err(g, f"latte_grad::{k}", named[k].grad) < 1e-4, k
    xkey = "__x__"
    sd = dict(net.state_dict())
    sd[xkey] = x

    def lf(P, c):
        dt = P["Latte.t_embedder.mlp.0.weight"].dtype
        yo = DO.latte_net(P, P[xkey], t, 2, 6, pos_table=pos.to(dt), temp_table=temp.to(dt))
        gc = c(gr)
        return (yo.real * gc.real + yo.imag * gc.imag).sum()
    hip = {n: p.grad for n, p in named.items() if p.grad is not None and _tr(n)}
    hip[xkey] = xg.grad
    o32, o64 = (oracle_grads(lf, sd, dt, _tr) for dt in (torch.float32, torch.float64))
    assert_f64_floor(hip, o32, o64, "latte")


def test_latte_rect_grid(golden):
    """A non-square grid (24 x 40: 6 x 10 patches) -- the position index binds its
    loop variables crosswise (lat:183)."""
    g = golden("latte")
    net = _net(504)
    with torch.no_grad():
        y = net(recipe.crandn(505, (B, E, Tt, 24, 40)).to(DEV), torch.tensor([37]).to(DEV), torch.tensor([1]).to(DEV))
    assert golden_err(g, "latte_rect_y", y) < 1e-5


def test_latte_pgd2_training_step(golden, tables):
    """unrolledLatte.ProximalGradientDescent (ulat:233-265), 2 unrolls, x0 = A^H y,
    complex-L1 loss: prediction, loss and gradients vs the reference."""
    from dl_cs.models import unrolledLatte
    from dl_cs.mri import transforms as T
    from test_oracle_latte import latte_config
    g = golden("latte")
    model = unrolledLatte.ProximalGradientDescent(latte_config(2))
    model.eval()
    recipe.fill_module(model, 511)
    model = model.to(DEV)
    maps = recipe.sense_maps(512, B, E, C, Y, X)
    mask = recipe.binary_mask(513, (B, 1, Tt, Y, X))
    yk = recipe.crandn(514, (B, C, Tt, Y, X)) * mask
    target = recipe.crandn(515, (B, E, Tt, Y, X))
    t, lab = torch.tensor([37]), torch.tensor([1])
    A = T.SenseModel(maps.to(DEV), weights=mask.to(DEV))
    x0 = A(yk.to(DEV), adjoint=True)
    pred = model(x0, t.to(DEV), A, lab.to(DEV))
    loss = torch.mean(torch.abs(target.to(DEV) - pred))
    loss.backward()
    assert golden_err(g, "lattepgd2_pred", pred) < 1e-5
    assert abs(float(loss) - float(g["lattepgd2_loss"])) < 1e-5 * float(g["lattepgd2_loss"])
    named = dict(model.named_parameters())
    for k in grad_keys(g, "lattepgd2_"):
        assert golden_err(g, f"lattepgd2_grad::{k}", named[k].grad) < 1e-3, k
    pos, temp = DO.latte_pos_table(192), DO.latte_temp_table(192)

    def lf(P, c):
        dt = P["step_size"].dtype
        xo = O.sense_adjoint(c(yk), c(maps), c(mask))
        po = DO.latte_pgd(DO.split_unrolls(P, 2), xo, t, c(maps), c(mask), 2, 6, pos_table=pos.to(dt),
                          temp_table=temp.to(dt))
        return torch.mean(torch.abs(c(target) - po))
    o32, o64 = (oracle_grads(lf, model.state_dict(), dt, _tr) for dt in (torch.float32, torch.float64))
    assert_f64_floor({n: p.grad for n, p in named.items() if p.grad is not None and _tr(n)}, o32, o64,
                     "latte pgd2")


def test_latte_full_slice_forward(tables):
    """LatteNet at the BASELINE slice (T = 20 -> 24 padded frames, 192 x 160: 1,920
    patches per frame -- spatial attention over 1,920 tokens, temporal over 24),
    config_latte widths (192 features, 6 heads), 2 layers, eval forward vs the
    fp32 oracle; then the fp8 inference path within its budget (5e-2)."""
    from dl_cs.models import dit_engine
    pos, temp = tables
    net = _net(521)
    x = recipe.crandn(522, (1, 2, 20, 192, 160))
    t, lab = torch.tensor([500]), torch.tensor([1])
    with torch.no_grad():
        y = net(x.to(DEV), t.to(DEV), lab.to(DEV)).cpu()
        P = {k: v.detach().cpu() for k, v in net.state_dict().items()}
        ref = DO.latte_net(P, x, t, 2, 6, pos_table=pos, temp_table=temp)
        err = nrmse(ref.numpy(), y.numpy())
        dit_engine.set_fp8(True)
        try:
            y8 = net(x.to(DEV), t.to(DEV), lab.to(DEV)).cpu()
        finally:
            dit_engine.set_fp8(False)
    err8 = nrmse(ref.numpy(), y8.numpy())
    print(f"full-slice LatteNet fwd NRMSE vs oracle {err:.3g}; fp8 inference {err8:.3g}")
    assert err < 1e-5 and err8 < 5e-2
