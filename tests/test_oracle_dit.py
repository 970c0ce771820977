"""The DiT oracle (oracle/dit_oracle.py) pinned to the reference's own outputs
(tests/golden/dit.npz, made by tests/golden/make_golden.py --only dit with the
timm Attention / Mlp restatement -- parity unpinned against timm itself):
embeddings and diffusion constants exactly, DiTResNet / DiTNet fwd + bwd, the
2-unroll PGD training step and the DDPM_X data-consistency step."""
import numpy as np
import pytest
import torch

from goldutil import golden_err, grad_keys
from oracle import dit_oracle as DO
from oracle import dlcs_oracle as O
from oracle import recipe

B, E, C, Tt, Y, X = 1, 2, 8, 4, 32, 32


@pytest.fixture(scope="module")
def table():
    return DO.pos_embed_table(384)


def _sd(cls_name, seed, unrolls=None, arch=None):
    from dl_cs.models import DiT
    if unrolls is None:
        net = getattr(DiT, cls_name)(num_blocks=0, in_chans=4, chans=384, kernel_size=3, num_heads=16, num_layers=2)
        recipe.fill_module(net, seed)
        return net.state_dict()
    from dl_cs.models import unrolledDiT
    m = getattr(unrolledDiT, arch)(dit_config(unrolls))
    recipe.fill_module(m, seed)
    return m.state_dict()


def dit_config(n):
    from dl_cs.config import get_cfg
    cfg = get_cfg()
    P = cfg.MODEL.PARAMETERS
    P.NUM_UNROLLS, P.NUM_RESBLOCKS, P.NUM_FEATURES, P.NUM_LAYERS, P.NUM_HEADS = n, 0, 384, 2, 16
    P.NUM_EMAPS, P.SHARE_WEIGHTS, P.FIX_STEP_SIZE, P.LEARN_SIGMA = 2, False, True, False
    P.CONV_BLOCK.COMPLEX, P.CONV_BLOCK.CIRCULAR_PAD = False, True
    return cfg


def _params(sd, dtype=torch.float32):
    return {k: (v.to(dtype).clone().requires_grad_("pos_embed_table" not in k and "step_size" not in k)
                if torch.is_floating_point(v) else v.clone()) for k, v in sd.items()}


def test_embeddings_and_schedules(golden):
    g = golden("dit")
    t = torch.from_numpy(g["temb_t"])
    assert np.abs(DO.timestep_embedding(t).numpy() - g["temb"]).max() < 1e-6
    for s in ("linear", "squaredcos_cap_v2"):
        ab = DO.alphas_cumprod(s)
        np.testing.assert_allclose(np.sqrt(ab), g[f"sqrt_ab_{s}"], rtol=0, atol=1e-15)
        np.testing.assert_allclose(np.sqrt(1 - ab), g[f"sqrt_1mab_{s}"], rtol=0, atol=1e-15)
    np.testing.assert_array_equal(DO.pos_index((12, 48, 40)), g["pos_index_12x48x40"])


def test_pos_table(golden, table):
    g = golden("dit")
    assert np.array_equal(table[g["pos_table_rows"]].numpy(), g["pos_table_sample"])
    rows = table[torch.from_numpy(DO.pos_index((12, 48, 40)))]
    assert abs(float(rows.double().norm()) - float(g["pos_12x48x40_norm"])) < 1e-9 * float(g["pos_12x48x40_norm"])


@pytest.mark.parametrize("tag,cls,fn", [("ditres", "DiTResNet", DO.dit_resnet), ("ditnet", "DiTNet", DO.dit_net)])
def test_dit_regularizer_fwd_bwd(golden, table, tag, cls, fn):
    g = golden("dit")
    P = _params(_sd(cls, 301))
    x = recipe.crandn(302, (B, E, Tt, Y, X)).requires_grad_()
    y = fn(P, x, torch.tensor([37]), torch.tensor([1]), 2, 16, pos_table=table)
    gr = recipe.crandn(303, y.shape)
    (y.real * gr.real + y.imag * gr.imag).sum().backward()
    assert golden_err(g, f"{tag}_y", y) < 1e-5
    assert golden_err(g, f"{tag}_dx", x.grad) < 1e-5
    keys = grad_keys(g, f"{tag}_")
    assert len(keys) > 20
    for k in keys:
        assert golden_err(g, f"{tag}_grad::{k}", P[k].grad) < 1e-4, k


def test_dit_pgd2_training_step(golden, table):
    g = golden("dit")
    P = _params(_sd(None, 311, unrolls=2, arch="ProximalGradientDescent"))
    maps = recipe.sense_maps(312, B, E, C, Y, X)
    mask = recipe.binary_mask(313, (B, 1, Tt, Y, X))
    yk = recipe.crandn(314, (B, C, Tt, Y, X)) * mask
    target = recipe.crandn(315, (B, E, Tt, Y, X))
    x0 = O.sense_adjoint(yk, maps, mask)
    pred = DO.pgd(DO.split_unrolls(P, 2), x0, torch.tensor([37]), torch.tensor([1]), maps, mask, 2, 16,
                  pos_table=table)
    loss = torch.mean(torch.abs(target - pred))
    loss.backward()
    assert golden_err(g, "ditpgd2_pred", pred) < 1e-5
    assert abs(float(loss) - float(g["ditpgd2_loss"])) < 1e-5 * float(g["ditpgd2_loss"])
    for k in grad_keys(g, "ditpgd2_"):
        assert golden_err(g, f"ditpgd2_grad::{k}", P[k].grad) < 1e-3, k


def test_dit_ddpm_x_kspace_loss(golden, table):
    g = golden("dit")
    P = _params(_sd(None, 321, unrolls=2, arch="DataConsistency"))
    maps = recipe.sense_maps(312, B, E, C, Y, X)
    mask_p = recipe.binary_mask(322, (B, 1, Tt, Y, X))
    target = recipe.crandn(323, (B, E, Tt, Y, X))
    noise = recipe.randn(324, (B, 2 * E, Tt, Y, X))
    t = torch.tensor([613])
    Ps = DO.split_unrolls(P, 2)
    model = lambda xt: DO.data_consistency(Ps, xt, t, torch.tensor([1]), maps, mask_p, 2, 16, pos_table=table)  # noqa
    loss, out, x_t = DO.training_kspace_loss(model, target, t, maps, target, noise)
    loss.backward()
    assert golden_err(g, "ditdc2_xt", x_t) < 1e-6
    assert golden_err(g, "ditdc2_pred", out) < 1e-5
    assert abs(float(loss) - float(g["ditdc2_loss"])) < 1e-5 * float(g["ditdc2_loss"])
    for k in grad_keys(g, "ditdc2_"):
        assert golden_err(g, f"ditdc2_grad::{k}", P[k].grad) < 1e-3, k
