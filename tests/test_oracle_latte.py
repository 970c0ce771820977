"""The Latte oracle (oracle/dit_oracle.py, latte_*) pinned to the reference's own
outputs (tests/golden/latte.npz, made by tests/golden/make_golden.py --only latte
with the timm Mlp restatement -- parity unpinned against timm itself): the 2-D
position and frame tables, LatteNet fwd + bwd (one spatial / temporal block
pair), a non-square grid, and the 2-unroll PGD training step."""
import numpy as np
import pytest
import torch

from goldutil import golden_err, grad_keys
from oracle import dit_oracle as DO
from oracle import dlcs_oracle as O
from oracle import recipe

B, E, C, Tt, Y, X = 1, 2, 8, 4, 32, 32


@pytest.fixture(scope="module")
def tables():
    return DO.latte_pos_table(192), DO.latte_temp_table(192)


def latte_config(n):
    from dl_cs.config import get_cfg
    cfg = get_cfg()
    P = cfg.MODEL.PARAMETERS
    P.NUM_UNROLLS, P.NUM_RESBLOCKS, P.NUM_FEATURES, P.NUM_LAYERS, P.NUM_HEADS = n, 0, 192, 2, 6
    P.NUM_EMAPS, P.SHARE_WEIGHTS, P.FIX_STEP_SIZE, P.LEARN_SIGMA = 2, False, True, False
    P.CONV_BLOCK.COMPLEX, P.CONV_BLOCK.CIRCULAR_PAD = False, True
    return cfg


def _sd(seed, unrolls=None):
    if unrolls is None:
        from dl_cs.models import Latte
        net = Latte.LatteNet(num_blocks=0, in_chans=4, chans=192, kernel_size=3, num_heads=6, num_layers=2)
    else:
        from dl_cs.models import unrolledLatte
        net = unrolledLatte.ProximalGradientDescent(latte_config(unrolls))
    recipe.fill_module(net, seed)
    return net.state_dict()


def _params(sd, dtype=torch.float32):
    frozen = ("pos_embed_table", "temp_embed_table", "step_size")
    return {k: (v.to(dtype).clone().requires_grad_(not any(f in k for f in frozen))
                if torch.is_floating_point(v) else v.clone()) for k, v in sd.items()}


def test_latte_tables(golden, tables):
    g = golden("latte")
    pos, temp = tables
    assert np.array_equal(pos[g["pos_table_rows"]].numpy(), g["pos_table_sample"])
    assert np.array_equal(temp.numpy(), g["temp_table"])
    idx = DO.latte_pos_index(48, 40)
    assert np.array_equal(pos[idx][:, :4].numpy(), g["pos_index_48x40"])
    # the product model's frozen tables are the reference's
    sd = _sd(501)
    assert torch.equal(sd["Latte.pos_embedder.pos_embed_table"][0], pos)
    assert torch.equal(sd["Latte.temp_embedder.temp_embed_table"][0], temp)


def test_latte_schema(golden):
    """LatteNet's state_dict keys are the reference's (recorded gradient names)."""
    g = golden("latte")
    keys = set(grad_keys(g, "latte_"))
    sd = _sd(501)
    assert keys <= set(sd.keys()) and len(keys) > 25
    assert "SFE.layers.2.conv.weight" in sd and "final_layer.layers.2.conv.weight" in sd


def test_latte_fwd_bwd(golden, tables):
    g = golden("latte")
    pos, temp = tables
    P = _params(_sd(501))
    x = recipe.crandn(502, (B, E, Tt, Y, X)).requires_grad_()
    y = DO.latte_net(P, x, torch.tensor([37]), 2, 6, pos_table=pos, temp_table=temp)
    gr = recipe.crandn(503, y.shape)
    (y.real * gr.real + y.imag * gr.imag).sum().backward()
    assert golden_err(g, "latte_y", y) < 1e-5
    assert golden_err(g, "latte_dx", x.grad) < 1e-5
    keys = grad_keys(g, "latte_")
    assert len(keys) > 25
    for k in keys:
        assert golden_err(g, f"latte_grad::{k}", P[k].grad) < 1e-4, k


def test_latte_rect_grid(golden, tables):
    g = golden("latte")
    pos, temp = tables
    P = _params(_sd(504))
    with torch.no_grad():
        y = DO.latte_net(P, recipe.crandn(505, (B, E, Tt, 24, 40)), torch.tensor([37]), 2, 6, pos_table=pos,
                         temp_table=temp)
    assert golden_err(g, "latte_rect_y", y) < 1e-5


def test_latte_pgd2_training_step(golden, tables):
    g = golden("latte")
    pos, temp = tables
    P = _params(_sd(511, unrolls=2))
    maps = recipe.sense_maps(512, B, E, C, Y, X)
    mask = recipe.binary_mask(513, (B, 1, Tt, Y, X))
    yk = recipe.crandn(514, (B, C, Tt, Y, X)) * mask
    target = recipe.crandn(515, (B, E, Tt, Y, X))
    x0 = O.sense_adjoint(yk, maps, mask)
    pred = DO.latte_pgd(DO.split_unrolls(P, 2), x0, torch.tensor([37]), maps, mask, 2, 6, pos_table=pos,
                        temp_table=temp)
    loss = torch.mean(torch.abs(target - pred))
    loss.backward()
    assert golden_err(g, "lattepgd2_pred", pred) < 1e-5
    assert abs(float(loss) - float(g["lattepgd2_loss"])) < 1e-5 * float(g["lattepgd2_loss"])
    for k in grad_keys(g, "lattepgd2_"):
        assert golden_err(g, f"lattepgd2_grad::{k}", P[k].grad) < 1e-3, k
