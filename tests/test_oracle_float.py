"""Oracle pin: fp32 restatement vs goldens produced by the reference itself.

Tolerance: NRMSE <= 1e-5 (fp32 noise floor 3.5e-7 at 10 unrolls);
the only differences are summation order inside conv / GEMM / FFT libraries.
"""
import numpy as np
import pytest
import torch

from goldutil import golden_err, grad_keys
from oracle import dlcs_oracle as O
from oracle import recipe, windex

TOL = 1e-5


@pytest.mark.parametrize("tag", ["small", "mid"])
def test_sense(golden, tag):
    g = golden("sense")
    B, E, C, T, Y, X = (int(v) for v in g[f"shape_{tag}"])
    maps = recipe.sense_maps(11, B, E, C, Y, X)
    w = recipe.binary_mask(12, (B, 1, T, Y, X))
    x = recipe.crandn(13, (B, E, T, Y, X))
    y = recipe.crandn(14, (B, C, T, Y, X))
    assert golden_err(g, f"fwd_{tag}", O.sense_forward(x, maps, w)) < TOL
    assert golden_err(g, f"adj_{tag}", O.sense_adjoint(y, maps, w)) < TOL
    assert golden_err(g, f"fwd_nomask_{tag}", O.sense_forward(x, maps, None)) < TOL


def _check_grads(g, prefix, P, grads, tol=1e-4):
    names = grad_keys(g, prefix)
    assert names
    for name in names:
        assert name in grads and grads[name] is not None, name
        assert golden_err(g, f"{prefix}grad::{name}", grads[name]) < tol, name


def _leaf_params(sd, prefix=""):
    P = {}
    for k, v in sd.items():
        t = v.clone()
        if torch.is_floating_point(t) and "relative_position_index" not in k:
            t.requires_grad_()
        P[k] = t
    return P


def test_window_attention(golden):
    g = golden("blocks")
    keys = {"qkv.weight": (480, 160), "qkv.bias": (480,), "proj.weight": (160, 160),
            "proj.bias": (160,), "relative_position_bias_table": (2925, 8)}
    mask = torch.from_numpy(windex.compute_mask(7, 8, 16, (7, 8, 8), (0, 0, 4)))
    for tag, m in (("mask", mask), ("nomask", None)):
        P = {k: recipe.param_value(21, k, s).requires_grad_() for k, s in keys.items()}
        x = recipe.randn(22, (2, 448, 160)).requires_grad_()
        dy = recipe.randn(23, (2, 448, 160))
        y = O.window_attention(P, "", x, m, 8, (7, 8, 8))
        (y * dy).sum().backward()
        assert golden_err(g, f"attn_{tag}_y", y.detach()) < TOL
        assert golden_err(g, f"attn_{tag}_dx", x.grad) < TOL
        _check_grads(g, f"attn_{tag}_", P, {k: v.grad for k, v in P.items()})


def test_mlp(golden):
    g = golden("blocks")
    keys = {"fc1.weight": (640, 160), "fc1.bias": (640,), "fc2.weight": (160, 640), "fc2.bias": (160,)}
    P = {k: recipe.param_value(24, k, s).requires_grad_() for k, s in keys.items()}
    x = recipe.randn(25, (896, 160)).requires_grad_()
    dy = recipe.randn(26, (896, 160))
    y = O.mlp(P, "", x)
    (y * dy).sum().backward()
    assert golden_err(g, "mlp_y", y.detach()) < TOL
    assert golden_err(g, "mlp_dx", x.grad) < TOL
    _check_grads(g, "mlp_", P, {k: v.grad for k, v in P.items()})


BLOCK_KEYS = {"norm1.weight": (160,), "norm1.bias": (160,),
              "attn.relative_position_bias_table": (2925, 8),
              "attn.qkv.weight": (480, 160), "attn.qkv.bias": (480,),
              "attn.proj.weight": (160, 160), "attn.proj.bias": (160,),
              "norm2.weight": (160,), "norm2.bias": (160,),
              "mlp.fc1.weight": (640, 160), "mlp.fc1.bias": (640,),
              "mlp.fc2.weight": (160, 640), "mlp.fc2.bias": (160,)}


@pytest.mark.parametrize("tag,grid", [("blk", (7, 16, 16)), ("blkpad", (7, 12, 10))])
def test_swin_block(golden, tag, grid):
    g = golden("blocks")
    P = {k: recipe.param_value(27, k, s).requires_grad_() for k, s in BLOCK_KEYS.items()}
    ws, ss = windex.get_window_size(grid, (7, 8, 8), (3, 4, 4))
    Dp, Hp, Wp = windex.padded_grid(*grid, ws)
    m = torch.from_numpy(windex.compute_mask(Dp, Hp, Wp, ws, ss))
    x = recipe.randn(28, (1,) + grid + (160,)).requires_grad_()
    dy = recipe.randn(29, (1,) + grid + (160,))
    y = O.swin_block(P, "", x, (3, 4, 4), m, 8, (7, 8, 8))
    (y * dy).sum().backward()
    assert golden_err(g, f"{tag}_y", y.detach()) < TOL
    assert golden_err(g, f"{tag}_dx", x.grad) < TOL
    _check_grads(g, f"{tag}_", P, {k: v.grad for k, v in P.items()})


def swinnet_state(seed, num_swinblocks=1):
    """Recipe-filled parameter dict for SwinTransformer3DNet (reference keys)."""
    from oracle.shapes import swinnet_param_shapes
    sd = {}
    for k, s in swinnet_param_shapes(num_swinblocks=num_swinblocks).items():
        sd[k] = recipe.param_value(seed, k, s)
    return sd


def test_swinnet_forward_backward(golden):
    g = golden("swinnet")
    torch.set_num_threads(8)
    P = _leaf_params(swinnet_state(31))
    x = recipe.crandn(32, (1, 2, 20, 32, 32)).requires_grad_()
    y = O.swinnet(P, x)
    assert golden_err(g, "net32_y", y.detach()) < TOL
    gr = recipe.crandn(33, y.shape)
    (y.real * gr.real + y.imag * gr.imag).sum().backward()
    assert golden_err(g, "net32_dx", x.grad) < TOL
    _check_grads(g, "net32_", P, {k: v.grad for k, v in P.items() if v.requires_grad})


def test_swinnet_two_swinblocks(golden):
    """NUM_SWINBLOCKS = 2 (defaults.py:34; s3d:347-357, pad 6 at s3d:380) vs the
    reference run (tests/golden/make_golden.py::gen_swinnet, nb2_*)."""
    g = golden("swinnet")
    torch.set_num_threads(8)
    P = _leaf_params(swinnet_state(34, 2))
    x = recipe.crandn(35, (1, 2, 20, 32, 32)).requires_grad_()
    y = O.swinnet(P, x, num_swinblocks=2)
    assert golden_err(g, "nb2_y", y.detach()) < TOL
    gr = recipe.crandn(36, y.shape)
    (y.real * gr.real + y.imag * gr.imag).sum().backward()
    assert golden_err(g, "nb2_dx", x.grad) < TOL
    _check_grads(g, "nb2_", P, {k: v.grad for k, v in P.items() if v.requires_grad})


@pytest.mark.slow
def test_swinnet_padded_grid(golden):
    g = golden("swinnet")
    P = swinnet_state(31)
    with torch.no_grad():
        y = O.swinnet(P, recipe.crandn(32, (1, 2, 20, 48, 40)))
    assert golden_err(g, "net4840_y", y) < TOL


def test_pgd2_loss_and_grads(golden):
    g = golden("pgd")
    from oracle.shapes import swinnet_param_shapes
    torch.set_num_threads(8)
    B, E, C, T, Y, X = 1, 2, 8, 20, 32, 32
    Ps = []
    for i in range(2):
        Ps.append(_leaf_params({k: recipe.param_value(41, f"cnn_update.{i}.{k}", s)
                                for k, s in swinnet_param_shapes().items()}))
    maps = recipe.sense_maps(42, B, E, C, Y, X)
    mask = recipe.binary_mask(43, (B, 1, T, Y, X))
    y = recipe.crandn(44, (B, C, T, Y, X)) * mask
    target = recipe.crandn(45, (B, E, T, Y, X))
    pred = O.pgd(Ps, y, maps, mask)
    loss = O.l1(target, pred)
    loss.backward()
    assert golden_err(g, "pgd2_pred", pred.detach()) < TOL
    assert abs(float(loss.detach()) - float(g["pgd2_loss"])) < 1e-5 * float(g["pgd2_loss"])
    grads = {}
    for i, P in enumerate(Ps):
        for k, v in P.items():
            if v.requires_grad and v.grad is not None:
                grads[f"cnn_update.{i}.{k}"] = v.grad
    _check_grads(g, "pgd2_", None, grads, tol=1e-3)


def test_hqs2_loss_and_grads(golden):
    """HQS / MoDL (urs:125-172, alg:11-73) restatement vs the reference: 2 unrolls
    x 10 CG steps, learnable lamda."""
    g = golden("hqs")
    from oracle.shapes import swinnet_param_shapes
    torch.set_num_threads(8)
    B, E, C, T, Y, X = 1, 2, 8, 20, 32, 32
    Ps = []
    for i in range(2):
        Ps.append(_leaf_params({k: recipe.param_value(61, f"cnn_update.{i}.{k}", s)
                                for k, s in swinnet_param_shapes().items()}))
    lamda = torch.tensor([0.1], requires_grad=True)
    maps = recipe.sense_maps(62, B, E, C, Y, X)
    mask = recipe.binary_mask(63, (B, 1, T, Y, X))
    y = recipe.crandn(64, (B, C, T, Y, X)) * mask
    target = recipe.crandn(65, (B, E, T, Y, X))
    pred = O.hqs(Ps, y, maps, mask, lamda=lamda)
    loss = O.l1(target, pred)
    loss.backward()
    assert golden_err(g, "hqs2_pred", pred.detach()) < TOL
    assert abs(float(loss.detach()) - float(g["hqs2_loss"])) < 1e-5 * float(g["hqs2_loss"])
    assert abs(float(lamda.grad) - float(g["hqs2_lamda_grad"][0])) < 1e-3 * abs(float(g["hqs2_lamda_grad"][0]))
    grads = {"lamda": lamda.grad}
    for i, P in enumerate(Ps):
        for k, v in P.items():
            if v.requires_grad and v.grad is not None:
                grads[f"cnn_update.{i}.{k}"] = v.grad
    _check_grads(g, "hqs2_", None, grads, tol=1e-3)


def test_resnet_pgd2_loss_and_grads(golden):
    """The "dlespirit" unrolled ResNet (BASELINE config 1; ur:69-122, r3d:243-317)
    restatement vs the reference: prediction, loss, parameter gradients."""
    g = golden("resnet")
    torch.set_num_threads(8)
    B, E, C, T, Y, X = 1, 1, 8, 20, 32, 32
    names = sorted({k.split("grad::")[1].split("@")[0] for k in g if k.startswith("res2_grad::")})
    Ps = []
    for i in range(2):
        pre = f"cnn_update.{i}."
        shapes = {n[len(pre):]: tuple(g[f"res2_grad::{n}"].shape) if f"res2_grad::{n}" in g
                  else tuple(g[f"res2_grad::{n}@shape"]) for n in names if n.startswith(pre)}
        Ps.append(_leaf_params({k: recipe.param_value(81, pre + k, s) for k, s in shapes.items()}))
    maps = recipe.sense_maps(82, B, E, C, Y, X)
    mask = recipe.binary_mask(83, (B, 1, T, Y, X))
    y = recipe.crandn(84, (B, C, T, Y, X)) * mask
    target = recipe.crandn(85, (B, E, T, Y, X))
    pred = O.pgd(Ps, y, maps, mask, reg=O.resnet)
    loss = O.l1(target, pred)
    loss.backward()
    assert golden_err(g, "res2_pred", pred.detach()) < TOL
    assert abs(float(loss.detach()) - float(g["res2_loss"])) < 1e-5 * float(g["res2_loss"])
    grads = {}
    for i, P in enumerate(Ps):
        for k, v in P.items():
            if v.requires_grad and v.grad is not None:
                grads[f"cnn_update.{i}.{k}"] = v.grad
    _check_grads(g, "res2_", None, grads, tol=1e-3)


def test_metrics(golden):
    g = golden("misc")
    ref = recipe.crandn(61, (1, 2, 4, 8, 8))
    pred = ref + 0.1 * recipe.crandn(62, (1, 2, 4, 8, 8))
    assert abs(float(O.l1(ref, pred)) - float(g["metric_l1"])) < 1e-6
    assert abs(float(O.l2(ref, pred)) - float(g["metric_l2"])) < 1e-6
    assert abs(float(O.psnr(ref, pred)) - float(g["metric_psnr"])) < 1e-4
