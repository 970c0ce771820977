"""HIP SENSE operator vs the oracle / goldens (tr:12-110).  Tolerance NRMSE <= 1e-5."""
import numpy as np
import pytest
import torch

from goldutil import golden_err, nrmse
from oracle import dlcs_oracle as O
from oracle import recipe

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = "cuda"


def _T():
    from dl_cs.mri import transforms as T
    return T


@pytest.mark.parametrize("tag", ["small", "mid"])
def test_sense_golden(golden, tag):
    T = _T()
    g = golden("sense")
    B, E, C, Tt, Y, X = (int(v) for v in g[f"shape_{tag}"])
    maps = recipe.sense_maps(11, B, E, C, Y, X)
    w = recipe.binary_mask(12, (B, 1, Tt, Y, X))
    x = recipe.crandn(13, (B, E, Tt, Y, X))
    y = recipe.crandn(14, (B, C, Tt, Y, X))
    A = T.SenseModel(maps.to(DEV), weights=w.to(DEV))
    assert golden_err(g, f"fwd_{tag}", A(x.to(DEV)).cpu()) < TOL
    assert golden_err(g, f"adj_{tag}", A(y.to(DEV), adjoint=True).cpu()) < TOL
    A1 = T.SenseModel(maps.to(DEV))
    assert golden_err(g, f"fwd_nomask_{tag}", A1(x.to(DEV)).cpu()) < TOL


@pytest.mark.parametrize("shape", [(1, 2, 8, 20, 192, 160), (1, 2, 8, 4, 192, 64), (2, 1, 3, 2, 30, 50)])
def test_sense_full_size_vs_oracle(shape):
    T = _T()
    B, E, C, Tt, Y, X = shape
    maps = recipe.sense_maps(1, B, E, C, Y, X)
    w = recipe.binary_mask(2, (B, 1, Tt, Y, X))
    x = recipe.crandn(3, (B, E, Tt, Y, X))
    y = recipe.crandn(4, (B, C, Tt, Y, X))
    A = T.SenseModel(maps.to(DEV), weights=w.to(DEV))
    assert nrmse(O.sense_forward(x, maps, w).numpy(), A(x.to(DEV)).cpu().numpy()) < TOL
    assert nrmse(O.sense_adjoint(y, maps, w).numpy(), A(y.to(DEV), adjoint=True).cpu().numpy()) < TOL


def test_adjointness():
    T = _T()
    B, E, C, Tt, Y, X = 1, 2, 8, 6, 192, 160
    maps = recipe.sense_maps(5, B, E, C, Y, X).to(DEV)
    w = recipe.binary_mask(6, (B, 1, Tt, Y, X)).to(DEV)
    A = T.SenseModel(maps, weights=w)
    x = recipe.crandn(7, (B, E, Tt, Y, X)).to(DEV)
    y = recipe.crandn(8, (B, C, Tt, Y, X)).to(DEV)
    lhs = torch.vdot(A(x).reshape(-1).to(torch.complex128), y.reshape(-1).to(torch.complex128))
    rhs = torch.vdot(x.reshape(-1).to(torch.complex128), A(y, adjoint=True).reshape(-1).to(torch.complex128))
    assert abs(complex(lhs - rhs)) <= 1e-5 * abs(complex(lhs))


@pytest.mark.parametrize("Y,X", [(192, 160), (160, 192), (80, 96), (50, 64), (20, 24), (48, 40), (64, 64), (1, 5), (27, 125)])
def test_fft2_vs_numpy(Y, X):
    T = _T()
    x = recipe.crandn(9, (3, Y, X))
    F = T.FFT(2)
    out = F(x.to(DEV)).cpu().numpy()
    ref = np.fft.fftn(x.numpy().astype(np.complex128), axes=(-1, -2), norm="ortho")
    assert nrmse(ref, out) < 2e-6
    inv = F(x.to(DEV), adjoint=True).cpu().numpy()
    refi = np.fft.ifftn(x.numpy().astype(np.complex128), axes=(-1, -2), norm="ortho")
    assert nrmse(refi, inv) < 2e-6


# (96, 80) and (64, 128) take the wave-per-line fast kernels (3 and 10 coils:
# fewer coils than row-pass waves, and more); (48, 40) the generic ones
@pytest.mark.parametrize("C,Y,X", [(8, 48, 40), (3, 96, 80), (10, 64, 128)])
def test_normal_dc_and_grad(C, Y, X):
    T = _T()
    B, E, Tt = 1, 2, 4
    maps = recipe.sense_maps(15, B, E, C, Y, X)
    w = recipe.binary_mask(16, (B, 1, Tt, Y, X))
    x = recipe.crandn(17, (B, E, Tt, Y, X))
    aty = recipe.crandn(18, (B, E, Tt, Y, X))
    ref = x + (-2.0) * (O.sense_adjoint(O.sense_forward(x, maps, w), maps, w) - aty)
    A = T.SenseModel(maps.to(DEV), weights=w.to(DEV))
    xg = x.to(DEV).requires_grad_()
    out = A.normal_dc(xg, aty.to(DEV), -2.0)
    assert nrmse(ref.numpy(), out.detach().cpu().numpy()) < TOL
    # gradient vs autograd through the oracle
    g = recipe.crandn(19, out.shape)
    (out.real * g.real.to(DEV) + out.imag * g.imag.to(DEV)).sum().backward()
    xo = x.clone().requires_grad_()
    refo = xo + (-2.0) * (O.sense_adjoint(O.sense_forward(xo, maps, w), maps, w) - aty)
    (refo.real * g.real + refo.imag * g.imag).sum().backward()
    assert nrmse(xo.grad.numpy(), xg.grad.cpu().numpy()) < TOL


def test_sense_autograd_matches_oracle():
    T = _T()
    B, E, C, Tt, Y, X = 1, 2, 4, 3, 24, 20
    maps = recipe.sense_maps(20, B, E, C, Y, X)
    w = recipe.binary_mask(21, (B, 1, Tt, Y, X))
    x = recipe.crandn(22, (B, E, Tt, Y, X))
    g = recipe.crandn(23, (B, E, Tt, Y, X))
    A = T.SenseModel(maps.to(DEV), weights=w.to(DEV))
    xg = x.to(DEV).requires_grad_()
    o = A(A(xg), adjoint=True)
    (o.real * g.real.to(DEV) + o.imag * g.imag.to(DEV)).sum().backward()
    xo = x.clone().requires_grad_()
    oo = O.sense_adjoint(O.sense_forward(xo, maps, w), maps, w)
    (oo.real * g.real + oo.imag * g.imag).sum().backward()
    assert nrmse(xo.grad.numpy(), xg.grad.cpu().numpy()) < TOL


def test_mixed_devices_raise_and_host_path_agrees():
    """CPU tensors take the explicit host path (DataLoader workers, pp:140-164),
    GPU tensors the HIP kernels; mixing the two raises instead of copying."""
    T = _T()
    maps = recipe.sense_maps(1, 1, 2, 3, 8, 8)
    mask = recipe.binary_mask(3, (1, 1, 2, 8, 8))
    x = recipe.crandn(2, (1, 2, 2, 8, 8))
    with pytest.raises(RuntimeError):
        T.SenseModel(maps.cuda(), weights=mask.cuda())(x)
    host = T.SenseModel(maps, weights=mask)(x)
    dev = T.SenseModel(maps.cuda(), weights=mask.cuda())(x.cuda())
    assert nrmse(host.numpy(), dev.cpu().numpy()) < 1e-6


@pytest.mark.parametrize("shape", [(1, 2, 8, 20, 192, 160), (1, 2, 8, 4, 32, 32), (2, 1, 3, 2, 30, 50)])
@pytest.mark.parametrize("weighted", [True, False])
def test_sense_normal_vs_oracle(shape, weighted):
    """dlcs_sense_normal: base_scale * x + step * (A^H A x - sub) in both uses
    (PGD DC: 1, s, ATy; HQS: lamda, 1, None); fast path (fused column pass) and
    the generic sizes (30 x 50)."""
    T = _T()
    B, E, C, Tt, Y, X = shape
    maps = recipe.sense_maps(21, B, E, C, Y, X)
    w = recipe.binary_mask(22, (B, 1, Tt, Y, X)) * (1.0 + recipe.crandn(25, (B, 1, Tt, Y, X)).real.abs()) \
        if weighted else None
    x = recipe.crandn(23, (B, E, Tt, Y, X))
    sub = recipe.crandn(24, (B, E, Tt, Y, X))
    AhA = O.sense_adjoint(O.sense_forward(x, maps, w), maps, w)
    wd = w.to(DEV) if w is not None else None
    out = T.sense_normal_raw(x.to(DEV), maps.to(DEV), wd, sub=sub.to(DEV), base_scale=1.0, step=-2.0)
    assert nrmse((x - 2.0 * (AhA - sub)).numpy(), out.cpu().numpy()) < TOL
    out = T.sense_normal_raw(x.to(DEV), maps.to(DEV), wd, sub=None, base_scale=0.1, step=1.0)
    assert nrmse((AhA + 0.1 * x).numpy(), out.cpu().numpy()) < TOL


@pytest.mark.parametrize("shape", [(1, 2, 8, 20, 192, 160), (1, 2, 8, 4, 32, 32), (2, 1, 3, 2, 30, 50)])
def test_sense_cg_vs_oracle(shape):
    """dlcs_sense_cg: 10 device-resident CG steps (alg:50-73) on the HQS normal
    equations vs the oracle's CG loop; the reference's own 10-step CG on these
    operands is matched by the HQS goldens (test_gpu_swin.py::test_hqs*)."""
    T = _T()
    B, E, C, Tt, Y, X = shape
    maps = recipe.sense_maps(31, B, E, C, Y, X)
    w = recipe.binary_mask(32, (B, 1, Tt, Y, X))
    x0 = recipe.crandn(33, (B, E, Tt, Y, X))
    b = recipe.crandn(34, (B, E, Tt, Y, X))
    lam = 0.1
    normal = lambda m: O.sense_adjoint(O.sense_forward(m, maps, w), maps, w) + lam * m
    ref = O.conjugate_gradient(normal, x0, b, 10)
    A = T.SenseModel(maps.to(DEV), weights=w.to(DEV))
    out = A.cg(x0.to(DEV), b.to(DEV), lam, 10)
    assert nrmse(ref.numpy(), out.cpu().numpy()) < TOL
    # num_iter = 0 returns x unchanged
    assert torch.equal(A.cg(x0.to(DEV), b.to(DEV), lam, 0).cpu(), x0)


def _vdkt_mask():
    """The reference's VDkt cine mask (subsample.py, seed 1000) at the BASELINE
    slice, from the committed golden bits: [1, 1, 20, 192, 160]."""
    g = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "misc.npz"))
    sh = tuple(int(v) for v in g["vdkt_seed1000_shape"])
    m = np.unpackbits(g["vdkt_seed1000_bits"])[: int(np.prod(sh))].reshape(sh)
    return torch.from_numpy(m.astype(np.float32))


def _row_sparse_mask(seed, shape, frac=0.1, empty_frame=None):
    """Random line-sparse weights: per (b, w, t) a random subset of ky lines, each
    with its own random non-negative x profile (non-separable), optionally one
    frame with no line at all."""
    gen = torch.Generator().manual_seed(seed)
    B, Wc, Tt, Y, X = shape
    lines = (torch.rand((B, Wc, Tt, Y, 1), generator=gen) < frac).float()
    prof = torch.rand((B, Wc, Tt, Y, X), generator=gen) * (torch.rand((B, Wc, Tt, Y, X), generator=gen) < 0.8)
    w = lines * (0.5 + prof)
    if empty_frame is not None:
        w[:, :, empty_frame] = 0
    return w


@pytest.mark.parametrize("kind", ["vdkt", "sparse", "coil", "empty"])
def test_sense_normal_rows_vs_oracle(kind):
    """dlcs_sense_normal_rows (the row-sparse normal operator) vs the oracle's
    A^H (W^2 (A x)) on the reference's VDkt mask at the BASELINE slice, random
    line-sparse non-separable weights, per-coil weights (Wc = C) and an
    all-empty mask / empty frames; also against the dense three-launch operator."""
    T = _T()
    if kind == "vdkt":
        B, E, C, Tt, Y, X = 1, 2, 8, 20, 192, 160
        w = _vdkt_mask()
    elif kind == "sparse":
        B, E, C, Tt, Y, X = 2, 2, 4, 3, 96, 80
        w = _row_sparse_mask(41, (B, 1, Tt, Y, X), empty_frame=1)
    elif kind == "coil":
        B, E, C, Tt, Y, X = 1, 1, 6, 2, 64, 128
        w = _row_sparse_mask(42, (B, C, Tt, Y, X), frac=0.2)
    else:
        B, E, C, Tt, Y, X = 1, 2, 4, 2, 160, 192
        w = torch.zeros((B, 1, Tt, Y, X))
    maps = recipe.sense_maps(43, B, E, C, Y, X)
    x = recipe.crandn(44, (B, E, Tt, Y, X))
    sub = recipe.crandn(45, (B, E, Tt, Y, X))
    AhA = O.sense_adjoint(O.sense_forward(x, maps, w), maps, w)
    wd = w.to(DEV)
    # a mask's first use reads nothing back (row capacity Y); its second use reads the line counts once
    tab, jmax, lines = T._rowtab(wd, wd.contiguous(), w.shape[1], B, Tt, Y, X)
    assert jmax is None and lines is None
    tab, jmax, lines = T._rowtab(wd, wd.contiguous(), w.shape[1], B, Tt, Y, X)
    assert jmax == int((w.abs().sum(-1) > 0).sum(-1).max()) and lines == int((w.abs().sum(-1) > 0).sum())
    out = T.sense_normal_raw(x.to(DEV), maps.to(DEV), wd, sub=sub.to(DEV), base_scale=1.0, step=-2.0)
    ref = (x - 2.0 * (AhA - sub)).numpy()
    assert nrmse(ref, out.cpu().numpy()) < TOL
    # a fresh mask tensor (first use, capacity Y): the same result
    out_y = T.sense_normal_raw(x.to(DEV), maps.to(DEV), wd.clone(), sub=sub.to(DEV), base_scale=1.0, step=-2.0)
    assert nrmse(out.cpu().numpy(), out_y.cpu().numpy()) < 1e-6
    out2 = T.sense_normal_raw(x.to(DEV), maps.to(DEV), wd, sub=None, base_scale=0.1, step=1.0)
    assert nrmse((AhA + 0.1 * x).numpy(), out2.cpu().numpy()) < TOL
    import os
    os.environ["DLCS_SENSE_ROWS"] = "0"
    os.environ["DLCS_DIAG"] = "1"
    try:
        dense = T.sense_normal_raw(x.to(DEV), maps.to(DEV), wd, sub=sub.to(DEV), base_scale=1.0, step=-2.0)
    finally:
        os.environ.pop("DLCS_SENSE_ROWS")
        os.environ.pop("DLCS_DIAG")
    assert nrmse(dense.cpu().numpy(), out.cpu().numpy()) < TOL


@pytest.mark.parametrize("kind", ["vdkt", "sparse", "coil", "empty"])
def test_sense_adj_rows_vs_oracle(kind):
    """dlcs_sense_adj_rows (the row-sparse adjoint: y read on the sampled ky lines
    only) vs the oracle's A^H y (transforms.py:84-90) on the VDkt mask at the
    BASELINE slice, line-sparse non-separable weights, per-coil weights and an empty
    mask; with and without the base / sub epilogue; and against the dense adjoint."""
    import os
    T = _T()
    if kind == "vdkt":
        B, E, C, Tt, Y, X = 1, 2, 8, 20, 192, 160
        w = _vdkt_mask()
    elif kind == "sparse":
        B, E, C, Tt, Y, X = 2, 2, 4, 3, 96, 80
        w = _row_sparse_mask(46, (B, 1, Tt, Y, X), empty_frame=1)
    elif kind == "coil":
        B, E, C, Tt, Y, X = 1, 1, 6, 2, 64, 128
        w = _row_sparse_mask(47, (B, C, Tt, Y, X), frac=0.2)
    else:
        B, E, C, Tt, Y, X = 1, 2, 4, 2, 160, 192
        w = torch.zeros((B, 1, Tt, Y, X))
    maps = recipe.sense_maps(48, B, E, C, Y, X)
    y = recipe.crandn(49, (B, C, Tt, Y, X))            # NOT pre-masked: the operator applies W itself
    base = recipe.crandn(50, (B, E, Tt, Y, X))
    sub = recipe.crandn(51, (B, E, Tt, Y, X))
    ref = O.sense_adjoint(y, maps, w)
    wd, md, yd = w.to(DEV), maps.to(DEV), y.to(DEV)
    out = T.sense_adj_raw(yd, md, wd)
    assert nrmse(ref.numpy(), out.cpu().numpy()) < TOL
    out2 = T.sense_adj_raw(yd, md, wd, base=base.to(DEV), sub=sub.to(DEV), step=-2.0)
    assert nrmse((base - 2.0 * (ref - sub)).numpy(), out2.cpu().numpy()) < TOL
    os.environ["DLCS_SENSE_ROWS"] = "0"
    os.environ["DLCS_DIAG"] = "1"
    try:
        dense = T.sense_adj_raw(yd, md, wd)
    finally:
        os.environ.pop("DLCS_SENSE_ROWS")
        os.environ.pop("DLCS_DIAG")
    assert nrmse(dense.cpu().numpy(), out.cpu().numpy()) < TOL
    # the SenseModel call path takes it too (A(y, adjoint=True))
    A = T.SenseModel(md, weights=wd)
    assert nrmse(ref.numpy(), A(yd, adjoint=True).cpu().numpy()) < TOL


def test_sense_cg_rows_vdkt():
    """dlcs_sense_cg_rows: the device CG on the row-sparse operator, VDkt mask,
    BASELINE slice, vs the oracle's CG loop."""
    T = _T()
    B, E, C, Tt, Y, X = 1, 2, 8, 20, 192, 160
    maps = recipe.sense_maps(51, B, E, C, Y, X)
    w = _vdkt_mask()
    x0 = recipe.crandn(53, (B, E, Tt, Y, X))
    b = recipe.crandn(54, (B, E, Tt, Y, X))
    lam = 0.05
    normal = lambda m: O.sense_adjoint(O.sense_forward(m, maps, w), maps, w) + lam * m
    ref = O.conjugate_gradient(normal, x0, b, 10)
    A = T.SenseModel(maps.to(DEV), weights=w.to(DEV))
    out = A.cg(x0.to(DEV), b.to(DEV), lam, 10)
    assert nrmse(ref.numpy(), out.cpu().numpy()) < TOL
