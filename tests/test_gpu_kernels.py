"""Unit checks of individual HIP kernels (GEMM layouts / epilogues, conv3d
fwd / dgrad / wgrad, LayerNorm) against plain fp32 CPU computations of the same
op, in both storage dtypes."""
import math

import pytest
import torch
import torch.nn.functional as F

from goldutil import nrmse

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _K():
    from dl_cs.models import _ops as K
    return K


def _need_diag(name):
    """Skip unless the loaded library is the DIAG build that carries `name`."""
    from dl_cs import _lib
    if not _lib.has_symbol(name):
        pytest.skip(f"{name}: DIAG build only (make DIAG=1, DLCS_HIP_LIB=.../libdlcs_hip_diag.so)")


def _rnd(shape, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-6), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("a_t,b_t", [(0, 0), (0, 1), (1, 1), (1, 0)])
@pytest.mark.parametrize("M,N,K_", [(300, 160, 200), (129, 480, 160), (64, 70, 33), (1000, 640, 160)])
def test_gemm_layouts(dtype, tol, a_t, b_t, M, N, K_):
    K = _K()
    A = _rnd((K_, M) if a_t else (M, K_), 1)
    B = _rnd((K_, N) if b_t else (N, K_), 2)
    bias = _rnd((N,), 3)
    Am = A.t() if a_t else A
    Bm = B.t() if b_t else B
    ref = Am.to(dtype).double() @ Bm.to(dtype).double().t() + bias.double()
    C = torch.empty((M, N), dtype=torch.float32, device=DEV)
    K.gemm(A.to(DEV, dtype), B.to(DEV, dtype), C, M, N, K_, A.shape[1], B.shape[1], N, a_trans=a_t, b_trans=b_t,
           bias=bias.to(DEV))
    assert nrmse(ref.numpy(), C.cpu().double().numpy()) < max(tol, 1e-6)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogues_and_splitk(dtype):
    K = _K()
    M, N, K_ = 256, 160, 320
    A, B, bias = _rnd((M, K_), 4), _rnd((N, K_), 5), _rnd((N,), 6)
    res = _rnd((M, N), 7)
    Ad, Bd = A.to(DEV, dtype), B.to(DEV, dtype)
    pre = Ad.float().cpu().double() @ Bd.float().cpu().double().t() + bias.double()
    # GELU + aux output + alpha + residual
    C = torch.empty((M, N), device=DEV)
    aux = torch.empty((M, N), device=DEV, dtype=dtype)
    K.gemm(Ad, Bd, C, M, N, K_, K_, K_, N, bias=bias.to(DEV), act=1, aux_out=aux, ldaux=N, alpha=0.5,
           res=res.to(DEV), ldr=N)
    ref = 0.5 * F.gelu(pre) + res.double()
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    assert nrmse(ref.numpy(), C.cpu().double().numpy()) < tol
    assert nrmse(pre.numpy(), aux.float().cpu().double().numpy()) < (1e-6 if dtype == torch.float32 else 1e-2)
    # ReLU epilogue (act 3)
    C4 = torch.empty((M, N), device=DEV)
    K.gemm(Ad, Bd, C4, M, N, K_, K_, K_, N, bias=bias.to(DEV), act=3)
    assert nrmse(torch.relu(pre).numpy(), C4.cpu().double().numpy()) < tol
    # split-K accumulate into fp32
    C2 = res.clone().to(DEV)
    K.gemm(Ad, Bd, C2, M, N, K_, K_, K_, N, accumulate=1, splitk=4)
    ref2 = pre - bias.double() + res.double()
    assert nrmse(ref2.numpy(), C2.cpu().double().numpy()) < tol
    # accumulate without split-K (plain read-modify-write of fp32 C)
    C5 = res.clone().to(DEV)
    K.gemm(Ad, Bd, C5, M, N, K_, K_, K_, N, accumulate=1)
    assert nrmse(ref2.numpy(), C5.cpu().double().numpy()) < tol
    # two scaled residuals (the embed backward: + 2 g_h + g_b), bf16 / fp32 output
    res2 = _rnd((M, N), 9).to(dtype)
    for cdt in (torch.float32, dtype):
        C6 = torch.empty((M, N), device=DEV, dtype=cdt)
        K.gemm(Ad, Bd, C6, M, N, K_, K_, K_, N, bias=bias.to(DEV), res=res.to(DEV), ldr=N, res_scale=2.0,
               res2=res2.to(DEV), ldr2=N, res2_scale=-0.5)
        ref6 = pre + 2.0 * res.double() - 0.5 * res2.double()
        assert nrmse(ref6.numpy(), C6.float().cpu().double().numpy()) < tol
    # row scatter
    perm = torch.randperm(M, generator=torch.Generator().manual_seed(8)).to(torch.int32)
    C3 = torch.zeros((M, N), device=DEV)
    K.gemm(Ad, Bd, C3, M, N, K_, K_, K_, N, row_map=perm.to(DEV))
    ref3 = torch.zeros_like(pre)
    ref3[perm.long()] = pre - bias.double()
    assert nrmse(ref3.numpy(), C3.cpu().double().numpy()) < tol


def _to_blocked(x):
    """[B, C, D, H, W] -> blocked rows [B*D*H*W, C] (layout.hip)."""
    B, C, D, H, W = x.shape
    t = x.permute(0, 2, 3, 4, 1).reshape(B, D // 4, 4, H // 4, 4, W // 4, 4, C)
    return t.permute(0, 1, 3, 5, 2, 4, 6, 7).reshape(-1, C)


def _from_blocked(r, B, C, D, H, W):
    t = r.reshape(B, D // 4, H // 4, W // 4, 4, 4, 4, C).permute(0, 1, 4, 2, 5, 3, 6, 7)
    return t.reshape(B, D, H, W, C).permute(0, 4, 1, 2, 3)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1.5e-2)])
@pytest.mark.parametrize("cin,cout,grid", [(160, 160, (1, 8, 16, 12)), (4, 160, (1, 4, 8, 8)),
                                           (160, 4, (2, 4, 8, 16))])
def test_conv3d_fwd_dgrad_wgrad(dtype, tol, cin, cout, grid):
    K = _K()
    B, D, H, W = grid
    x = _rnd((B, cin, D, H, W), 10)
    w = _rnd((cout, cin, 3, 3, 3), 11) / (27 * cin) ** 0.5
    b = _rnd((cout,), 12)
    res = _rnd((B, cout, D, H, W), 13)
    cin_ld = max(8, cin)
    xr = torch.zeros((B * D * H * W, cin_ld))
    xr[:, :cin] = _to_blocked(x)
    xd = xr.to(DEV, dtype)
    xq = _from_blocked(xd[:, :cin].float().cpu(), B, cin, D, H, W)      # quantised input
    wq = w.to(dtype).float()
    # forward with relu prologue + residual epilogue
    wp = K.conv_pack(w.to(DEV), dtype, 0)
    out_ld = max(8, cout)
    out = K.conv3d(xd, cin, wp, cout, out_ld, grid, bias=b.to(DEV), relu_in=1,
                   res=_pad_cols(_to_blocked(res), out_ld).to(DEV), res_scale=2.0, out_dtype=torch.float32)
    ref = F.conv3d(F.relu(xq).double(), wq.double(), b.double(), padding=1) + 2 * res.double()
    got = _from_blocked(out[:, :cout].cpu(), B, cout, D, H, W)
    assert nrmse(ref.numpy(), got.double().numpy()) < tol
    # dgrad with relu mask: dx = conv_T(g) * (x > 0)
    gout = _rnd((B, cout, D, H, W), 14)
    gr = torch.zeros((B * D * H * W, out_ld))
    gr[:, :cout] = _to_blocked(gout)
    gd = gr.to(DEV, dtype)
    gq = _from_blocked(gd[:, :cout].float().cpu(), B, cout, D, H, W)
    wd = K.conv_pack(w.to(DEV), dtype, 1)
    dx = K.conv3d(gd, cout, wd, cin, cin_ld, grid, mask=xd, out_dtype=torch.float32)
    xr_ = xq.double().requires_grad_()
    yy = F.conv3d(F.relu(xr_), wq.double(), None, padding=1)
    yy.backward(gq.double())
    got = _from_blocked(dx[:, :cin].cpu(), B, cin, D, H, W)
    assert nrmse(xr_.grad.numpy(), got.double().numpy()) < tol
    # wgrad (+ the bias gradient: fused in the bf16 SFE-shape kernel, a column-sum launch otherwise)
    dwp = torch.zeros((27, K.pad32(cout), K.pad32(cin)), device=DEV)
    db = torch.full((cout,), -0.25, device=DEV)
    K.conv3d_wgrad(xd, cin, 1, gd, cout, grid, dwp, vox_per_block=256, dbias=db)
    assert nrmse((gq.double().sum(dim=(0, 2, 3, 4)) - 0.25).numpy(), db.cpu().double().numpy()) < 1e-6
    gw = torch.zeros((cout, cin, 3, 3, 3), device=DEV)
    K.conv_unpack_grad(dwp, gw, cout, cin)
    wr_ = wq.double().requires_grad_()
    yy = F.conv3d(F.relu(xq.double()), wr_, None, padding=1)
    yy.backward(gq.double())
    assert nrmse(wr_.grad.numpy(), gw.cpu().double().numpy()) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1.5e-2)])
@pytest.mark.parametrize("grid", [(1, 8, 16, 12), (1, 12, 8, 24), (2, 8, 12, 20)])
def test_conv3d_relu_out_residual(dtype, tol, grid):
    """The 160->160 path used by the regularizer (v2 kernel for bf16): no ReLU
    prologue, fp32 / bf16 residual with scale, ReLU epilogue."""
    K = _K()
    B, D, H, W = grid
    C = 160
    x = _rnd((B, C, D, H, W), 30)
    w = _rnd((C, C, 3, 3, 3), 31) / (27 * C) ** 0.5
    b = _rnd((C,), 32)
    res = _rnd((B, C, D, H, W), 33)
    xd = _to_blocked(x).to(DEV, dtype)
    rd = _to_blocked(res).to(DEV, dtype)
    xq = _from_blocked(xd.float().cpu(), B, C, D, H, W)
    rq = _from_blocked(rd.float().cpu(), B, C, D, H, W)
    wp = K.conv_pack(w.to(DEV), dtype, 0)
    out = K.conv3d(xd, C, wp, C, C, grid, bias=b.to(DEV), res=rd, res_scale=2.0, relu_out=1,
                   out_dtype=torch.float32)
    ref = F.relu(F.conv3d(xq.double(), w.to(dtype).double(), b.double(), padding=1) + 2 * rq.double())
    got = _from_blocked(out.cpu(), B, C, D, H, W)
    # quantised operands, fp32 accumulation and fp32 output: only summation-order error remains
    assert nrmse(ref.numpy(), got.double().numpy()) < min(tol, 1e-5)
    # wgrad without ReLU prologue (bf16: the 3-tap-row DMA kernel), g = res, with the
    # bias gradient (bf16: fused into the kernel as g^T 1; fp32: a column-sum launch)
    dwp = torch.zeros((27, C, C), device=DEV)
    db = torch.full((C,), 0.5, device=DEV)
    K.conv3d_wgrad(xd, C, 0, rd, C, grid, dwp, dbias=db)
    gw = torch.zeros((C, C, 3, 3, 3), device=DEV)
    K.conv_unpack_grad(dwp, gw, C, C)
    wr_ = w.to(dtype).double().requires_grad_()
    F.conv3d(xq.double(), wr_, None, padding=1).backward(rq.double())
    assert nrmse(wr_.grad.numpy(), gw.cpu().double().numpy()) < tol
    db_ref = 0.5 + rq.double().sum(dim=(0, 2, 3, 4))
    assert nrmse(db_ref.numpy(), db.cpu().double().numpy()) < 1e-6


@pytest.mark.parametrize("kern", ["v7", "v6"])
@pytest.mark.parametrize("grid", [(1, 8, 16, 12), (1, 4, 136, 128), (2, 8, 12, 20)])
def test_conv3d_bf16_v6(grid, kern, monkeypatch):
    """The bf16 160 -> 160 forward / input gradient -- conv3d_v6.inc (default: six taps
    per step) and conv3d_v7.inc (DLCS_CONV_V7=1: two 4-wave workgroups per CU, units of
    256 voxels x 80 output channels, one tap row per step) -- in their two
    production epilogues, bf16 out: bias + bf16 residual (x 2) + ReLU-out, and
    bias-free input gradient behind a bf16 ReLU mask, vs float64 on the bf16-quantised
    operands (only the bf16 rounding of the output remains: NRMSE <= 4e-3); grid
    (1, 4, 136, 128) has 272 tiles = 256 + 16 (v7: 544 units = 512 + 32), so its last
    partial round runs as single-chunk workgroups + a fixed-order reduce: the same
    output as the unsplit launch (fp32 summation order, then one bf16 rounding) and
    bit-identical across runs."""
    monkeypatch.setenv("DLCS_DIAG", "1")
    monkeypatch.setenv("DLCS_CONV_V7", "1" if kern == "v7" else "0")
    tail_hook = "DLCS_V6_TAIL" if kern == "v6" else "DLCS_V7_TAIL"
    K = _K()
    B, D, H, W = grid
    C = 160
    x = _rnd((B, C, D, H, W), 40)
    w = _rnd((C, C, 3, 3, 3), 41) / (27 * C) ** 0.5
    b = _rnd((C,), 42)
    res = _rnd((B, C, D, H, W), 43)
    xd = _to_blocked(x).to(DEV, torch.bfloat16)
    rd = _to_blocked(res).to(DEV, torch.bfloat16)
    xq = _from_blocked(xd.float().cpu(), B, C, D, H, W).double()
    rq = _from_blocked(rd.float().cpu(), B, C, D, H, W).double()
    wq = w.to(torch.bfloat16).double()
    wp, wdp = K.conv_pack(w.to(DEV), torch.bfloat16, 0), K.conv_pack(w.to(DEV), torch.bfloat16, 1)

    def run(tail):
        monkeypatch.setenv(tail_hook, "1" if tail else "0")
        f = K.conv3d(xd, C, wp, C, C, grid, bias=b.to(DEV), res=rd, res_scale=2.0, relu_out=1)
        d = K.conv3d(rd, C, wdp, C, C, grid, mask=xd)
        return f.cpu(), d.cpu()

    f1, d1 = run(True)
    ref = F.relu(F.conv3d(xq, wq, b.double(), padding=1) + 2 * rq)
    assert nrmse(ref.numpy(), _from_blocked(f1.float(), B, C, D, H, W).double().numpy()) < 4e-3
    xr_ = xq.clone().requires_grad_()
    F.conv3d(F.relu(xr_), wq, None, padding=1).backward(rq)
    assert nrmse(xr_.grad.numpy(), _from_blocked(d1.float(), B, C, D, H, W).double().numpy()) < 4e-3
    f0, d0 = run(False)
    f2, d2 = run(True)
    assert torch.equal(f1, f2) and torch.equal(d1, d2)
    assert nrmse(f0.double().numpy(), f1.double().numpy()) < 4e-3
    assert nrmse(d0.double().numpy(), d1.double().numpy()) < 4e-3


@pytest.mark.parametrize("M,N", [(13440, 10240), (300, 320), (64, 160), (300, 1280)])
def test_gemm_k160_f16x3(M, N):
    """K = 160 GEMM on fp16 matrix cores (2-plane split): the unembed forward's
    bias + ReLU epilogue and the embed input gradient's two scaled residuals,
    on a gradient-sized A (~1e-7), vs float64; partial row tiles (M = 300)."""
    K = _K()
    g = torch.Generator().manual_seed(5)
    A = torch.randn((M, 160), generator=g) * 1e-7
    B = torch.randn((N, 160), generator=g) / 160 ** 0.5
    bias = torch.randn((N,), generator=g)
    r1 = torch.randn((M, N), generator=g)
    r2 = torch.randn((M, N), generator=g)
    Ad, Bd = A.to(DEV), B.to(DEV)
    C = torch.empty((M, N), device=DEV)
    K.gemm_k160_f16x3(K.split2(Ad), M, K.split2(Bd), N, C, bias=bias.to(DEV) * 1e-7, act=3)
    ref = torch.relu(A.double() @ B.double().t() + bias.double() * 1e-7)
    assert nrmse(ref.numpy(), C.cpu().double().numpy()) < 2e-6
    pc = K.planes_alloc(M, DEV)
    K.gemm_k160_f16x3(K.split2(Ad), M, K.split2(Bd), N, C, res=r1.to(DEV), res_scale=2.0, res2=r2.to(DEV),
                      out_max=K.planes_max(pc, M))
    assert float(pc[M * 640:M * 640 + 4].view(torch.float32)[0]) == float(C.abs().max())
    ref = A.double() @ B.double().t() + 2.0 * r1.double() + r2.double()
    assert nrmse(ref.numpy(), C.cpu().double().numpy()) < 2e-6


def _planes_back(planes, rows):
    """(hi + lo) / s of a split2 buffer [rows] and its trailer word as a float."""
    pl = planes[:rows * 640].view(torch.float16).view(rows, 5, 2, 32).float()
    mx = float(planes[rows * 640:rows * 640 + 4].view(torch.float32)[0])
    f, e = math.frexp(mx)
    scale = 2.0 ** (14 - (e - 1 if f == 0.5 else e)) if mx > 0 else 1.0
    return (pl[:, :, 0] + pl[:, :, 1]).reshape(rows, 160) / scale, mx


def _check_producer_planes(planes, out, rows, bound_ref):
    """The producer-written planes: trailer = the bound (>= max|out|, = the host-side
    bound to fp32 rounding), and (hi + lo) / s reassembles out to the split's
    guarantee |back - out| <= 2^-22 |out| + 2^-38 B (with margin 2x)."""
    back, B = _planes_back(planes, rows)
    assert B >= float(out.abs().max())
    assert abs(B / (bound_ref * (1 + 2 ** -10)) - 1) < 1e-5
    err = (back.double() - out.double()).abs()
    tol = 2.0 ** -21 * out.double().abs() + 2.0 ** -37 * B
    assert bool((err <= tol).all()), float((err / tol).max())


def test_producer_planes():
    """Producer-side split: the conv (residual and mask forms, including the tail-split
    reduce: 272 tiles here) and the K = 160 GEMM write their output's planes with the
    scale of a bound set beforehand (dlcs_planes_bound from dlcs_abs_row_sum_max
    norms); the planes reassemble the fp32 output to the split's guarantee, the bound
    covers max|out|, and a conv reading them matches one reading split2(out) (same
    budget as the split: NRMSE <= 1e-6 between the two)."""
    K = _K()
    grid = (1, 4, 136, 128)
    rows = 4 * 136 * 128
    g = torch.Generator(device=DEV).manual_seed(19)
    x = torch.randn((rows, 160), device=DEV, generator=g)
    r = torch.randn((rows, 160), device=DEV, generator=g)
    w = torch.randn((160, 160, 3, 3, 3), device=DEV, generator=g) / (27 * 160) ** 0.5
    bias = torch.randn((160,), device=DEV, generator=g)
    xp = K.split2(x)
    wf, wd = K.conv_pack_f16x3(w, 0), K.conv_pack_f16x3(w, 1)
    # ||W||_inf of the forward (rows co) and of the dgrad (rows ci)
    nf = K.abs_row_sum_max(w, 160, 27 * 160, 27 * 160)
    nd = K.abs_row_sum_max(w, 160, 27, 27, n_outer=160, outer_stride=27 * 160)
    nf_ref = float(w.double().abs().sum(dim=(1, 2, 3, 4)).max())
    nd_ref = float(w.double().abs().sum(dim=(0, 2, 3, 4)).max())
    assert abs(float(nf.view(torch.float32)[0]) / nf_ref - 1) < 1e-5
    assert abs(float(nd.view(torch.float32)[0]) / nd_ref - 1) < 1e-5
    # the engine's cached norms, including the k4s4 patch weights read in their own layout
    from dl_cs.models import engine as E
    wp = torch.randn((160, 160, 4, 4, 4), device=DEV, generator=g)
    for wt, kind, ref in ((w, False, nf_ref), (w, True, nd_ref),
                          (wp, "patch", float(wp.double().abs().sum(0).max()))):
        assert abs(float(E._conv_norm(wt, 160, dgrad=kind).view(torch.float32)[0]) / ref - 1) < 1e-5
    xm = xp[rows * 640:rows * 640 + 4].view(torch.int32)
    rm = K.absmax(r)
    # forward: relu(conv(x) + b + 2 r), out_max still the true max
    po = K.planes_alloc(rows, DEV)
    K.planes_bound(po, rows, m0=xm, n0=nf, m1=rm, c1=2.0, vec=bias)
    om = K.zeros((1,), torch.int32, DEV)
    out = K.conv3d_f16x3(xp, wf, grid, bias=bias, res=r, res_scale=2.0, relu_out=1, out_max=K.p(om), out_planes=po)
    ref_out = K.conv3d_f16x3(xp, wf, grid, bias=bias, res=r, res_scale=2.0, relu_out=1)
    assert torch.equal(out, ref_out)
    assert float(om.view(torch.float32)[0]) == float(out.abs().max())
    bref = (float(x.abs().max()) * float(nf.view(torch.float32)[0]) + 2 * float(r.abs().max())
            + float(bias.abs().max()))
    _check_producer_planes(po, out, rows, bref)
    # the ReLU mask read from the planes (hi | lo != 0) is exactly out > 0 (a nonzero value
    # whose planes would both round to zero keeps its sign in the smallest subnormal)
    pl = po[:rows * 640].view(torch.int16).view(rows, 5, 2, 32)
    nz = (((pl[:, :, 0] & 0x7FFF) != 0) | ((pl[:, :, 1] & 0x7FFF) != 0)).reshape(rows, 160)
    assert torch.equal(nz, out > 0)
    gq = K.split2(torch.randn((rows, 160), device=DEV, generator=g))
    assert torch.equal(K.conv3d_f16x3(gq, wd, grid, mask_planes=po), K.conv3d_f16x3(gq, wd, grid, mask=out))
    # a consumer of the producer's planes vs one of split2(out)
    y1 = K.conv3d_f16x3(po, wf, grid)
    y2 = K.conv3d_f16x3(K.split2(out), wf, grid)
    assert nrmse(y2.double().cpu().numpy(), y1.double().cpu().numpy()) < 1e-6
    # dgrad with a ReLU mask on a gradient-sized operand
    gd = torch.randn((rows, 160), device=DEV, generator=g) * 1e-7
    gp = K.split2(gd)
    pd = K.planes_alloc(rows, DEV)
    K.planes_bound(pd, rows, m0=gp[rows * 640:rows * 640 + 4].view(torch.int32), n0=nd)
    dx = K.conv3d_f16x3(gp, wd, grid, mask=x, out_planes=pd)
    assert torch.equal(dx, K.conv3d_f16x3(gp, wd, grid, mask=x))
    _check_producer_planes(pd, dx, rows, float(gd.abs().max()) * float(nd.view(torch.float32)[0]))
    # planes only (no fp32 output) with the column sums (the DFE input gradient g_out and the
    # stage tail's bias gradient), through the tail split (272 = 256 + 16 tiles)
    cs = torch.full((160,), 0.5, device=DEV)
    pd2 = K.planes_alloc(rows, DEV)
    K.planes_bound(pd2, rows, m0=gp[rows * 640:rows * 640 + 4].view(torch.int32), n0=nd)
    assert K.conv3d_f16x3(gp, wd, grid, mask=x, out_planes=pd2, planes_only=True, colsum=cs) is None
    _check_producer_planes(pd2, dx, rows, float(gd.abs().max()) * float(nd.view(torch.float32)[0]))
    assert nrmse(dx.double().sum(0).cpu().numpy() + 0.5, cs.double().cpu().numpy()) < 1e-6
    cs2 = torch.full((160,), 0.5, device=DEV)
    K.conv3d_f16x3(gp, wd, grid, mask=x, out_planes=pd2, planes_only=True, colsum=cs2)
    assert torch.equal(cs, cs2)                                      # fixed-order sums
    # the K = 160 GEMM: relu(A B^T + b) as [M N / 160][160] rows
    M, N = 300, 1600
    A = torch.randn((M, 160), device=DEV, generator=g)
    Bm = torch.randn((N, 160), device=DEV, generator=g) / 160 ** 0.5
    bn = torch.randn((N,), device=DEV, generator=g)
    ap = K.split2(A)
    nb = K.abs_row_sum_max(Bm, N, 160, 160)
    rowsC = M * N // 160
    pc = K.planes_alloc(rowsC, DEV)
    K.planes_bound(pc, rowsC, m0=ap[M * 640:M * 640 + 4].view(torch.int32), n0=nb, vec=bn)
    Cm = torch.empty((M, N), device=DEV)
    K.gemm_k160_f16x3(ap, M, K.split2(Bm), N, Cm, bias=bn, act=3, out_planes=pc)
    bref = float(A.abs().max()) * float(nb.view(torch.float32)[0]) + float(bn.abs().max())
    _check_producer_planes(pc, Cm.view(rowsC, 160), rowsC, bref)
    # planes-only output (C = None) with the column sums of the [M N / 160][160] view
    # (the embed gradient's g_s: planes for the SFE conv, column sums = its bias gradient)
    r1 = torch.randn((M, N), device=DEV, generator=g)
    bp = K.split2(Bm)
    pc2 = K.planes_alloc(rowsC, DEV)
    K.planes_bound(pc2, rowsC, m0=ap[M * 640:M * 640 + 4].view(torch.int32), n0=nb, m1=K.absmax(r1), c1=2.0)
    cs = torch.full((160,), 0.25, device=DEV)
    assert K.gemm_k160_f16x3(ap, M, bp, N, None, res=r1, res_scale=2.0, out_planes=pc2, colsum=cs) is None
    Cr = torch.empty((M, N), device=DEV)
    K.gemm_k160_f16x3(ap, M, bp, N, Cr, res=r1, res_scale=2.0)
    bref2 = float(A.abs().max()) * float(nb.view(torch.float32)[0]) + 2 * float(r1.abs().max())
    _check_producer_planes(pc2, Cr.view(rowsC, 160), rowsC, bref2)
    assert nrmse(Cr.view(rowsC, 160).double().sum(0).cpu().numpy() + 0.25, cs.double().cpu().numpy()) < 1e-6
    # residuals read from planes ((hi + lo) / s) in place of the fp32 tensors
    Cq = torch.empty((M, N), device=DEV)
    K.gemm_k160_f16x3(ap, M, bp, N, Cq, res_planes=pc, res_scale=2.0, res2_planes=pc2, res2_scale=-1.0)
    Cf = torch.empty((M, N), device=DEV)
    K.gemm_k160_f16x3(ap, M, bp, N, Cf, res=Cm, res_scale=2.0, res2=Cr, res2_scale=-1.0)
    assert nrmse(Cf.double().cpu().numpy(), Cq.double().cpu().numpy()) < 1e-6
    # the conv refuses planes on the generic epilogue (no fused residual / mask form)
    with pytest.raises(RuntimeError):
        K.conv3d_f16x3(xp, wf, grid, out_planes=K.planes_alloc(rows, DEV))


def test_conv3d_f16x3_tail_split(monkeypatch):
    """The last partial round of tiles (272 = 256 + 16 here; 3360 = 13 x 256 + 32 at
    BASELINE size) runs as single-chunk workgroups plus a fixed-order reduce: the
    same result as the unsplit launch to fp32 summation order (NRMSE <= 1e-6) for
    the forward (bias + residual + ReLU-out + out_max) and the dgrad (ReLU mask),
    and bit-identical across runs."""
    K = _K()
    grid = (1, 4, 136, 128)
    rows = 4 * 136 * 128
    g = torch.Generator(device=DEV).manual_seed(9)
    x = torch.randn((rows, 160), device=DEV, generator=g)
    r = torch.randn((rows, 160), device=DEV, generator=g)
    w = torch.randn((160, 160, 3, 3, 3), device=DEV, generator=g) / (27 * 160) ** 0.5
    bias = torch.randn((160,), device=DEV, generator=g)
    xp = K.split2(x)
    wf, wd = K.conv_pack_f16x3(w, 0), K.conv_pack_f16x3(w, 1)

    def run(tail):
        monkeypatch.setenv("DLCS_DIAG", "1")
        monkeypatch.setenv("DLCS_H3_TAIL", "1" if tail else "0")
        pm = K.planes_alloc(rows, DEV)
        f = K.conv3d_f16x3(xp, wf, grid, bias=bias, res=r, relu_out=1, out_max=K.planes_max(pm, rows))
        d = K.conv3d_f16x3(xp, wd, grid, mask=r)
        mx = float(pm[rows * 640:rows * 640 + 4].view(torch.float32)[0])
        return f.cpu(), d.cpu(), mx

    f0, d0, m0 = run(False)
    f1, d1, m1 = run(True)
    f2, d2, m2 = run(True)
    assert nrmse(f0.double().numpy(), f1.double().numpy()) < 1e-6
    assert nrmse(d0.double().numpy(), d1.double().numpy()) < 1e-6
    assert m1 == float(f1.abs().max()) and abs(m1 - m0) <= 1e-5 * m0
    assert torch.equal(f1, f2) and torch.equal(d1, d2)


@pytest.mark.parametrize("M,N,Kd", [(13440, 160, 10240), (300, 320, 1000), (64, 160, 36)])
def test_gemm_f32_splitk_det(M, N, Kd):
    """fp32 split-K GEMM with fixed-order partial sums (the patch embed forward):
    C += A B^T vs float64 (NRMSE <= 1e-6), and bit-identical across runs."""
    K = _K()
    g = torch.Generator().manual_seed(7)
    A = torch.randn((M, Kd), generator=g)
    B = torch.randn((N, Kd), generator=g) / Kd ** 0.5
    C0 = torch.randn((M, N), generator=g)
    Ad, Bd = A.to(DEV), B.to(DEV)
    outs = []
    for _ in range(2):
        C = C0.to(DEV)
        K.gemm_f32_splitk_det(Ad, Bd, C, M, N, Kd, Kd, Kd)
        outs.append(C.cpu())
    ref = C0.double() + A.double() @ B.double().t()
    assert nrmse(ref.numpy(), outs[0].double().numpy()) < 1e-6
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("M,N,Kd,lda,wide", [(13440, 160, 10240, 10240, False), (300, 320, 1024, 1040, True),
                                             (65, 160, 32, 32, False), (1, 160, 96, 100, True)])
def test_gemm_nt_x6(M, N, Kd, lda, wide):
    """The fp32 patch-embed forward on the bf16 3-plane split (dlcs_gemm_nt_x6):
    C += A B^T vs float64 at the fp32 floor (NRMSE <= 1e-6, and within 2x of the
    f32-MFMA split-K kernel's own error), ragged M, strided A rows, a single
    k step, operands spanning 2^+-40 ('wide'); bit-identical across runs; an
    unsupported N is refused.  DIAG build only (libdlcs_hip_diag.so): the product's
    patch-embed forward is dlcs_gemm_h3r's split-K path (test_gemm_h3r_segments)."""
    K = _K()
    _need_diag("dlcs_gemm_nt_x6")
    g = torch.Generator().manual_seed(11)
    A = torch.randn((M, lda), generator=g)
    B = torch.randn((N, Kd), generator=g) / Kd ** 0.5
    if wide:
        A *= torch.exp2(torch.randint(-40, 40, (M, 1), generator=g).float())
        B *= torch.exp2(torch.randint(-40, 40, (1, Kd), generator=g).float())
    C0 = torch.randn((M, N), generator=g)
    Ad, Bd = A.to(DEV), B.to(DEV)
    outs = []
    for _ in range(2):
        C = C0.to(DEV)
        K.gemm_nt_x6(Ad, Bd, C, M, N, Kd, lda, Kd)
        outs.append(C.cpu())
    ref = C0.double() + A[:, :Kd].double() @ B.double().t()
    err = nrmse(ref.numpy(), outs[0].double().numpy())
    assert err < 1e-6
    assert torch.equal(outs[0], outs[1])
    if lda == Kd:
        C = C0.to(DEV)
        K.gemm_f32_splitk_det(Ad, Bd, C, M, N, Kd, Kd, Kd)
        assert err <= 2 * nrmse(ref.numpy(), C.cpu().double().numpy()) + 1e-9
    with pytest.raises(Exception):
        K.gemm_nt_x6(Ad, Bd[:100].contiguous(), torch.zeros((M, 100), device=DEV), M, 100, Kd, lda, Kd)


@pytest.mark.parametrize("M,N", [(13440, 640), (13440, 480), (300, 160)])
def test_linear_k160_f16x3(M, N):
    """The Swin block's in = 160 Linears on the f16x3 split (dlcs_linear_k160_f16x3):
    fc1 forward (bias + GELU, pre-activation to aux_out), the fc2 input gradient
    (times GELU'(aux)), and the proj forward's window_reverse scatter (row_map,
    skipped rows, residual at the mapped row, alpha) vs float64; NRMSE <= 2e-6."""
    import math
    K = _K()
    g = torch.Generator().manual_seed(6)
    x = torch.randn((M, 160), generator=g)
    w = torch.randn((N, 160), generator=g) / 160 ** 0.5
    b = torch.randn((N,), generator=g) * 0.1
    xd, wd = x.to(DEV), w.to(DEV)
    xp, wp = K.split2(xd), K.split2(wd)
    pre = x.double() @ w.double().t() + b.double()
    gelu = 0.5 * pre * (1.0 + torch.erf(pre / math.sqrt(2.0)))
    out = torch.empty((M, N), device=DEV)
    aux = torch.empty((M, N), device=DEV)
    K.linear_k160_f16x3(xp, M, wp, N, out, bias=b.to(DEV), act=1, aux_out=aux)
    assert nrmse(pre.numpy(), aux.cpu().double().numpy()) < 2e-6
    assert nrmse(gelu.numpy(), out.cpu().double().numpy()) < 2e-6
    dgelu = 0.5 * (1.0 + torch.erf(pre / math.sqrt(2.0))) + pre * torch.exp(-0.5 * pre * pre) / math.sqrt(2 * math.pi)
    K.linear_k160_f16x3(xp, M, wp, N, out, act=2, aux=aux)
    ref = (x.double() @ w.double().t()) * dgelu
    assert nrmse(ref.numpy(), out.cpu().double().numpy()) < 2e-6
    # scatter: row m -> perm[m] (every 7th row skipped), residual read at the mapped row
    perm = torch.randperm(M, generator=g).to(torch.int32)
    perm[::7] = -1
    res = torch.randn((M, N), generator=g)
    out2 = torch.full((M, N), 123.0, device=DEV)
    K.linear_k160_f16x3(xp, M, wp, N, out2, bias=b.to(DEV), alpha=0.5, res=res.to(DEV), row_map=perm.to(DEV))
    ref2 = torch.full((M, N), 123.0, dtype=torch.float64)
    keep = perm >= 0
    ref2[perm[keep].long()] = 0.5 * pre[keep] + res.double()[perm[keep].long()]
    assert nrmse(ref2.numpy(), out2.cpu().double().numpy()) < 2e-6


def _rel_err(ref, got):
    """||got - ref|| / ||ref|| (float64)."""
    return float((got.double() - ref).norm() / ref.norm())


@pytest.mark.parametrize("M,N,Kd,trans", [(13440, 480, 160, False), (13440, 160, 640, False), (13440, 160, 480, True),
                                          (13440, 640, 160, True), (300, 160, 160, False), (77, 320, 640, True)])
def test_gemm_h3r(M, N, Kd, trans):
    """Row-scaled f16x3 token Linear (dlcs_gemm_h3r, B packed by dlcs_h3r_pack_multi
    from W or W^T) vs float64: plain, bias + GELU (pre-activation to aux_out),
    times GELU'(aux), and the row_map scatter with alpha + residual + skipped rows.
    Bar: within 4x torch's own fp32 GEMM error vs float64 (and <= 2e-6 NRMSE);
    then heavy-tailed rows (row magnitudes over 1e-6 .. 1e3 and one column x1e4),
    where the per-row scale must keep every row at fp32 accuracy."""
    K = _K()
    g = torch.Generator().manual_seed(16)
    x = torch.randn((M, Kd), generator=g)
    w = torch.randn((Kd, N) if trans else (N, Kd), generator=g) / Kd ** 0.5
    b = torch.randn((N,), generator=g) * 0.1
    wt = w.t() if trans else w                       # [N, K]: y = x wt^T
    xd = x.to(DEV)
    (wp,) = K.h3r_pack([(w.to(DEV), trans)])
    pre = x.double() @ wt.double().t()
    floor32 = _rel_err(pre, (x @ wt.t()))
    bar = lambda: max(2e-6, 4 * floor32)
    out = K.linear_h3r(xd, wp, N)
    e = _rel_err(pre, out.cpu())
    print(f"h3r {M}x{N}x{Kd} trans={trans}: err {e:.3g}, torch fp32 floor {floor32:.3g}")
    assert e <= bar()
    preb = pre + b.double()
    gelu = 0.5 * preb * (1.0 + torch.erf(preb / math.sqrt(2.0)))
    aux = torch.empty((M, N), device=DEV)
    out = K.linear_h3r(xd, wp, N, bias=b.to(DEV), act=1, aux_out=aux)
    assert _rel_err(preb, aux.cpu()) <= bar() and _rel_err(gelu, out.cpu()) <= bar()
    dgelu = 0.5 * (1.0 + torch.erf(preb / math.sqrt(2.0))) + preb * torch.exp(-0.5 * preb * preb) / math.sqrt(2 * math.pi)
    out = K.linear_h3r(xd, wp, N, act=2, aux=aux)
    assert _rel_err(pre * dgelu, out.cpu()) <= bar()
    perm = torch.randperm(M, generator=g).to(torch.int32)
    perm[::7] = -1
    res = torch.randn((M, N), generator=g)
    out2 = torch.full((M, N), 123.0, device=DEV)
    K.linear_h3r(xd, wp, N, out=out2, bias=b.to(DEV), alpha=0.5, res=res.to(DEV), row_map=perm.to(DEV))
    ref2 = torch.full((M, N), 123.0, dtype=torch.float64)
    keep = perm >= 0
    ref2[perm[keep].long()] = 0.5 * preb[keep] + res.double()[perm[keep].long()]
    assert _rel_err(ref2, out2.cpu()) <= bar()
    out3 = out2.clone()
    K.linear_h3r(xd, wp, N, out=out3, accumulate=1)
    assert _rel_err(ref2 + pre, out3.cpu()) <= bar()
    # heavy-tailed: each row at its own magnitude, one input column x 1e4
    rs = torch.exp(torch.empty((M, 1)).uniform_(math.log(1e-6), math.log(1e3), generator=g))
    xh = x * rs
    xh[:, 3] *= 1e4
    pre = xh.double() @ wt.double().t()
    out = K.linear_h3r(xh.to(DEV), wp, N).cpu().double()
    rowerr = ((out - pre).norm(dim=1) / pre.norm(dim=1)).max().item()
    row32 = (((xh @ wt.t()).double() - pre).norm(dim=1) / pre.norm(dim=1)).max().item()
    print(f"  heavy-tailed rows: worst row err {rowerr:.3g}, torch fp32 worst row {row32:.3g}")
    assert rowerr <= max(4e-6, 4 * row32)


@pytest.mark.parametrize("M,N,Kd,trans", [(23040, 1152, 384, False), (23040, 384, 1536, False),
                                          (23040, 384, 1152, True), (23040, 1536, 384, True),
                                          (5000, 576, 192, False), (777, 192, 768, False), (300, 64, 192, True),
                                          (13440, 160, 10240, True), (13440, 160, 10240, False)])
def test_gemm_h3r_segments(M, N, Kd, trans):
    """dlcs_gemm_h3r at the DiT / Latte token-Linear shapes (N tiles of 128 / 64, K
    in 192-wide segments with one scale per row and segment): plain, bias + GELU-tanh
    (pre-activation to aux_out), times GELU-tanh'(aux), row_map scatter + residual,
    and heavy-tailed rows with one column x1e4 -- vs float64, within 4x torch's own
    fp32 GEMM error (and <= 2e-6 NRMSE).  K = 10240 (the patch-embed forward and the
    unembed input gradient) runs split-K over eight XCD-group K ranges."""
    K = _K()
    g = torch.Generator().manual_seed(17)
    x = torch.randn((M, Kd), generator=g)
    w = torch.randn((Kd, N) if trans else (N, Kd), generator=g) / Kd ** 0.5
    b = torch.randn((N,), generator=g) * 0.1
    wt = w.t() if trans else w
    xd = x.to(DEV)
    (wp,) = K.h3r_pack([(w.to(DEV), trans)])
    pre = x.double() @ wt.double().t()
    floor32 = _rel_err(pre, (x @ wt.t()))
    bar = max(2e-6, 4 * floor32)
    e = _rel_err(pre, K.linear_h3r(xd, wp, N).cpu())
    print(f"h3r {M}x{N}x{Kd} trans={trans}: err {e:.3g}, torch fp32 floor {floor32:.3g}")
    assert e <= bar
    preb = pre + b.double()
    u = math.sqrt(2.0 / math.pi) * (preb + 0.044715 * preb ** 3)
    gelu = 0.5 * preb * (1.0 + torch.tanh(u))
    aux = torch.empty((M, N), device=DEV)
    out = K.linear_h3r(xd, wp, N, bias=b.to(DEV), act=4, aux_out=aux)
    assert _rel_err(preb, aux.cpu()) <= bar and _rel_err(gelu, out.cpu()) <= bar
    t = torch.tanh(u)
    dg = 0.5 * (1.0 + t) + 0.5 * preb * (1.0 - t * t) * math.sqrt(2.0 / math.pi) * (1.0 + 3 * 0.044715 * preb ** 2)
    out = K.linear_h3r(xd, wp, N, act=5, aux=aux)
    assert _rel_err(pre * dg, out.cpu()) <= bar
    perm = torch.randperm(M, generator=g).to(torch.int32)
    perm[::5] = -1
    res = torch.randn((M, N), generator=g)
    out2 = torch.full((M, N), 7.0, device=DEV)
    K.linear_h3r(xd, wp, N, out=out2, bias=b.to(DEV), res=res.to(DEV), row_map=perm.to(DEV))
    ref2 = torch.full((M, N), 7.0, dtype=torch.float64)
    keep = perm >= 0
    ref2[perm[keep].long()] = preb[keep] + res.double()[perm[keep].long()]
    assert _rel_err(ref2, out2.cpu()) <= bar
    rs = torch.exp(torch.empty((M, 1)).uniform_(math.log(1e-6), math.log(1e3), generator=g))
    xh = x * rs
    xh[:, 5] *= 1e4
    pre = xh.double() @ wt.double().t()
    out = K.linear_h3r(xh.to(DEV), wp, N).cpu().double()
    rowerr = ((out - pre).norm(dim=1) / pre.norm(dim=1)).max().item()
    row32 = (((xh @ wt.t()).double() - pre).norm(dim=1) / pre.norm(dim=1)).max().item()
    print(f"  heavy-tailed rows: worst row err {rowerr:.3g}, torch fp32 worst row {row32:.3g}")
    assert rowerr <= max(4e-6, 4 * row32)
    # K = 10240 takes the split-K path (eight K ranges, fixed-order reduce): its epilogue
    # with bias, alpha, residual and accumulate
    out4 = torch.full((M, N), 3.0, device=DEV)
    K.linear_h3r(xd, wp, N, out=out4, bias=b.to(DEV), alpha=0.5, res=res.to(DEV), accumulate=1)
    ref4 = 3.0 + 0.5 * (x.double() @ wt.double().t() + b.double()) + res.double()
    assert _rel_err(ref4, out4.cpu()) <= bar


@pytest.mark.parametrize("grid", [(1, 8, 16, 12), (1, 12, 8, 24), (2, 8, 12, 20), (1, 28, 48, 40)])
def test_conv3d_f16x3(grid):
    """fp32 Conv3d 160 -> 160 on fp16 matrix cores (2-plane split with a
    power-of-two scale per tensor, three plane products): forward with bias +
    residual + ReLU, plain forward, dgrad with the ReLU mask on a gradient-sized
    operand (~1e-7, where an unscaled fp16 split underflows), vs float64 -- the
    fp32 kernel's budget (NRMSE <= 2e-6)."""
    K = _K()
    B, D, H, W = grid
    C = 160
    x = _rnd((B, C, D, H, W), 40)
    w = _rnd((C, C, 3, 3, 3), 41) / (27 * C) ** 0.5
    b = _rnd((C,), 42)
    res = _rnd((B, C, D, H, W), 43)
    xd = _to_blocked(x).to(DEV)
    rd = _to_blocked(res).to(DEV)
    planes = K.split2(xd)
    rows = B * D * H * W
    # the planes reassemble x to ~2^-22 (the trailer holds max|x|)
    pl = planes[:rows * 640].view(torch.float16).view(rows, 5, 2, 32).float()
    mx = float(planes[rows * 640:rows * 640 + 4].view(torch.float32)[0])
    assert mx == float(xd.abs().max())
    f, e = math.frexp(mx)
    scale = 2.0 ** (14 - (e - 1 if f == 0.5 else e))         # the kernel's power-of-two scale
    back = (pl[:, :, 0] + pl[:, :, 1]).reshape(rows, C) / scale
    assert nrmse(xd.cpu().double().numpy(), back.cpu().double().numpy()) < 1e-6
    wf = K.conv_pack_f16x3(w.to(DEV), 0)
    out = K.conv3d_f16x3(planes, wf, grid, bias=b.to(DEV), res=rd, res_scale=2.0, relu_out=1)
    ref = F.relu(F.conv3d(x.double(), w.double(), b.double(), padding=1) + 2 * res.double())
    got = _from_blocked(out.cpu(), B, C, D, H, W)
    assert nrmse(ref.numpy(), got.double().numpy()) < 2e-6
    # out_max: the epilogue's atomicMax of |out| = the next split's trailer
    pb = K.planes_alloc(rows, DEV)
    out1 = K.conv3d_f16x3(planes, wf, grid, bias=b.to(DEV), res=rd, res_scale=2.0, relu_out=1,
                          out_max=K.planes_max(pb, rows))
    assert float(pb[rows * 640:rows * 640 + 4].view(torch.float32)[0]) == float(out1.abs().max())
    cs = torch.full((C,), 0.5, device=DEV)                      # colsum accumulates into its target
    K.split2(out1, colsum=cs)
    # fp32 column sums over up to 53760 rows, combined by float atomics in arrival
    # order: ~1e-6 NRMSE vs float64, varying run to run (1.01e-6 seen), so 4e-6
    assert nrmse(out1.double().sum(0).cpu().numpy() + 0.5, cs.double().cpu().numpy()) < 4e-6
    n = rows * 640 + 4                                          # planes + max word (the rest of the trailer is padding)
    assert torch.equal(K.split2(out1, out=pb, have_max=True)[:n], K.split2(out1)[:n])
    out0 = K.conv3d_f16x3(planes, wf, grid)
    ref0 = F.conv3d(x.double(), w.double(), None, padding=1)
    assert nrmse(ref0.numpy(), _from_blocked(out0.cpu(), B, C, D, H, W).double().numpy()) < 2e-6
    # dgrad with the ReLU mask of x, on a gradient-sized operand
    gout = _rnd((B, C, D, H, W), 44) * 1e-7
    gd = _to_blocked(gout).to(DEV)
    dx = K.conv3d_f16x3(K.split2(gd), K.conv_pack_f16x3(w.to(DEV), 1), grid, mask=xd)
    xr_ = x.double().requires_grad_()
    F.conv3d(F.relu(xr_), w.double(), None, padding=1).backward(gout.double())
    assert nrmse(xr_.grad.numpy(), _from_blocked(dx.cpu(), B, C, D, H, W).double().numpy()) < 2e-6
    # wgrad from the planes of x and the gradient-sized g
    dwp = torch.zeros((27, C, C), device=DEV)
    K.conv3d_wgrad_f16x3(planes, K.split2(gd), grid, dwp)
    gw = torch.zeros((C, C, 3, 3, 3), device=DEV)
    K.conv_unpack_grad(dwp, gw, C, C)
    wr_ = w.double().requires_grad_()
    F.conv3d(x.double(), wr_, None, padding=1).backward(gout.double())
    assert nrmse(wr_.grad.numpy(), gw.cpu().double().numpy()) < 2e-6
    # the weight gradient is run-to-run deterministic (raw per-range partials summed in
    # a fixed order, no float atomics) and accumulates into dW
    dwp2 = torch.full((27, C, C), 0.5, device=DEV)
    K.conv3d_wgrad_f16x3(planes, K.split2(gd), grid, dwp2)
    assert torch.equal(dwp2, dwp + 0.5)
    # all-zero input: scale 1, output = bias
    z = K.conv3d_f16x3(K.split2(torch.zeros_like(xd)), wf, grid, bias=b.to(DEV))
    assert torch.equal(z.cpu(), b.expand(rows, C).contiguous())


@pytest.mark.parametrize("grid", [(1, 8, 16, 12), (1, 12, 8, 24), (2, 8, 12, 20), (1, 28, 48, 40)])
def test_conv3d_x6(grid):
    """fp32 Conv3d 160 -> 160 on bf16 matrix cores (3-plane split, six plane
    products): forward with bias + residual + ReLU epilogue and dgrad with the
    ReLU mask, vs float64 on the unrounded fp32 operands -- the fp32 kernel's
    budget (NRMSE <= 2e-6), i.e. fp32 accuracy, not bf16's.  DIAG build only
    (libdlcs_hip_diag.so): the product's fp32 conv is the f16x3 split."""
    K = _K()
    _need_diag("dlcs_conv3d_k3_x6")
    B, D, H, W = grid
    C = 160
    x = _rnd((B, C, D, H, W), 40)
    w = _rnd((C, C, 3, 3, 3), 41) / (27 * C) ** 0.5
    b = _rnd((C,), 42)
    res = _rnd((B, C, D, H, W), 43)
    xd = _to_blocked(x).to(DEV)
    rd = _to_blocked(res).to(DEV)
    planes = K.split3(xd)
    # the planes reassemble x to fp32 precision
    back = planes[0].view(-1, 10, 2, 16).float().sum(2).reshape(-1, C) + planes[1].float()
    assert nrmse(xd.cpu().double().numpy(), back.cpu().double().numpy()) < 1e-7
    out = K.conv3d_x6(planes, K.conv_pack_x6(w.to(DEV), 0), grid, bias=b.to(DEV), res=rd, res_scale=2.0, relu_out=1)
    ref = F.relu(F.conv3d(x.double(), w.double(), b.double(), padding=1) + 2 * res.double())
    got = _from_blocked(out.cpu(), B, C, D, H, W)
    assert nrmse(ref.numpy(), got.double().numpy()) < 2e-6
    # plain forward (no epilogue operands)
    out0 = K.conv3d_x6(planes, K.conv_pack_x6(w.to(DEV), 0), grid)
    ref0 = F.conv3d(x.double(), w.double(), None, padding=1)
    assert nrmse(ref0.numpy(), _from_blocked(out0.cpu(), B, C, D, H, W).double().numpy()) < 2e-6
    # dgrad with the ReLU mask of x
    gout = _rnd((B, C, D, H, W), 44)
    gd = _to_blocked(gout).to(DEV)
    dx = K.conv3d_x6(K.split3(gd), K.conv_pack_x6(w.to(DEV), 1), grid, mask=xd)
    xr_ = x.double().requires_grad_()
    F.conv3d(F.relu(xr_), w.double(), None, padding=1).backward(gout.double())
    assert nrmse(xr_.grad.numpy(), _from_blocked(dx.cpu(), B, C, D, H, W).double().numpy()) < 2e-6
    # wgrad from the planes of x and g
    dwp = torch.zeros((27, C, C), device=DEV)
    K.conv3d_wgrad_x6(planes, K.split3(gd), grid, dwp)
    gw = torch.zeros((C, C, 3, 3, 3), device=DEV)
    K.conv_unpack_grad(dwp, gw, C, C)
    wr_ = w.double().requires_grad_()
    F.conv3d(x.double(), wr_, None, padding=1).backward(gout.double())
    assert nrmse(wr_.grad.numpy(), gw.cpu().double().numpy()) < 2e-6


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1.5e-2)])
@pytest.mark.parametrize("cin,cout", [(4, 160), (160, 4)])
@pytest.mark.parametrize("grid", [(1, 8, 16, 12), (2, 4, 12, 20)])
def test_conv3d_wgrad_thin(dtype, tol, cin, cout, grid):
    """The regularizer's thin ends (SFE 4->160, final 160->4) without ReLU
    prologue: bf16 takes the im2col-of-the-thin-side kernel."""
    K = _K()
    B, D, H, W = grid
    x = _rnd((B, cin, D, H, W), 40)
    g = _rnd((B, cout, D, H, W), 41)
    xr = _pad_cols(_to_blocked(x), max(8, cin)).to(DEV, dtype)
    gr = _pad_cols(_to_blocked(g), max(8, cout)).to(DEV, dtype)
    xq = _from_blocked(xr[:, :cin].float().cpu(), B, cin, D, H, W)
    gq = _from_blocked(gr[:, :cout].float().cpu(), B, cout, D, H, W)
    dwp = torch.zeros((27, K.pad32(cout), K.pad32(cin)), device=DEV)
    K.conv3d_wgrad(xr, cin, 0, gr, cout, grid, dwp)
    gw = torch.zeros((cout, cin, 3, 3, 3), device=DEV)
    K.conv_unpack_grad(dwp, gw, cout, cin)
    w_ = torch.zeros((cout, cin, 3, 3, 3), dtype=torch.float64, requires_grad=True)
    F.conv3d(xq.double(), w_, None, padding=1).backward(gq.double())
    assert nrmse(w_.grad.numpy(), gw.cpu().double().numpy()) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1.5e-2)])
@pytest.mark.parametrize("grid", [(1, 8, 16, 12), (2, 4, 12, 20)])
@pytest.mark.parametrize("out_dtype", [torch.float32, None])
def test_conv3d_thin_in(dtype, tol, grid, out_dtype):
    """4 -> 160 without ReLU prologue (SFE forward; the final conv's dgrad has the
    same shape with a mask): bf16 takes the thin-input kernel."""
    K = _K()
    B, D, H, W = grid
    cin, C = 4, 160
    x = _rnd((B, cin, D, H, W), 50)
    w = _rnd((C, cin, 3, 3, 3), 51) / (27 * cin) ** 0.5
    b = _rnd((C,), 52)
    res = _rnd((B, C, D, H, W), 53)
    m = _rnd((B, C, D, H, W), 54)
    xd = _pad_cols(_to_blocked(x), 8).to(DEV, dtype)
    rd = _to_blocked(res).to(DEV, dtype)
    md = _to_blocked(m).to(DEV, dtype)
    xq = _from_blocked(xd[:, :cin].float().cpu(), B, cin, D, H, W)
    rq = _from_blocked(rd.float().cpu(), B, C, D, H, W)
    mq = _from_blocked(md.float().cpu(), B, C, D, H, W)
    wp = K.conv_pack(w.to(DEV), dtype, 0)
    out = K.conv3d(xd, cin, wp, C, C, grid, bias=b.to(DEV), res=rd, res_scale=0.5, mask=md, relu_out=1,
                   out_dtype=out_dtype)
    pre = F.conv3d(xq.double(), w.to(dtype).double(), b.double(), padding=1) * (mq > 0).double()
    ref = F.relu(pre + 0.5 * rq.double())
    got = _from_blocked(out.float().cpu(), B, C, D, H, W)
    assert nrmse(ref.numpy(), got.double().numpy()) < (tol if out_dtype is not None or dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1.5e-2)])
@pytest.mark.parametrize("grid", [(1, 8, 16, 12), (2, 4, 12, 20)])
@pytest.mark.parametrize("out_dtype", [torch.float32, None])
def test_conv3d_thin_out(dtype, tol, grid, out_dtype):
    """160 -> 4, plain (final conv forward with bias; SFE dgrad = the same on the
    transposed-flipped pack): bf16 takes the output-shift kernel."""
    K = _K()
    B, D, H, W = grid
    C, co = 160, 4
    x = _rnd((B, C, D, H, W), 60)
    w = _rnd((co, C, 3, 3, 3), 61) / (27 * C) ** 0.5
    b = _rnd((co,), 62)
    xd = _to_blocked(x).to(DEV, dtype)
    xq = _from_blocked(xd.float().cpu(), B, C, D, H, W)
    wp = K.conv_pack(w.to(DEV), dtype, 0)
    out = K.conv3d(xd, C, wp, co, 8, grid, bias=b.to(DEV), out_dtype=out_dtype)
    ref = F.conv3d(xq.double(), w.to(dtype).double(), b.double(), padding=1)
    got = _from_blocked(out[:, :co].float().cpu(), B, co, D, H, W)
    assert nrmse(ref.numpy(), got.double().numpy()) < tol
    # dgrad of a 4 -> 160 conv: dx = conv_T(g)
    w2 = _rnd((C, co, 3, 3, 3), 63) / (27 * co) ** 0.5
    wd = K.conv_pack(w2.to(DEV), dtype, 1)
    dx = K.conv3d(xd, C, wd, co, 8, grid, out_dtype=out_dtype)
    xr_ = torch.zeros((B, co, D, H, W), dtype=torch.float64, requires_grad=True)
    F.conv3d(xr_, w2.to(dtype).double(), None, padding=1).backward(xq.double())
    got = _from_blocked(dx[:, :co].float().cpu(), B, co, D, H, W)
    assert nrmse(xr_.grad.numpy(), got.double().numpy()) < tol


@pytest.mark.parametrize("grid", [(1, 8, 16, 12), (2, 4, 12, 20), (1, 28, 48, 40)])
def test_conv3d_thin_f16x3(grid):
    """The fp32 thin ends (SFE 4 -> 160, final 160 -> 4) on fp16 matrix cores
    (dlcs_conv3d_thin_f16x3 / _wgrad_f16x3, in-register 2-plane split): thin-input
    forward with bias + mask + residual + ReLU + out_max, thin-output forward with
    bias, both dgrads (mode-1 packs), both weight gradients on a gradient-sized
    operand (~1e-7) and the fused SFE bias column sums -- vs float64 at the fp32
    kernels' budget (NRMSE <= 2e-6).  The 4-channel volumes carry NaN in their
    padding columns (never read into a product)."""
    K = _K()
    B, D, H, W = grid
    C, e = 160, 4
    rows = B * D * H * W
    x4 = _rnd((B, e, D, H, W), 70)
    x160 = _rnd((B, C, D, H, W), 71)
    w_sfe = _rnd((C, e, 3, 3, 3), 72) / (27 * e) ** 0.5
    w_fin = _rnd((e, C, 3, 3, 3), 73) / (27 * C) ** 0.5
    b160, b4 = _rnd((C,), 74), _rnd((e,), 75)
    res, m = _rnd((B, C, D, H, W), 76), _rnd((B, C, D, H, W), 77)
    g160 = _rnd((B, C, D, H, W), 78) * 1e-7
    g4 = _rnd((B, e, D, H, W), 79) * 1e-7

    def thin_dev(t):
        r = torch.full((rows, 8), float("nan"))
        r[:, :e] = _to_blocked(t)
        return r.to(DEV)
    x4d, g4d = thin_dev(x4), thin_dev(g4)
    x160d, g160d = _to_blocked(x160).to(DEV), _to_blocked(g160).to(DEV)
    rd, md = _to_blocked(res).to(DEV), _to_blocked(m).to(DEV)
    back = lambda o, c: _from_blocked(o[:, :c].cpu(), B, c, D, H, W).double().numpy()
    # thin input forward (SFE): 4 -> 160 with the full epilogue and out_max
    wp = K.thin_pack_f16x3(K.conv_pack(w_sfe.to(DEV), torch.float32, 0), C, e, 0)
    omax = torch.zeros((1,), dtype=torch.int32, device=DEV)
    out = K.conv3d_thin_f16x3(x4d, e, K.absmax(x4d[:, :e].contiguous()), wp, C, C, grid, bias=b160.to(DEV), mask=md,
                              res=rd, res_scale=0.5, relu_out=1, out_max=omax)
    pre = F.conv3d(x4.double(), w_sfe.double(), b160.double(), padding=1) * (m > 0).double()
    ref = F.relu(pre + 0.5 * res.double())
    assert nrmse(ref.numpy(), back(out, C)) < 2e-6
    assert float(omax.view(torch.float32)[0]) == float(out.abs().max())
    # thin input dgrad (final conv): g_h = conv_T(g4) masked
    wdp = K.thin_pack_f16x3(K.conv_pack(w_fin.to(DEV), torch.float32, 1), C, e, 0)
    gh = K.conv3d_thin_f16x3(g4d, e, K.absmax(_to_blocked(g4).to(DEV)), wdp, C, C, grid, mask=md)
    xr_ = x160.double().requires_grad_()
    F.conv3d(xr_, w_fin.double(), None, padding=1).backward(g4.double())
    assert nrmse((xr_.grad * (m > 0)).numpy(), back(gh, C)) < 2e-6
    # the same as planes only with the column sums (the final conv's g_h and the DFE bias
    # gradient): scale from the bound ||W_fin^T||_inf max|g4|
    g4m = K.absmax(_to_blocked(g4).to(DEV))
    nfin = K.abs_row_sum_max(w_fin.to(DEV), C, 27, 27, n_outer=e, outer_stride=27 * C)
    ph = K.planes_alloc(rows, DEV)
    K.planes_bound(ph, rows, m0=g4m, n0=nfin)
    cs = torch.full((C,), 0.5, device=DEV)
    assert K.conv3d_thin_f16x3(g4d, e, g4m, wdp, C, C, grid, mask=md, out_planes=ph, planes_only=True,
                               colsum=cs) is None
    back_ph, bnd = _planes_back(ph, rows)
    assert bnd >= float(gh.abs().max())
    err = (back_ph.double() - gh.double()).abs()
    assert bool((err <= 2.0 ** -21 * gh.double().abs() + 2.0 ** -37 * bnd).all())
    assert nrmse(gh.double().sum(0).cpu().numpy() + 0.5, cs.double().cpu().numpy()) < 1e-6
    # thin output forward (final conv) 160 -> 4 with bias
    wo = K.thin_pack_f16x3(K.conv_pack(w_fin.to(DEV), torch.float32, 0), e, C, 1)
    o = K.conv3d_thin_f16x3(x160d, C, K.absmax(x160d), wo, e, 8, grid, bias=b4.to(DEV))
    ref = F.conv3d(x160.double(), w_fin.double(), b4.double(), padding=1)
    assert nrmse(ref.numpy(), back(o, e)) < 2e-6
    # thin output dgrad (SFE): g_u = conv_T(g160)
    wso = K.thin_pack_f16x3(K.conv_pack(w_sfe.to(DEV), torch.float32, 1), e, C, 1)
    gu = K.conv3d_thin_f16x3(g160d, C, K.absmax(g160d), wso, e, 8, grid)
    xr_ = x4.double().requires_grad_()
    F.conv3d(xr_, w_sfe.double(), None, padding=1).backward(g160.double())
    assert nrmse(xr_.grad.numpy(), back(gu, e)) < 2e-6
    # weight gradients: SFE (x4, g160) with the bias column sums, final (x160, g4)
    dwp = torch.zeros((27, C, K.pad32(e)), device=DEV)
    cs = torch.full((C,), 0.25, device=DEV)
    K.conv3d_thin_wgrad_f16x3(x4d, e, K.absmax(_to_blocked(x4).to(DEV)), g160d, C, K.absmax(g160d), grid, dwp,
                              colsum=cs)
    gw = torch.zeros((C, e, 3, 3, 3), device=DEV)
    K.conv_unpack_grad(dwp, gw, C, e)
    w_ = w_sfe.double().requires_grad_()
    F.conv3d(x4.double(), w_, None, padding=1).backward(g160.double())
    assert nrmse(w_.grad.numpy(), gw.cpu().double().numpy()) < 2e-6
    assert nrmse(g160.double().sum((0, 2, 3, 4)).numpy() + 0.25, cs.cpu().double().numpy()) < 4e-6
    dwp = torch.zeros((27, K.pad32(e), C), device=DEV)
    K.conv3d_thin_wgrad_f16x3(x160d, C, K.absmax(x160d), g4d, e, K.absmax(_to_blocked(g4).to(DEV)), grid, dwp)
    gw = torch.zeros((e, C, 3, 3, 3), device=DEV)
    K.conv_unpack_grad(dwp, gw, e, C)
    w_ = w_fin.double().requires_grad_()
    F.conv3d(x160.double(), w_, None, padding=1).backward(g4.double())
    assert nrmse(w_.grad.numpy(), gw.cpu().double().numpy()) < 2e-6


@pytest.mark.parametrize("grid", [(1, 8, 16, 12), (2, 4, 12, 20), (1, 12, 20, 8), (1, 28, 48, 40)])
def test_conv3d_thin_planes(grid):
    """The thin ends from split2 planes of the 160-channel operand
    (dlcs_conv3d_thin_out_planes_f16x3 / _thin_wgrad_planes_f16x3; odd patch
    counts in y exercise the partial 1 x 2 x 1-patch tiles): final-conv forward
    with bias + ReLU + accumulate, SFE input gradient, both weight gradients on a
    gradient-sized operand (~1e-7) -- vs float64 at the fp32 kernels' budget
    (NRMSE <= 2e-6); the weight gradients are run-to-run deterministic."""
    K = _K()
    B, D, H, W = grid
    C, e = 160, 4
    rows = B * D * H * W
    x4 = _rnd((B, e, D, H, W), 80)
    x160 = _rnd((B, C, D, H, W), 81)
    w_sfe = _rnd((C, e, 3, 3, 3), 82) / (27 * e) ** 0.5
    w_fin = _rnd((e, C, 3, 3, 3), 83) / (27 * C) ** 0.5
    b4 = _rnd((e,), 85)
    g160 = _rnd((B, C, D, H, W), 88) * 1e-7
    g4 = _rnd((B, e, D, H, W), 89) * 1e-7

    def thin_dev(t):
        r = torch.full((rows, 8), float("nan"))
        r[:, :e] = _to_blocked(t)
        return r.to(DEV)
    x4d, g4d = thin_dev(x4), thin_dev(g4)
    px, pg = K.split2(_to_blocked(x160).to(DEV)), K.split2(_to_blocked(g160).to(DEV))
    back = lambda o, c: _from_blocked(o[:, :c].cpu(), B, c, D, H, W).double().numpy()
    # thin output forward (final conv) 160 -> 4: bias, accumulate onto 0.5, ReLU
    wo = K.thin_pack_f16x3(K.conv_pack(w_fin.to(DEV), torch.float32, 0), e, C, 1)
    o = torch.full((rows, 8), 0.5, device=DEV)
    K.conv3d_thin_out_planes(px, wo, e, 8, grid, bias=b4.to(DEV), out=o, accumulate=1, relu_out=1)
    ref = F.relu(F.conv3d(x160.double(), w_fin.double(), b4.double(), padding=1)) + 0.5
    assert nrmse(ref.numpy(), back(o, e)) < 2e-6
    # thin output dgrad (SFE): g_u = conv_T(g160)
    wso = K.thin_pack_f16x3(K.conv_pack(w_sfe.to(DEV), torch.float32, 1), e, C, 1)
    gu = K.conv3d_thin_out_planes(pg, wso, e, 8, grid)
    xr_ = x4.double().requires_grad_()
    F.conv3d(xr_, w_sfe.double(), None, padding=1).backward(g160.double())
    assert nrmse(xr_.grad.numpy(), back(gu, e)) < 2e-6
    # weight gradients: SFE (planes = g160, thin = x4), final (planes = x160, thin = g4)
    dwp = torch.zeros((27, C, K.pad32(e)), device=DEV)
    K.conv3d_thin_wgrad_planes(pg, x4d, e, K.absmax(_to_blocked(x4).to(DEV)), 1, grid, dwp)
    gw = torch.zeros((C, e, 3, 3, 3), device=DEV)
    K.conv_unpack_grad(dwp, gw, C, e)
    w_ = w_sfe.double().requires_grad_()
    F.conv3d(x4.double(), w_, None, padding=1).backward(g160.double())
    assert nrmse(w_.grad.numpy(), gw.cpu().double().numpy()) < 2e-6
    dwp2 = torch.zeros_like(dwp)
    K.conv3d_thin_wgrad_planes(pg, x4d, e, K.absmax(_to_blocked(x4).to(DEV)), 1, grid, dwp2)
    assert torch.equal(dwp, dwp2)
    dwp = torch.zeros((27, K.pad32(e), C), device=DEV)
    K.conv3d_thin_wgrad_planes(px, g4d, e, K.absmax(_to_blocked(g4).to(DEV)), 0, grid, dwp)
    gw = torch.zeros((e, C, 3, 3, 3), device=DEV)
    K.conv_unpack_grad(dwp, gw, e, C)
    w_ = w_fin.double().requires_grad_()
    F.conv3d(x160.double(), w_, None, padding=1).backward(g4.double())
    assert nrmse(w_.grad.numpy(), gw.cpu().double().numpy()) < 2e-6


def _pad_cols(r, ld):
    if r.shape[1] == ld:
        return r
    out = torch.zeros((r.shape[0], ld))
    out[:, :r.shape[1]] = r
    return out


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layernorm_gather(dtype):
    K = _K()
    rows, C = 500, 160
    x = _rnd((rows, C), 20)
    gam, bet = 1 + 0.1 * _rnd((C,), 21), 0.1 * _rnd((C,), 22)
    idx = torch.randperm(rows, generator=torch.Generator().manual_seed(3)).to(torch.int32)
    idx[:7] = -1
    out, mean, rstd = K.layernorm_fwd(x.to(DEV), gam.to(DEV), bet.to(DEV), rows, src_map=idx.to(DEV),
                                      out_dtype=dtype)
    xs = torch.where(idx[:, None] >= 0, x[idx.clamp(min=0).long()], torch.zeros(1))
    ref = F.layer_norm(xs.double(), (C,), gam.double(), bet.double(), 1e-5)
    ref[:7] = 0
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    assert nrmse(ref.numpy(), out.float().cpu().double().numpy()) < tol
    # backward
    dy = _rnd((rows, C), 23)
    dx = torch.zeros((rows, C), device=DEV)
    dg = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)
    K.layernorm_bwd(dy.to(DEV), x.to(DEV), gam.to(DEV), mean, rstd, dx, dg, db, src_map=idx.to(DEV))
    xr = x.double().requires_grad_()
    g_ = gam.double().requires_grad_()
    b_ = bet.double().requires_grad_()
    xs = xr[idx.clamp(min=0).long()]
    o = F.layer_norm(xs, (C,), g_, b_, 1e-5)
    keep = (idx >= 0).double()[:, None]
    (o * dy.double() * keep).sum().backward()
    assert nrmse(xr.grad.numpy(), dx.cpu().double().numpy()) < 1e-6
    assert nrmse(g_.grad.numpy(), dg.cpu().double().numpy()) < 1e-6
    assert nrmse(b_.grad.numpy(), db.cpu().double().numpy()) < 1e-6


def _attn_reference(qkv, table, labels, mask, nwin, N, heads, hd, window, scale, dout, round_q=True):
    """float64 window attention fwd + bwd on the (already rounded) operands:
    vst:139-170 with the relative-position bias of vst:111-129 and the -100 shift
    mask of vst:342-355 (from region labels) or an explicit additive mask."""
    import itertools
    wd, wh, ww = window
    coords = torch.tensor(list(itertools.product(range(wd), range(wh), range(ww))))[:N]
    rel = coords[:, None, :] - coords[None, :, :]
    idx = (rel[..., 0] + wd - 1) * (2 * wh - 1) * (2 * ww - 1) + (rel[..., 1] + wh - 1) * (2 * ww - 1) + rel[..., 2] + ww - 1
    C = heads * hd
    x = qkv.double().view(nwin, N, 3, heads, hd).permute(2, 0, 3, 1, 4)        # [3, nw, h, N, hd]
    q = x[0] * scale
    if round_q:
        q = q.to(torch.bfloat16).double()                                       # the bf16 kernels round scale*q
    q = q.requires_grad_()
    k = x[1].clone().requires_grad_()
    v = x[2].clone().requires_grad_()
    tb = table.double().clone().requires_grad_()
    s = q @ k.transpose(-1, -2) + tb[idx.reshape(-1)].reshape(N, N, heads).permute(2, 0, 1)[None]
    if labels is not None:
        lab = labels.view(nwin, N)
        s = s + torch.where(lab[:, None, :, None] != lab[:, None, None, :], -100.0, 0.0).double()
    if mask is not None:
        s = s + mask.double()[torch.arange(nwin) % mask.shape[0]][:, None]
    o = torch.softmax(s, -1) @ v                                                # [nw, h, N, hd]
    o.backward(dout.double().view(nwin, N, heads, hd).permute(0, 2, 1, 3))
    out = o.permute(0, 2, 1, 3).reshape(nwin * N, C)
    dq = (q.grad * scale).permute(0, 2, 1, 3).reshape(nwin * N, C)
    dk = k.grad.permute(0, 2, 1, 3).reshape(nwin * N, C)
    dv = v.grad.permute(0, 2, 1, 3).reshape(nwin * N, C)
    return out.detach(), torch.cat([dq, dk, dv], 1).detach(), tb.grad.detach()


@pytest.mark.parametrize("case", ["labels", "mask", "plain"])
def test_window_attention_bf16_kernels(case):
    """bf16 fused window attention forward and the split backward (dK/dV/table
    and dQ kernels) against float64 attention on the same bf16 operands."""
    K = _K()
    nwin, N, heads, hd, window = 3, 448, 8, 20, (7, 8, 8)
    C, scale = heads * hd, hd ** -0.5
    qkv = (_rnd((nwin * N, 3 * C), 60) * 1.5).to(torch.bfloat16)
    table = _rnd((13 * 15 * 15, heads), 61) * 0.3
    labels = (_rnd((nwin * N,), 62).abs() * 2).int().clamp(max=3) if case == "labels" else None
    mask = (torch.where(_rnd((2, N, N), 63) > 0.8, -100.0, 0.0)) if case == "mask" else None
    dout = _rnd((nwin * N, C), 64).to(torch.bfloat16)
    ref_o, ref_dqkv, ref_dt = _attn_reference(qkv, table, labels, mask, nwin, N, heads, hd, window, scale, dout)
    qd, td = qkv.to(DEV), table.to(DEV)
    ld = labels.to(DEV) if labels is not None else None
    md = mask.to(DEV) if mask is not None else None
    out, lse = K.attn_fwd(qd, td, ld, nwin, N, heads, hd, window, scale, mask=md, mask_nw=2 if md is not None else 0)
    assert nrmse(ref_o.numpy(), out.double().cpu().numpy()) < 1e-2
    dt = torch.zeros_like(td)
    # the backward sees the bf16 output the forward produced (as in the block)
    dqkv = K.attn_bwd(qd, out, dout.to(DEV), lse, td, ld, dt, nwin, N, heads, hd, window, scale,
                      mask=md, mask_nw=2 if md is not None else 0)
    got = dqkv.double().cpu()
    for name, sl in (("dq", slice(0, C)), ("dk", slice(C, 2 * C)), ("dv", slice(2 * C, 3 * C))):
        assert nrmse(ref_dqkv[:, sl].numpy(), got[:, sl].numpy()) < 2e-2, name
    assert nrmse(ref_dt.numpy(), dt.double().cpu().numpy()) < 2e-2


@pytest.mark.parametrize("case,N", [("labels", 448), ("plain", 448), ("mask", 448), ("labels", 200),
                                    ("plain", 96), ("labels", 32), ("mask", 100)])
def test_window_attention_f32_kernels(case, N):
    """fp32 window attention (head dim 20: the 32x32x2 f32 MFMA kernels) forward
    and backward vs float64 attention, full and ragged token counts; NRMSE <= 1e-5."""
    K = _K()
    nwin, heads, hd, window = 3, 8, 20, (7, 8, 8)
    C, scale = heads * hd, hd ** -0.5
    qkv = _rnd((nwin * N, 3 * C), 65) * 1.5
    table = _rnd((13 * 15 * 15, heads), 66) * 0.3
    labels = (_rnd((nwin * N,), 67).abs() * 2).int().clamp(max=3) if case == "labels" else None
    mask = (torch.where(_rnd((2, N, N), 68) > 0.8, -100.0, 0.0)) if case == "mask" else None
    dout = _rnd((nwin * N, C), 69)
    ref_o, ref_dqkv, ref_dt = _attn_reference(qkv, table, labels, mask, nwin, N, heads, hd, window, scale, dout,
                                              round_q=False)
    qd, td = qkv.to(DEV), table.to(DEV)
    ld = labels.to(DEV) if labels is not None else None
    md = mask.to(DEV) if mask is not None else None
    out, lse = K.attn_fwd(qd, td, ld, nwin, N, heads, hd, window, scale, mask=md, mask_nw=2 if md is not None else 0)
    assert nrmse(ref_o.numpy(), out.double().cpu().numpy()) < 1e-5
    dt = torch.zeros_like(td)
    dqkv = K.attn_bwd(qd, out, dout.to(DEV), lse, td, ld, dt, nwin, N, heads, hd, window, scale,
                      mask=md, mask_nw=2 if md is not None else 0)
    got = dqkv.double().cpu()
    for name, sl in (("dq", slice(0, C)), ("dk", slice(C, 2 * C)), ("dv", slice(2 * C, 3 * C))):
        assert nrmse(ref_dqkv[:, sl].numpy(), got[:, sl].numpy()) < 1e-5, name
    assert nrmse(ref_dt.numpy(), dt.double().cpu().numpy()) < 1e-5


def _attn_fwd_dtype(qkv, table, labels, mask, nwin, N, heads, hd, window, scale, dt, dout=None):
    """Window attention evaluated in dtype dt: out [rows, C], lse [nwin, heads, N] and,
    with dout, (dqkv [rows, 3C], dtable)."""
    import itertools
    wd, wh, ww = window
    coords = torch.tensor(list(itertools.product(range(wd), range(wh), range(ww))))[:N]
    rel = coords[:, None, :] - coords[None, :, :]
    idx = (rel[..., 0] + wd - 1) * (2 * wh - 1) * (2 * ww - 1) + (rel[..., 1] + wh - 1) * (2 * ww - 1) + rel[..., 2] + ww - 1
    xq = qkv.to(dt).clone().requires_grad_()
    tb = table.to(dt).clone().requires_grad_()
    x = xq.view(nwin, N, 3, heads, hd).permute(2, 0, 3, 1, 4)
    s = (x[0] * scale) @ x[1].transpose(-1, -2) + tb[idx.reshape(-1)].reshape(N, N, heads).permute(2, 0, 1)[None]
    if labels is not None:
        lab = labels.view(nwin, N)
        s = s + torch.where(lab[:, None, :, None] != lab[:, None, None, :], -100.0, 0.0).to(dt)
    if mask is not None:
        s = s + mask.to(dt)[torch.arange(nwin) % mask.shape[0]][:, None]
    o = (torch.softmax(s, -1) @ x[2]).permute(0, 2, 1, 3).reshape(nwin * N, heads * hd)
    lse = torch.logsumexp(s, -1)
    if dout is None:
        return o.detach(), lse.detach()
    o.backward(dout.to(dt))
    return o.detach(), lse.detach(), xq.grad, tb.grad


@pytest.mark.parametrize("case,N,tail", [("labels", 448, False), ("plain", 96, False), ("mask", 100, False),
                                         ("labels", 200, False), ("labels", 448, True), ("plain", 448, True)])
def test_window_attention_h3_floor(case, N, tail):
    """The fp32 window attention on the f16 split (attention_h3.inc: every product
    as three fp16 plane products with power-of-two scales) held to fp32's own
    distance from float64: output, log-sum-exp, dQ, dK, dV and the table gradient,
    err(HIP) <= max(1e-6, 4 x err(torch fp32)) (1e-5 floor for 'tail').  'tail': heavy-tailed operands --
    one channel of every head's q, k, v x 8 and a quarter of the tokens at 2^-20
    (the per-window image scales, per-row register scales, dS bound scale)."""
    K = _K()
    nwin, heads, hd, window = 3, 8, 20, (7, 8, 8)
    C, scale = heads * hd, hd ** -0.5
    qkv = _rnd((nwin * N, 3 * C), 165) * 1.5
    if tail:
        qkv.view(nwin * N, 3, heads, hd)[:, :, :, 3] *= 8.0
        qkv[torch.arange(nwin * N) % 4 == 1] *= 2.0 ** -20
    table = _rnd((13 * 15 * 15, heads), 166) * 0.3
    labels = (_rnd((nwin * N,), 167).abs() * 2).int().clamp(max=3) if case == "labels" else None
    mask = (torch.where(_rnd((2, N, N), 168) > 0.8, -100.0, 0.0)) if case == "mask" else None
    dout = _rnd((nwin * N, C), 169)
    r64 = _attn_fwd_dtype(qkv, table, labels, mask, nwin, N, heads, hd, window, scale, torch.float64, dout)
    r32 = _attn_fwd_dtype(qkv, table, labels, mask, nwin, N, heads, hd, window, scale, torch.float32, dout)
    ld = labels.to(DEV) if labels is not None else None
    md = mask.to(DEV) if mask is not None else None
    qd, td = qkv.to(DEV), table.to(DEV)
    mnw = 2 if md is not None else 0
    out, lse = K.attn_fwd(qd, td, ld, nwin, N, heads, hd, window, scale, mask=md, mask_nw=mnw)
    dt = torch.zeros_like(td)
    dqkv = K.attn_bwd(qd, out, dout.to(DEV), lse, td, ld, dt, nwin, N, heads, hd, window, scale, mask=md, mask_nw=mnw)
    got = (out, lse.view(nwin, heads, N), dqkv[:, :C], dqkv[:, C:2 * C], dqkv[:, 2 * C:], dt)
    refs = (r64[0], r64[1], r64[2][:, :C], r64[2][:, C:2 * C], r64[2][:, 2 * C:], r64[3])
    f32s = (r32[0], r32[1], r32[2][:, :C], r32[2][:, C:2 * C], r32[2][:, 2 * C:], r32[3])
    for name, ref, f32, g in zip(("out", "lse", "dq", "dk", "dv", "dtable"), refs, f32s, got):
        e32 = nrmse(ref.numpy(), f32.double().numpy())
        eh = nrmse(ref.numpy(), g.double().cpu().numpy())
        print(f"h3 attention {case} N={N} tail={tail} {name}: HIP {eh:.3g}, torch fp32 {e32:.3g}")
        # benign operands: within 4x of torch's own fp32 distance (1e-6 floor); the
        # heavy-tailed case: the repo-wide f64-floor bound max(1e-5, 4 x fp32) -- the
        # f16 plane pair represents each operand to 22 bits, fp32 to 24, which shows
        # in dV there (P = exp2(s - lse) carries the 2^-22 error of |s| ~ 40)
        assert eh <= max(1e-5 if tail else 1e-6, 4 * e32), name


def test_window_attention_large_window_fallback():
    """A window whose f16 plane images do not fit the LDS (8 x 8 x 8 = 512 tokens: the
    fp16-split dK / dV kernel needs 181 KB) runs the f32-MFMA kernels for those
    launches (the forward still fits): output and gradients vs float64 (NRMSE <= 1e-5)."""
    K = _K()
    nwin, heads, hd, window = 2, 8, 20, (8, 8, 8)
    N = 8 * 8 * 8
    C, scale = heads * hd, hd ** -0.5
    nrel = 15 * 15 * 15
    qkv = _rnd((nwin * N, 3 * C), 175) * 1.5
    table = _rnd((nrel, heads), 176) * 0.3
    labels = (_rnd((nwin * N,), 177).abs() * 2).int().clamp(max=3)
    dout = _rnd((nwin * N, C), 179)
    r64 = _attn_fwd_dtype(qkv, table, labels, None, nwin, N, heads, hd, window, scale, torch.float64, dout)
    qd, td, ld = qkv.to(DEV), table.to(DEV), labels.to(DEV)
    out, lse = K.attn_fwd(qd, td, ld, nwin, N, heads, hd, window, scale)
    dt = torch.zeros_like(td)
    dqkv = K.attn_bwd(qd, out, dout.to(DEV), lse, td, ld, dt, nwin, N, heads, hd, window, scale)
    assert nrmse(r64[0].numpy(), out.double().cpu().numpy()) < 1e-5
    assert nrmse(r64[2].numpy(), dqkv.double().cpu().numpy()) < 1e-5
    assert nrmse(r64[3].numpy(), dt.double().cpu().numpy()) < 1e-5


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_gemm_dw_grouped(dtype):
    """Grouped weight gradients dW += A^T B and the folded bias gradient, bf16 or
    fp32 operands, fp32 partial sums (no atomics) vs float64 on the same operands."""
    K = _K()
    T = 13440
    shapes = [(160, 640, 0), (640, 160, 0), (480, 160, 160), (10240, 160, 160)]
    groups, refs = [], []
    for i, (M, N, per) in enumerate(shapes):
        A = (_rnd((T, M), 70 + i) * 0.5).to(dtype)
        B = _rnd((T, N), 80 + i).to(dtype)
        dW0 = _rnd((M, N), 90 + i)
        P = per or M
        db0 = _rnd((P,), 95 + i)
        refW = dW0.double() + A.double().t() @ B.double()
        refb = db0.double() + A.double().sum(0).view(-1, P).sum(0)
        groups.append([A.to(DEV), B.to(DEV), dW0.to(DEV), db0.to(DEV), per])
        refs.append((refW, refb))
    K.gemm_dw_grouped(T, groups[:3])           # one launch, three problems (a Swin block's shapes)
    K.gemm_dw_grouped(T, groups[3:])           # the patch-unembed shape with its 64-fold bias
    for (refW, refb), g in zip(refs, groups):
        assert nrmse(refW.numpy(), g[2].double().cpu().numpy()) < 1e-5
        assert nrmse(refb.numpy(), g[3].double().cpu().numpy()) < 1e-5


def test_gemm_dw_grouped_fp32_edge_tiles():
    """fp32 grouped weight gradients with M, N not multiples of the 160 tile (the
    DiT / Latte Linears: D = 384, 3 D, 4 D, 6 D; edge tiles zero-filled on load,
    clipped on store) vs float64, with the bias gradient, in one launch."""
    K = _K()
    T = 23040
    shapes = [(1152, 384), (384, 1536), (1536, 384), (2304, 384)]
    groups, refs = [], []
    for i, (M, N) in enumerate(shapes):
        A = _rnd((T, M), 270 + i) * 0.5
        B = _rnd((T, N), 280 + i)
        dW0 = _rnd((M, N), 290 + i)
        db0 = _rnd((M,), 295 + i)
        refs.append((dW0.double() + A.double().t() @ B.double(), db0.double() + A.double().sum(0)))
        groups.append([A.to(DEV), B.to(DEV), dW0.to(DEV), db0.to(DEV), 0])
    assert K.dw_grouped_ok(T, [(g[0], g[1]) for g in groups])
    K.gemm_dw_grouped(T, groups)
    for (refW, refb), g in zip(refs, groups):
        assert nrmse(refW.numpy(), g[2].double().cpu().numpy()) < 1e-5
        assert nrmse(refb.numpy(), g[3].double().cpu().numpy()) < 1e-5


def test_gemm_dw_grouped_fp32_range():
    """fp32 grouped weight gradients (the fp16 2-plane h3 kernel, scale per column
    and 32-token step) at fp32 accuracy over a 1e9 dynamic range: A's columns scaled
    by 10^u, u in [-6, 3], B's by 10^v, v in [-4, 1] (tiny and huge gradient
    channels in one launch).  Per dW row and per bias entry, the error vs float64
    stays within 4x torch's own fp32 GEMM error (plus 1e-7 of the row norm) -- a
    per-tensor-scaled fp16 split would lose the small columns."""
    K = _K()
    T = 13440
    gen = torch.Generator().manual_seed(5)
    shapes = [(160, 640), (640, 160), (480, 160)]
    groups, refs = [], []
    for i, (M, N) in enumerate(shapes):
        A = _rnd((T, M), 170 + i) * torch.pow(10.0, torch.empty(M).uniform_(-6, 3, generator=gen))
        B = _rnd((T, N), 180 + i) * torch.pow(10.0, torch.empty(N).uniform_(-4, 1, generator=gen))
        dW0 = torch.zeros((M, N))
        db0 = torch.zeros((M,))
        refs.append((A.double().t() @ B.double(), A.double().sum(0), (A.t() @ B).double(), A.double().abs().sum(0)))
        groups.append([A.to(DEV), B.to(DEV), dW0.to(DEV), db0.to(DEV), 0])
    K.gemm_dw_grouped(T, groups)
    for (refW, refb, t32, asum), g in zip(refs, groups):
        got = g[2].double().cpu()
        rn = refW.norm(dim=1, keepdim=True)
        err = ((got - refW).norm(dim=1, keepdim=True) / rn).squeeze(1)
        terr = ((t32 - refW).norm(dim=1, keepdim=True) / rn).squeeze(1)
        assert bool((err <= 4 * terr + 1e-7).all()), float((err / (terr + 1e-12)).max())
        # bias: fp32 summation of T terms, bounded by T eps sum |a| per column
        gb = g[3].double().cpu()
        assert bool(((gb - refb).abs() <= T * 6e-8 * asum).all())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("T", [64, 128, 1024])
def test_gemm_dw_grouped_wide(T, dtype):
    """The PatchGAN patch-conv dW shape (patchgan.py _backward): M = 160 output
    channels, N = 64*160 = 10240 patch elements, a short token count T."""
    K = _K()
    M, N = 160, 10240
    A = (_rnd((T, M), 71) * 0.5).to(dtype)
    B = _rnd((T, N), 81).to(dtype)
    dW0 = _rnd((M, N), 91)
    db0 = _rnd((M,), 96)
    refW = dW0.double() + A.double().t() @ B.double()
    refb = db0.double() + A.double().sum(0)
    g = [A.to(DEV), B.to(DEV), dW0.to(DEV), db0.to(DEV), 0]
    assert K.dw_grouped_ok(T, [(g[0], g[1])])
    K.gemm_dw_grouped(T, [g])
    assert nrmse(refW.numpy(), g[2].double().cpu().numpy()) < 1e-5
    assert nrmse(refb.numpy(), g[3].double().cpu().numpy()) < 1e-5


# every fused-epilogue combination the Swin / patch GEMMs use (engine.py), at the
# model's N / K (160, 480, 640, 10240) with a ragged M: the v3 kernel's
# specialisations (gemm.hip DLCS_G3_CASES), resident-weight m-tile runs
# (N = 10240, M = 3000) and the 64-stage K = 10240 loop, vs torch fp32 on the
# same bf16 operands
_V3_CASES = [
    # name, M, N, K, b_trans, kwargs-builder
    ("qkv", 1000, 480, 160, 0, "bias"),
    ("proj", 1000, 160, 160, 0, "bias_resf32_rowmap"),
    ("fc1", 1000, 640, 160, 0, "bias_gelu"),
    ("fc2", 1000, 160, 640, 0, "bias_resf32"),
    ("embed", 1000, 160, 10240, 0, "acc"),
    ("unembed", 3000, 10240, 160, 0, "bias_relu"),
    ("dh", 1000, 640, 160, 1, "gelugrad"),
    ("dln2", 1000, 160, 640, 1, "f32"),
    ("dln1", 1000, 160, 480, 1, "f32"),
    ("datt", 1000, 160, 160, 1, "plain"),
    ("unembed_dgrad", 1000, 160, 10240, 1, "acc"),
    ("embed_dgrad", 3000, 10240, 160, 1, "res2"),
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("case", _V3_CASES, ids=[c[0] for c in _V3_CASES])
def test_gemm_model_epilogues(case, dtype):
    """bf16: the v3 kernel family; fp32: gemm_f32.inc (f32 MFMA), every operand
    and output fp32, checked in float64 (tolerance 1e-6)."""
    K = _K()
    name, M, N, K_, bt, kind = case
    bf = dtype
    g = torch.Generator(device="cpu").manual_seed(sum(map(ord, name)))
    A = torch.randn((M, K_), generator=g).to(DEV, bf)
    B = (torch.randn((K_, N), generator=g) if bt else torch.randn((N, K_), generator=g)).to(DEV, bf)
    Bm = B.double().t() if bt else B.double()
    pre = A.double() @ Bm.t()
    bias = torch.randn((N,), generator=g).to(DEV)
    kw, out_dt, ref = {}, bf, None
    if kind == "bias":
        kw, ref = dict(bias=bias), pre + bias
    elif kind == "bias_resf32_rowmap":
        res = torch.randn((M, N), generator=g).to(DEV).double()
        perm = torch.randperm(M, generator=g).to(torch.int32)
        kw = dict(bias=bias, alpha=0.8, res=res.float(), ldr=N, row_map=perm.to(DEV))
        out_dt = torch.float32
        ref = torch.empty_like(pre)
        ref[perm.long().to(DEV)] = 0.8 * (pre + bias) + res[perm.long().to(DEV)]
    elif kind == "bias_gelu":
        aux = torch.empty((M, N), device=DEV, dtype=bf)
        kw, ref = dict(bias=bias, act=1, aux_out=aux, ldaux=N), F.gelu(pre + bias)
    elif kind == "bias_resf32":
        res = torch.randn((M, N), generator=g).to(DEV)
        kw, out_dt, ref = dict(bias=bias, alpha=0.8, res=res, ldr=N), torch.float32, 0.8 * (pre + bias) + res.double()
    elif kind == "acc":
        out_dt = torch.float32
        kw = dict(accumulate=1, splitk=9)
        ref = pre + 1.5
    elif kind == "bias_relu":
        kw, ref = dict(bias=bias, act=3), torch.relu(pre + bias)
    elif kind == "gelugrad":
        h = torch.randn((M, N), generator=g).to(DEV, bf)
        x = h.double()
        cdf = 0.5 * (1 + torch.erf(x / 2 ** 0.5))
        kw, ref = dict(act=2, aux=h, ldaux=N), pre * (cdf + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5)
    elif kind == "f32":
        out_dt, ref = torch.float32, pre
    elif kind == "plain":
        ref = pre
    elif kind == "res2":
        r1 = torch.randn((M, N), generator=g).to(DEV, bf)
        r2 = torch.randn((M, N), generator=g).to(DEV, bf)
        kw = dict(res=r1, ldr=N, res_scale=2.0, res2=r2, ldr2=N)
        ref = pre + 2.0 * r1.double() + r2.double()
    if dtype == torch.float32:
        out_dt = torch.float32
    C = torch.full((M, N), 1.5, device=DEV, dtype=out_dt)
    K.gemm(A, B, C, M, N, K_, K_, N if bt else K_, N, b_trans=bt, **kw)
    torch.cuda.synchronize()
    tol = (1e-6 if dtype == torch.float32 else 1e-5) if out_dt == torch.float32 else 1e-2
    assert nrmse(ref.double().cpu().numpy(), C.double().cpu().numpy()) < tol
    if kind == "bias_gelu":
        assert nrmse((pre + bias).double().cpu().numpy(), kw["aux_out"].double().cpu().numpy()) < \
            (1e-6 if dtype == torch.float32 else 1e-2)
