"""Where does the f16x3 conv error come from inside the Swin regularizer?  Runs the
fp32 SwinTransformer3DNet forward + backward (as tools/grad_attrib.py) with the
160 -> 160 f16x3 conv entry points wrapped; for every launch it compares, in
float64 on the host:
    total   kernel output              vs conv64(x, w)      (what the network sees)
    kernel  kernel output              vs conv64(x~, w~)    (MFMA arithmetic, dropped xl wl)
    rep_x   conv64(x~, w)              vs conv64(x, w)      (activation split, per-tensor scale)
    rep_w   conv64(x, w~)              vs conv64(x, w)      (weight split)
    torch   torch fp32 conv(x, w)      vs conv64(x, w)
with x~ / w~ the operands as the split planes represent them.  Weight gradients:
total and torch only.     python tools/split_diag.py [X]
"""
import os
import sys

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "dl-swin-gan_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
from oracle import recipe  # noqa: E402


def blocked_to_ncdhw(r, grid):
    B, D, H, W = grid
    C = r.shape[1]
    return r.reshape(B, D // 4, H // 4, W // 4, 4, 4, 4, C).permute(0, 7, 1, 4, 2, 5, 3, 6).reshape(B, C, D, H, W)


def split_emulate(x):
    """x~ of the per-tensor f16 two-plane split (conv3d_f16x3.inc header), float64."""
    m = float(x.abs().max())
    if not m > 0:
        return x.double()
    e = torch.frexp(torch.tensor(m, dtype=torch.float64))[1].item()
    f = m / 2.0 ** e
    k = 14 - (e - 1 if f == 0.5 else e)
    s = 2.0 ** k
    u = (x.float() * s)
    xh = u.half()
    xl = (u - xh.float()).half()
    return (xh.double() + xl.double()) / s


def decode_planes(planes, rows):
    """split2 buffer -> x~ [rows, 160] float64 (the kernel's operand)."""
    f = planes[:rows * 640].view(torch.float16).view(rows, 5, 2, 32)
    mx = planes[rows * 640:rows * 640 + 4].view(torch.float32).item()
    e = torch.frexp(torch.tensor(mx, dtype=torch.float64))[1].item()
    fr = mx / 2.0 ** e
    s = 2.0 ** (14 - (e - 1 if fr == 0.5 else e)) if mx > 0 else 1.0
    x = (f[:, :, 0].double() + f[:, :, 1].double()) / s
    return x.reshape(rows, 160)


def rel(ref, x):
    return float((x.double() - ref).norm() / ref.norm())


def bias(ref, x):
    """mean signed error along the reference's sign, relative to mean |ref|"""
    d = x.double() - ref
    return float((d * ref.sign()).mean() / ref.abs().mean())


def main():
    X = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    torch.set_num_threads(16)
    from dl_cs.models import _ops as K
    from dl_cs.models import swin3D
    swin3D.set_compute_dtype(torch.float32)
    orig_split2, orig_pack, orig_conv, orig_wg = K.split2, K.conv_pack_f16x3, K.conv3d_f16x3, K.conv3d_wgrad_f16x3
    orig_k160 = K.gemm_k160_f16x3
    orig_x6 = K.gemm_nt_x6
    src = {}        # planes data_ptr -> fp32 original (cpu)
    wts = {}        # packed data_ptr -> (w fp32 cpu, mode)
    report = []

    def split2(x, out=None, have_max=False, colsum=None):
        r = orig_split2(x, out=out, have_max=have_max, colsum=colsum)
        src[r.data_ptr()] = x.detach().float().cpu().clone()
        return r

    def pack(w, mode):
        r = orig_pack(w, mode)
        wts[r.data_ptr()] = (w.detach().float().cpu().clone(), mode)
        return r

    def conv(planes, packed, grid, **kw):
        out = orig_conv(planes, packed, grid, **kw)
        raw = orig_conv(planes, packed, grid).cpu()
        rows = grid[0] * grid[1] * grid[2] * grid[3]
        x = src.get(planes.data_ptr())
        w, mode = wts.get(packed.data_ptr(), (None, None))
        if x is None or w is None:
            report.append(("conv", "operand not captured"))
            return out
        xt = decode_planes(planes.cpu(), rows)
        wk = w if mode == 0 else w.transpose(0, 1).flip(2, 3, 4)
        wt = split_emulate(w)
        wtk = wt if mode == 0 else wt.transpose(0, 1).flip(2, 3, 4)
        n = lambda v: blocked_to_ncdhw(v, grid)                      # noqa: E731
        c64 = lambda a, b: F.conv3d(n(a.double()), b.double(), padding=1)   # noqa: E731
        ref = c64(x, wk)
        got = n(raw.double())
        m = float(x.abs().max())
        small = float((x.abs() < m * 2.0 ** -17).float().mean())
        rms = float(x.double().pow(2).mean().sqrt())
        report.append((f"conv mode {mode}", dict(
            total=rel(ref, got), bias=bias(ref, got), kernel=rel(c64(xt, wtk), got), rep_x=rel(ref, c64(xt, wk)),
            rep_w=rel(ref, c64(x, wtk)), torch=rel(ref, F.conv3d(n(x), wk, padding=1)),
            x_max_over_rms=m / max(rms, 1e-30), x_frac_below_2m17=small,
            rep_x_elem=rel(x.double(), xt))))
        print(report[-1], flush=True)
        return out

    def wgrad(xp, gp, grid, dwp):
        before = dwp.clone()
        r = orig_wg(xp, gp, grid, dwp)
        x, g = src.get(xp.data_ptr()), src.get(gp.data_ptr())
        if x is None or g is None:
            report.append(("wgrad", "operand not captured"))
            return r
        dw = (dwp - before).cpu().double()                           # [27, co, ci]
        n = lambda v: blocked_to_ncdhw(v, grid)                      # noqa: E731
        x64, g64 = n(x.double()), n(g.double())
        ref = torch.nn.grad.conv3d_weight(x64, (160, 160, 3, 3, 3), g64, padding=1)     # [co, ci, 3,3,3]
        t32 = torch.nn.grad.conv3d_weight(n(x), (160, 160, 3, 3, 3), n(g), padding=1)
        got = dw.permute(1, 2, 0).reshape(160, 160, 3, 3, 3)
        report.append(("wgrad", dict(total=rel(ref, got), bias=bias(ref, got), torch=rel(ref, t32),
                                     g_max_over_rms=float(g.abs().max() / g.double().pow(2).mean().sqrt()))))
        print(report[-1], flush=True)
        return r

    def k160(a_planes, M, b_planes, N, C, **kw):
        r = orig_k160(a_planes, M, b_planes, N, C, **kw)
        a, b = src.get(a_planes.data_ptr()), src.get(b_planes.data_ptr())
        if a is None or b is None:
            report.append(("k160", "operand not captured"))
            return r
        raw = torch.zeros((M, N), dtype=torch.float32, device=C.device)
        orig_k160(a_planes, M, b_planes, N, raw)
        ref = a.double() @ b.double().t()
        at, bt = decode_planes(a_planes.cpu(), M), decode_planes(b_planes.cpu(), N)
        got = raw.cpu().double()
        m = float(a.abs().max())
        report.append((f"k160 {M}x{N}", dict(
            total=rel(ref, got), bias=bias(ref, got), kernel=rel(at @ bt.t(), got), rep_a=rel(ref, at @ b.double().t()),
            rep_b=rel(ref, a.double() @ bt.t()), torch=rel(ref, a @ b.t()),
            a_max_over_rms=m / max(float(a.double().pow(2).mean().sqrt()), 1e-30))))
        print(report[-1], flush=True)
        return r

    def x6(A, B, Cm, M, N, Kd, lda, ldb):
        c0 = Cm.detach().double().cpu().clone()
        r = orig_x6(A, B, Cm, M, N, Kd, lda, ldb)
        a, b = A.detach().reshape(M, Kd).cpu(), B.detach().reshape(N, Kd).cpu()
        ref = a.double() @ b.double().t()
        got = Cm.detach().double().cpu() - c0
        t32 = (a @ b.t()).double()
        report.append((f"x6 {M}x{N}x{Kd}", dict(total=rel(ref, got), bias=bias(ref, got), torch=rel(ref, t32),
                                               a_max_over_rms=float(a.abs().max() / a.double().pow(2).mean().sqrt()))))
        print(report[-1], flush=True)
        return r

    K.split2, K.conv_pack_f16x3, K.conv3d_f16x3, K.conv3d_wgrad_f16x3 = split2, pack, conv, wgrad
    K.gemm_k160_f16x3 = k160
    K.gemm_nt_x6 = x6
    seed = 71
    net = swin3D.SwinTransformer3DNet(num_swinblocks=1, in_chans=4, chans=160, kernel_size=3, window_size=(4, 4))
    net.eval()
    recipe.fill_module(net, seed)
    net = net.cuda()
    x = recipe.crandn(seed + 1, (1, 2, 20, 192, X))
    y = net(x.cuda())
    g = recipe.crandn(seed + 2, y.shape)
    (y.real * g.real.cuda() + y.imag * g.imag.cuda()).sum().backward()
    torch.cuda.synchronize()
    print("done", len(report))


if __name__ == "__main__":
    main()
