"""CPU check of an fp16 two-plane split (x = xh + xl, xh = fp16(s x) / s,
xl = fp16(s x - fp16(s x)) / s, s a power of two putting max|x| at 2^14) for
the fp32 Conv3d 160 -> 160: three plane products (hh + hl + lh) summed in fp32,
vs float64, beside PyTorch's fp32 conv and the bf16 x6 split.  Also on a
gradient-like operand (|g| ~ 1e-7 with a 1e6 dynamic range), where an unscaled
fp16 split would underflow.  python tools/f16x3_numerics.py"""
import math

import torch
import torch.nn.functional as F


def pow2_scale(t):
    m = float(t.abs().max())
    return 1.0 if m == 0 else 2.0 ** (14 - math.ceil(math.log2(m)))


def split2(t, s=None):
    s = pow2_scale(t) if s is None else s
    u = t * s
    h = u.half().float()
    lo = (u - h).half().float()
    return h / s, lo / s


def split3(t):
    h = t.bfloat16().float()
    r = t - h
    m = r.bfloat16().float()
    return h, m, (r - m).bfloat16().float()


def run(x, w, tag):
    ref = F.conv3d(x.double(), w.double(), padding=1)
    nr = lambda a: float((a.double() - ref).norm() / ref.norm())
    c = lambda a, b: F.conv3d(a, b, padding=1)
    xh, xl = split2(x)
    wh, wl = split2(w)
    print(f"[{tag}] fp32     ", nr(c(x, w)))
    print(f"[{tag}] f16x3    ", nr(c(xl, wh) + c(xh, wl) + c(xh, wh)))
    xh0, xl0 = split2(x, 1.0)
    wh0, wl0 = split2(w, 1.0)
    print(f"[{tag}] f16x3 s=1", nr(c(xl0, wh0) + c(xh0, wl0) + c(xh0, wh0)))
    a, b, cc = split3(x)
    d, e, f = split3(w)
    six = [(a, d), (a, e), (b, d), (a, f), (cc, d), (b, e)]
    print(f"[{tag}] bf16x6   ", nr(sum(c(p, q) for p, q in six[::-1])))


def main():
    torch.manual_seed(0)
    x = torch.randn(1, 160, 6, 24, 24)
    w = torch.randn(160, 160, 3, 3, 3) / (27 * 160) ** 0.5
    run(x, w, "activation")
    # gradient-like: tiny values, 1e6 dynamic range (log-uniform magnitudes)
    g = torch.randn(1, 160, 6, 24, 24) * 1e-7 * torch.exp(torch.rand(1, 160, 6, 24, 24) * math.log(1e6) - 6)
    run(g, w, "gradient")
    # wgrad-shaped contraction over voxels: dW = sum_v g[v] x[v+o] (as a conv of x by g)
    gg = g[:, :, :4, :12, :12]
    xx = x[:, :, :6, :14, :14]
    ref = F.conv3d(xx.transpose(0, 1).double(), gg.transpose(0, 1).double())
    nr = lambda a: float((a.double() - ref).norm() / ref.norm())
    c = lambda a, b: F.conv3d(a.transpose(0, 1), b.transpose(0, 1))
    xh, xl = split2(xx)
    gh, gl = split2(gg)
    print("[wgrad] fp32     ", nr(c(xx, gg)))
    print("[wgrad] f16x3    ", nr(c(xl, gh) + c(xh, gl) + c(xh, gh)))


if __name__ == "__main__":
    main()
