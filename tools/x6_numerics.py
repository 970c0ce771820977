"""CPU check of the 3-plane bf16 split behind the x6 conv kernels: NRMSE vs
float64 of (a) PyTorch's fp32 Conv3d 160 -> 160, (b) the six plane products
(x6), (c) three plane products, (d) plain bf16 -- each plane product summed in
fp32 as the MFMA accumulator does.  python tools/x6_numerics.py"""
import torch
import torch.nn.functional as F


def split3(t):
    h = t.bfloat16().float()
    r = t - h
    m = r.bfloat16().float()
    return h, m, (r - m).bfloat16().float()


def main():
    torch.manual_seed(0)
    x = torch.randn(1, 160, 6, 24, 24)
    w = torch.randn(160, 160, 3, 3, 3) / (27 * 160) ** 0.5
    ref = F.conv3d(x.double(), w.double(), padding=1)
    nr = lambda a: float((a.double() - ref).norm() / ref.norm())
    xh, xm, xl = split3(x)
    wh, wm, wl = split3(w)
    c = lambda a, b: F.conv3d(a, b, padding=1)
    six = [(xh, wh), (xh, wm), (xm, wh), (xh, wl), (xl, wh), (xm, wm)]
    print("fp32   ", nr(c(x, w)))
    print("bf16x6 ", nr(sum(c(a, b) for a, b in six[::-1])))
    print("bf16x3 ", nr(sum(c(a, b) for a, b in six[:3][::-1])))
    print("bf16   ", nr(c(xh, wh)))


if __name__ == "__main__":
    main()
