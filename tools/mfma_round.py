"""Accumulation rounding of the f16x3 kernels: with all-positive operands every
product adds coherently, so a per-instruction truncation of the MFMA accumulator
shows up as a relative error growing with the number of MFMAs per output (and a
negative mean), round-to-nearest as a small zero-mean error.  Compares the f16x3
conv (405 MFMAs per output), the f32-MFMA conv and the h3r GEMM (K = 640: 60 MFMAs)
against float64, for positive and for signed data.   python tools/mfma_round.py
"""
import os
import sys

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
from dl_cs.models import _ops as K  # noqa: E402
from wgrad_err import blocked, unblocked  # noqa: E402


def stats(ref, got):
    d = got.double() - ref
    return (f"rel {float(d.norm() / ref.norm()):.3e}  mean signed {float((d * ref.sign()).mean() / ref.abs().mean()):+.3e}")


def main():
    torch.set_num_threads(16)
    T, Y, X, C = 8, 32, 32, 160
    grid = (1, T, Y, X)
    for pos in (True, False):
        g0 = torch.Generator().manual_seed(3)
        x = torch.rand((1, C, T, Y, X), generator=g0) if pos else torch.randn((1, C, T, Y, X), generator=g0)
        w = torch.rand((C, C, 3, 3, 3), generator=g0) if pos else torch.randn((C, C, 3, 3, 3), generator=g0)
        w = w / (27 * C) ** 0.5
        ref = F.conv3d(x.double(), w.double(), padding=1)
        xb = blocked(x).cuda()
        y16 = K.conv3d_f16x3(K.split2(xb), K.conv_pack_f16x3(w.cuda(), 0), grid)
        y32 = K.conv3d(xb, C, K.conv_pack(w.cuda(), torch.float32, 0), C, C, grid, out_dtype=torch.float32)
        torch.cuda.synchronize()
        tag = "positive" if pos else "signed  "
        print(f"{tag} conv f16x3 : {stats(ref, unblocked(y16.cpu(), T, Y, X))}")
        print(f"{tag} conv f32   : {stats(ref, unblocked(y32.cpu(), T, Y, X))}")
        print(f"{tag} torch fp32 : {stats(ref, F.conv3d(x, w, padding=1))}")
        M, Kd, N = 4096, 640, 160
        a = torch.rand((M, Kd), generator=g0) if pos else torch.randn((M, Kd), generator=g0)
        b = torch.rand((N, Kd), generator=g0) if pos else torch.randn((N, Kd), generator=g0)
        (bp,) = K.h3r_pack([(b.cuda(), False)])
        o = K.linear_h3r(a.cuda(), bp, N).cpu()
        rg = a.double() @ b.double().t()
        print(f"{tag} h3r K=640  : {stats(rg, o)}")
        print(f"{tag} torch K=640: {stats(rg, a @ b.t())}")


if __name__ == "__main__":
    main()
