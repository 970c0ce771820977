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
    T, Y, X, C = 16, 48, 48, 160
    grid = (1, T, Y, X)
    for pos, exact in ((True, False), (True, True), (False, False)):
        g0 = torch.Generator().manual_seed(3)
        x = torch.rand((1, C, T, Y, X), generator=g0) if pos else torch.randn((1, C, T, Y, X), generator=g0)
        w = torch.rand((C, C, 3, 3, 3), generator=g0) if pos else torch.randn((C, C, 3, 3, 3), generator=g0)
        w = w / 64.0
        if exact:       # operands exactly representable in fp16 (the low planes are zero: hh products only)
            x, w = x.half().float(), w.half().float()
        ref = F.conv3d(x.double(), w.double(), padding=1)
        xb = blocked(x).cuda()
        y16 = K.conv3d_f16x3(K.split2(xb), K.conv_pack_f16x3(w.cuda(), 0), grid)
        y32 = K.conv3d(xb, C, K.conv_pack(w.cuda(), torch.float32, 0), C, C, grid, out_dtype=torch.float32)
        torch.cuda.synchronize()
        tag = ("positive" if pos else "signed  ") + (" f16-exact" if exact else "          ")
        print(f"{tag} conv f16x3 : {stats(ref, unblocked(y16.cpu(), T, Y, X))}")
        print(f"{tag} conv f32   : {stats(ref, unblocked(y32.cpu(), T, Y, X))}")
        print(f"{tag} torch fp32 : {stats(ref, F.conv3d(x, w, padding=1))}")
        M, Kd, N = 4096, 640, 160
        a = torch.rand((M, Kd), generator=g0) if pos else torch.randn((M, Kd), generator=g0)
        b = torch.rand((N, Kd), generator=g0) if pos else torch.randn((N, Kd), generator=g0)
        if exact:
            a, b = a.half().float(), b.half().float()
        (bp,) = K.h3r_pack([(b.cuda(), False)])
        o = K.linear_h3r(a.cuda(), bp, N).cpu()
        rg = a.double() @ b.double().t()
        print(f"{tag} h3r K=640  : {stats(rg, o)}")
        print(f"{tag} torch K=640: {stats(rg, a @ b.t())}")
        # the patch-embed shape: [M, 10240] x [160, 10240]^T on the x6 split and on f32 MFMA split-K
        M2, K2 = 2048, 10240
        a2 = torch.rand((M2, K2), generator=g0) if pos else torch.randn((M2, K2), generator=g0)
        b2 = torch.rand((C, K2), generator=g0) if pos else torch.randn((C, K2), generator=g0)
        if exact:
            a2, b2 = a2.half().float(), b2.half().float()
        r2 = a2.double() @ b2.double().t()
        o6 = torch.zeros((M2, C), device="cuda")
        K.gemm_nt_x6(a2.cuda(), b2.cuda(), o6, M2, C, K2, K2, K2)
        of = torch.zeros((M2, C), device="cuda")
        K.gemm_f32_splitk_det(a2.cuda(), b2.cuda(), of, M2, C, K2, K2, K2)
        print(f"{tag} x6 K=10240 : {stats(r2, o6.cpu())}")
        print(f"{tag} f32 K=10240: {stats(r2, of.cpu())}")
        print(f"{tag} torch 10240: {stats(r2, a2 @ b2.t())}")
        # the 160 -> 160 weight gradient (one voxel-range chain per workgroup)
        gy = torch.rand((1, C, T, Y, X), generator=g0) if pos else torch.randn((1, C, T, Y, X), generator=g0)
        if exact:
            gy = gy.half().float()
        rw = torch.nn.grad.conv3d_weight(x.double(), (C, C, 3, 3, 3), gy.double(), padding=1)
        dwp = torch.zeros((27, C, C), device="cuda")
        K.conv3d_wgrad_f16x3(K.split2(xb), K.split2(blocked(gy).cuda()), grid, dwp)
        dw = dwp.cpu().double().permute(1, 2, 0).reshape(C, C, 3, 3, 3)
        print(f"{tag} wgrad f16x3: {stats(rw, dw)}")
        print(f"{tag} wgrad torch: {stats(rw, torch.nn.grad.conv3d_weight(x, (C, C, 3, 3, 3), gy, padding=1))}")


if __name__ == "__main__":
    main()
