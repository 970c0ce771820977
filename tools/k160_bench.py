"""The K = 160 f16x3 patch GEMMs at the BASELINE size (13440 tokens x 160 ->
10240: the patch unembed forward with bias + ReLU, the embed input gradient with
two residuals), us per launch; DLCS_K160_XCD=0 selects the 2-D tile order."""
import os
os.environ.setdefault("DLCS_DIAG", "1")         # the diagnostic switches below are live
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
import torch  # noqa: E402
from dl_cs.models import _ops as K  # noqa: E402

M, N = 13440, 10240
g = torch.Generator(device="cuda").manual_seed(0)
A = K.split2(torch.randn((M, 160), device="cuda", generator=g))
B = K.split2(torch.randn((N, 160), device="cuda", generator=g) * 0.05)
C = torch.empty((M, N), device="cuda")
bias = torch.zeros(N, device="cuda")
r1, r2 = torch.randn((M, N), device="cuda", generator=g), torch.randn((M, N), device="cuda", generator=g)


def run(name, fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    print(f"{name:14s} {us:8.1f} us  ({M * N * 4 / us / 1e3:.0f} GB/s of C written)")


run("unembed fwd", lambda: K.gemm_k160_f16x3(A, M, B, N, C, bias=bias, act=3))
run("embed dgrad", lambda: K.gemm_k160_f16x3(A, M, B, N, C, res=r1, res_scale=2.0, res2=r2))
