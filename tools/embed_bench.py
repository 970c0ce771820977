"""Patch-embed forward GEMM at the BASELINE size (13440 tokens x 10240 -> 160, fp32):
the plain f32 kernel (no split) vs the deterministic split-K entry vs the bf16
3-plane split (dlcs_gemm_nt_x6; DLCS_NT_X6_S sets its K splits) vs the row-scaled f16
split (dlcs_gemm_h3r, K = 10240 split into DLCS_H3R_KSPLIT XCD-group ranges, default 4)."""
import os
os.environ.setdefault("DLCS_DIAG", "1")         # the diagnostic switches below are live
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
import torch  # noqa: E402
from dl_cs.models import _ops as K  # noqa: E402

M, N, Kd = 13440, 160, 10240
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn((M, Kd), device="cuda", generator=g)
B = torch.randn((N, Kd), device="cuda", generator=g)
C = torch.zeros((M, N), device="cuda")


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
    print(f"{name:12s} {us:8.1f} us  {2.0 * M * N * Kd / us / 1e6:6.1f} TFLOP/s")


run("plain", lambda: K.gemm(A, B, C, M, N, Kd, Kd, Kd, N, accumulate=1, splitk=1))
run("splitk_det", lambda: K.gemm_f32_splitk_det(A, B, C, M, N, Kd, Kd, Kd))
run("splitk_atom", lambda: K.gemm(A, B, C, M, N, Kd, Kd, Kd, N, accumulate=1, splitk=4))
try:                                              # the x6 NT GEMM is in the DIAG library only
    run("nt_x6", lambda: K.gemm_nt_x6(A, B, C, M, N, Kd, Kd, Kd))
except K._lib.DlcsError:
    print("nt_x6        (DIAG library only)")
(wp,) = K.h3r_pack([(B, False)])
run("h3r", lambda: K.linear_h3r(A, wp, N, out=C))
