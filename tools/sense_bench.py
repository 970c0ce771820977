"""Micro-benchmark of the SENSE operator at the BASELINE size (8 coils x 20
frames x 192 x 160, 2 maps, mask): forward, adjoint and the fused PGD
normal-op + DC update, in us per op and algorithmic GB/s (each operand read or
written once; for the fused normal operator x, maps, mask, A^H y in and out --
its k-space never reaches HBM); then the HQS conjugate-gradient solve (10 steps,
alg:50-73) as one device-resident dlcs_sense_cg vs the reference's torch CG loop
on the same fused normal operator.  DLCS_SENSE_GENERIC=1 times the generic
kernels instead.  The mask is the reference's VDkt cine mask (seed 1000, the
bench slice's); each normal-operator line is timed on the row-sparse operator
(dlcs_sense_normal_rows) and on the dense three-launch one (DLCS_SENSE_ROWS=0),
and once more with a 10 % random element mask (every line sampled)."""
import os
os.environ.setdefault("DLCS_DIAG", "1")         # the diagnostic switches below are live
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
import torch  # noqa: E402
from dl_cs.mri import transforms as T  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
B, E, C, Tt, Y, X = 1, 2, 8, 20, 192, 160
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
cr = lambda *s: torch.complex(torch.randn(s, device=dev, generator=g), torch.randn(s, device=dev, generator=g))
maps = cr(B, E, C, 1, Y, X)
import numpy as np  # noqa: E402
_g = np.load(os.path.join(REPO, "tests", "golden", "misc.npz"))
_sh = tuple(int(v) for v in _g["vdkt_seed1000_shape"])
mask = torch.from_numpy(np.unpackbits(_g["vdkt_seed1000_bits"])[: int(np.prod(_sh))].reshape(_sh).astype(np.float32)).to(dev)
rmask = (torch.rand((B, 1, Tt, Y, X), device=dev, generator=g) < 0.1).float()
x, y = cr(B, E, Tt, Y, X), cr(B, C, Tt, Y, X)
A = T.SenseModel(maps, weights=mask)
img, ksp = B * E * Tt * Y * X * 8, B * C * Tt * Y * X * 8
mb, wb = B * E * C * Y * X * 8, B * Tt * Y * X * 4


def run(name, fn, nbytes):
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
    print(f"{name:18s} {us:8.1f} us  {nbytes / us / 1e3:7.1f} GB/s  ({nbytes / us / 1e3 / 8000 * 100:4.1f}% of 8 TB/s)")


only_nrm = len(sys.argv) > 2 and sys.argv[2] == "nrm"   # rocprof: the VDkt normal operators only
with torch.no_grad():
    if only_nrm:
        aty = A(y, adjoint=True)
        for rows in ("1", "0"):
            os.environ["DLCS_SENSE_ROWS"] = rows
            run(f"normal_dc/{'rows' if rows == '1' else 'dense'}", lambda: A.normal_dc(x, aty, -2.0), 3 * img + mb + wb)
        sys.exit(0)
    run("forward", lambda: A(x), img + mb + wb + ksp)
    run("adjoint", lambda: A(y, adjoint=True), ksp + mb + wb + img)
    aty = A(y, adjoint=True)
    lines = int((mask.sum(-1) > 0).sum())
    lb = lines * X * 4                       # the sampled weight lines (row-sparse operator)
    for rows in ("1", "0"):
        os.environ["DLCS_SENSE_ROWS"] = rows
        tag = "rows" if rows == "1" else "dense"
        wbytes = lb if rows == "1" else wb
        run(f"normal_dc/{tag}", lambda: A.normal_dc(x, aty, -2.0), 3 * img + mb + wbytes)
        run(f"normal+lam/{tag}", lambda: A.normal(x, 0.1), 2 * img + mb + wbytes)
    os.environ["DLCS_SENSE_ROWS"] = "1"
    Ar = T.SenseModel(maps, weights=rmask)
    run("normal_dc/rand10%", lambda: Ar.normal_dc(x, aty, -2.0), 3 * img + mb + wb)
    from dl_cs.mri.algorithms import ConjugateGradient
    cg_torch = ConjugateGradient(lambda m: A.normal(m, 0.1), 10)
    # per CG step: one normal op + the vector updates (p, Ap, x, r read / written)
    cg_bytes = 11 * (2 * img + mb + wb) + 10 * 7 * img
    run("cg10_dev", lambda: A.cg(x, aty, 0.1, 10), cg_bytes)
    os.environ["DLCS_SENSE_ROWS"] = "0"
    run("cg10_dense", lambda: A.cg(x, aty, 0.1, 10), cg_bytes)
    os.environ["DLCS_SENSE_ROWS"] = "1"
    run("cg10_torch", lambda: cg_torch(x, aty), cg_bytes)
