"""Time the Swin block's eight fp32 Linear GEMMs (forward + input gradient) on the
f32-MFMA path (dlcs_gemm) vs the row-scaled f16x3 path (dlcs_gemm_h3r) at the
BASELINE token count (13440), HIP events around 20 launches each."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "dl-swin-gan_amd"))
from dl_cs.models import _ops as K  # noqa: E402

M = 13440
DEV = "cuda"
SHAPES = [  # name, K, N, trans (B = W^T for input gradients)
    ("qkv fwd", 160, 480, False), ("proj fwd", 160, 160, False), ("fc1 fwd", 160, 640, False),
    ("fc2 fwd", 640, 160, False), ("fc2 dx", 160, 640, True), ("fc1 dx", 640, 160, True),
    ("proj dx", 160, 160, True), ("qkv dx", 480, 160, True),
]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    tot32 = toth3 = 0.0
    for name, Kd, N, trans in SHAPES:
        x = torch.randn((M, Kd), device=DEV)
        w = torch.randn((Kd, N) if trans else (N, Kd), device=DEV) / Kd ** 0.5
        out = torch.empty((M, N), device=DEV)
        if trans:
            f32 = lambda: K.linear_dx(x, w, out=out)
        else:
            f32 = lambda: K.linear(x, w, out=out)
        (wp,) = K.h3r_pack([(w, trans)])
        b = torch.randn((N,), device=DEV)
        r = torch.randn((M, N), device=DEV)
        h3 = lambda: K.linear_h3r(x, wp, N, out=out)
        h3e = lambda: K.linear_h3r(x, wp, N, out=out, bias=b, res=r)      # the fwd epilogue: bias + residual
        t32, th3, th3e = timeit(f32), timeit(h3), timeit(h3e)
        fl = 2.0 * M * N * Kd
        tot32 += t32
        toth3 += th3
        print(f"{name:9s} K={Kd:3d} N={N:3d}: f32 {t32:7.1f} us ({fl / t32 / 1e6:6.1f} TF/s)   "
              f"h3r {th3:7.1f} us ({fl / th3 / 1e6:6.1f} TF/s fp32-equiv, {3 * fl / th3 / 1e6 / 2500:.3f} of fp16 peak)  +bias+res {th3e:6.1f} us")
    print(f"sum per block: f32 {tot32:.1f} us, h3r {toth3:.1f} us; x60 per step: {60 * tot32 / 1e3:.2f} vs {60 * toth3 / 1e3:.2f} ms")
    pk = [(torch.randn((N, Kd) if not t else (Kd, N), device=DEV), t) for _, Kd, N, t in SHAPES] * 6
    print(f"pack of 48 weights (one network): {timeit(lambda: K.h3r_pack(pk), 10):.1f} us")


def sweep():
    """h3r time vs M at fixed K / N: the intercept is the per-workgroup latency
    floor, the slope the throughput (python tools/h3r_bench.py sweep)."""
    for name, Kd, N, trans in SHAPES[:4]:
        w = torch.randn((N, Kd), device=DEV) / Kd ** 0.5
        (wp,) = K.h3r_pack([(w, False)])
        row = []
        for m in (1680, 3360, 6720, 13440, 26880, 53760):
            x = torch.randn((m, Kd), device=DEV)
            out = torch.empty((m, N), device=DEV)
            row.append(f"M={m}: {timeit(lambda: K.linear_h3r(x, wp, N, out=out)):6.1f}")
        print(f"{name:9s} K={Kd:3d} N={N:3d} | " + "  ".join(row))


if __name__ == "__main__":
    sweep() if sys.argv[1:] == ["sweep"] else main()
