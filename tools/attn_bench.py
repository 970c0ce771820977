"""Micro-benchmark of the fused window attention at the BASELINE geometry
(30 windows x 8 heads x 448 tokens, head dim 20; shifted blocks: region labels):
forward and backward, fp32 or bf16.  python tools/attn_bench.py [iters] [fp32|bf16] [labels|plain]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
import torch  # noqa: E402
from dl_cs.models import _ops as K  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dt = torch.float32 if (len(sys.argv) > 2 and sys.argv[2] == "fp32") else torch.bfloat16
case = sys.argv[3] if len(sys.argv) > 3 else "labels"
PEAK = 157.3 if dt == torch.float32 else 2500.0
nwin, N, heads, hd, window = 30, 448, 8, 20, (7, 8, 8)
C, scale = heads * hd, hd ** -0.5
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn((nwin * N, 3 * C), device=dev, generator=g).to(dt)
table = torch.randn((13 * 15 * 15, heads), device=dev, generator=g) * 0.1
labels = (torch.rand((nwin * N,), device=dev, generator=g) * 4).int() if case == "labels" else None
dout = torch.randn((nwin * N, C), device=dev, generator=g).to(dt)
dtab = torch.zeros_like(table)
flops_f = 4.0 * nwin * heads * N * N * hd
out, lse = K.attn_fwd(qkv, table, labels, nwin, N, heads, hd, window, scale)


def run(name, fn, flops):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    print(f"{name:5s} {dt} {case}: {us:8.1f} us  {flops / us / 1e6:7.1f} TFLOP/s  ({flops / us / 1e6 / PEAK * 100:5.1f}% of peak)")


run("fwd", lambda: K.attn_fwd(qkv, table, labels, nwin, N, heads, hd, window, scale), flops_f)
run("bwd", lambda: K.attn_bwd(qkv, out, dout, lse, table, labels, dtab, nwin, N, heads, hd, window, scale), 2.5 * flops_f)
