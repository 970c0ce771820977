"""Micro-benchmark of the Conv3d k3 kernels at the BASELINE size (for rocprofv3
and A/B timing): fwd (160->160, relu_out + residual), dgrad, wgrad."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
import torch  # noqa: E402
from dl_cs.models import _ops as K  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "all"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dt = torch.bfloat16
grid = (1, 28, 192, 160)
rows = 28 * 192 * 160
C = 160
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn((rows, C), device=dev, generator=g).to(dt)
r = torch.randn((rows, C), device=dev, generator=g).to(dt)
w = torch.randn((C, C, 3, 3, 3), device=dev, generator=g) / (27 * C) ** 0.5
bias = torch.zeros(C, device=dev)
wf = K.conv_pack(w, dt, 0)
wd = K.conv_pack(w, dt, 1)
dwp = torch.zeros((27, C, C), device=dev)
flops = 2.0 * rows * C * C * 27


def run(name, fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    print(f"{name:6s} {ms:7.3f} ms  {flops / ms / 1e9:7.1f} TFLOP/s  ({flops / ms / 1e9 / 2500 * 100:4.1f}% of bf16 dense peak)")


if which in ("all", "fwd"):
    run("fwd", lambda: K.conv3d(x, C, wf, C, C, grid, bias=bias, res=r, relu_out=1))
if which in ("all", "dgrad"):
    run("dgrad", lambda: K.conv3d(x, C, wd, C, C, grid, mask=r))
if which in ("all", "wgrad"):
    run("wgrad", lambda: K.conv3d_wgrad(x, C, 0, r, C, grid, dwp))
