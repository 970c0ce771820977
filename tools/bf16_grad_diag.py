"""bf16 vs fp32 gradients of SwinTransformer3DNet at NUM_SWINBLOCKS = 1 and 2 (the
tests/test_gpu_swin.py::test_bf16_swinnet_two_swinblocks setup): NRMSE of the input
gradient and of every parameter gradient, to tell the bf16 build's rounding growth
with depth from a defect of one branch.  GPU box:  python tools/bf16_grad_diag.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
sys.path.insert(0, REPO)
from dl_cs.models import swin3D  # noqa: E402
from oracle import recipe  # noqa: E402

DEV = "cuda"


def rel(a, b):
    return float((a - b).abs().pow(2).sum().sqrt() / b.abs().pow(2).sum().sqrt().clamp_min(1e-30))


def run(net, x, gr, dtype):
    swin3D.set_compute_dtype(dtype)
    try:
        for p in net.parameters():
            p.grad = None
        xx = x.clone().requires_grad_()
        y = net(xx)
        (y.real * gr.real + y.imag * gr.imag).sum().backward()
        return y.detach(), xx.grad.detach(), {n: p.grad.detach().clone() for n, p in net.named_parameters()
                                              if p.grad is not None}
    finally:
        swin3D.set_compute_dtype(torch.float32)


for nb in (1, 2):
    net = swin3D.SwinTransformer3DNet(num_swinblocks=nb, in_chans=4, chans=160, kernel_size=3, window_size=(4, 4))
    net.eval()
    recipe.fill_module(net, 34)
    net = net.to(DEV)
    x = recipe.crandn(35, (1, 2, 20, 32, 32)).to(DEV)
    gr = recipe.crandn(36, (1, 2, 20, 32, 32)).to(DEV)
    y16, dx16, g16 = run(net, x, gr, torch.bfloat16)
    y32, dx32, g32 = run(net, x, gr, torch.float32)
    print(f"nb={nb}  y {rel(y16, y32):.4f}  dx {rel(dx16, dx32):.4f}  |dx32| {float(dx32.abs().pow(2).mean().sqrt()):.3e}")
    rows = sorted(((rel(g16[n], g32[n]), n) for n in g32 if g32[n].abs().sum() > 0), reverse=True)
    for r, n in rows[:12]:
        print(f"   {r:.4f}  {n}")
    print(f"   median {rows[len(rows) // 2][0]:.4f} over {len(rows)} tensors", flush=True)
