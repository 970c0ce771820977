"""Micro-benchmark of the grouped weight gradients of one Swin block backward at
the BASELINE token count (T = 13440): qkv (480 x 160), proj (160 x 160), fc1
(640 x 160), fc2 (160 x 640) in one dlcs_gemm_dw_grouped launch (+ the partial
reduce), then the patch unembed / embed weight gradients (10240 x 160, 44 GFLOP
each), and the DiT block's four Linears (D = 384, T = 23040, edge tiles) next to
the f32-MFMA linear_dw GEMM; fp32 operands; DLCS_DW_F32=1 / DLCS_DW_X6=1 select the
f32-MFMA / bf16 3-plane kernels instead of the default fp16 2-plane one."""
import os
os.environ.setdefault("DLCS_DIAG", "1")         # the diagnostic switches below are live
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
import torch  # noqa: E402
from dl_cs.models import _ops as K  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
T = 13440
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
shapes = [(480, 160), (160, 160), (640, 160), (160, 640)]
groups = []
for M, N in shapes:
    groups.append([torch.randn((T, M), device=dev, generator=g), torch.randn((T, N), device=dev, generator=g),
                   torch.zeros((M, N), device=dev), torch.zeros((M,), device=dev), 0])


def run(name, grp):
    flops = sum(2.0 * T * a.shape[1] * b.shape[1] for a, b, *_ in grp)
    for _ in range(3):
        K.gemm_dw_grouped(T, grp)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        K.gemm_dw_grouped(T, grp)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    print(f"{name} (T={T}, {flops / 1e9:.2f} GFLOP): {us:.1f} us  {flops / us / 1e6:.1f} TFLOP/s fp32-equiv")


run("block dW (4 Linears)", groups)
tok = torch.randn((T, 160), device=dev, generator=g)
big = torch.randn((T, 10240), device=dev, generator=g)
run("unembed dW 10240x160", [[big, tok, torch.zeros((10240, 160), device=dev), torch.zeros(160, device=dev), 160]])
run("embed dW 160x10240", [[tok, big, torch.zeros((160, 10240), device=dev), torch.zeros(160, device=dev), 0]])

Td = 23040
dshapes = [(1152, 384), (384, 1536), (1536, 384), (2304, 384)]
dgroups = [[torch.randn((Td, M), device=dev, generator=g), torch.randn((Td, N), device=dev, generator=g),
            torch.zeros((M, N), device=dev), torch.zeros((M,), device=dev), 0] for M, N in dshapes]
T = Td
run("DiT block dW (4 Linears, D=384)", dgroups)
for _ in range(3):
    for a_, b_, w_, *_r in dgroups:
        K.linear_dw(a_, b_, w_)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    for a_, b_, w_, *_r in dgroups:
        K.linear_dw(a_, b_, w_)
e1.record()
torch.cuda.synchronize()
print(f"DiT block dW via linear_dw (f32 MFMA, no bias): {e0.elapsed_time(e1) * 1e3 / iters:.1f} us")
