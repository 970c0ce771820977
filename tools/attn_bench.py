"""Window attention fwd / bwd at the BASELINE shape: 30 windows x 448 tokens,
8 heads x 20 (bf16), shifted-block labels; FLOPs counted for QK^T + PV (fwd) and
the 5 products of the backward (S recompute, dP, dV, dK, dQ)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
import torch  # noqa: E402
from dl_cs import _lib  # noqa: E402
from dl_cs.models import _ops as K  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
nwin, N, H, hd = 30, 448, 8, 20
C = H * hd
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn((nwin * N, 3 * C), device=dev, generator=g).bfloat16()
table = 0.02 * torch.randn((13 * 15 * 15, H), device=dev, generator=g)
labels = torch.randint(0, 27, (nwin * N,), device=dev, generator=g, dtype=torch.int32)
out = torch.empty((nwin * N, C), device=dev, dtype=torch.bfloat16)
lse = torch.empty((nwin, H, N), device=dev)
dout = torch.randn((nwin * N, C), device=dev, generator=g).bfloat16()
dqkv = torch.zeros((nwin * N, 3 * C), device=dev)
dtable = torch.zeros_like(table)
S = _lib.stream


def fwd():
    _lib.call("dlcs_window_attn_fwd", 1, _lib.ptr(qkv), _lib.ptr(out), _lib.ptr(lse), _lib.ptr(table),
              _lib.ptr(labels), None, 0, nwin, N, H, hd, 7, 8, 8, hd ** -0.5, S())


def bwd():
    _lib.call("dlcs_window_attn_bwd", 1, _lib.ptr(qkv), _lib.ptr(out), _lib.ptr(dout), _lib.ptr(lse),
              _lib.ptr(table), _lib.ptr(labels), None, 0, _lib.ptr(dqkv), _lib.ptr(dtable),
              nwin, N, H, hd, 7, 8, 8, hd ** -0.5, S())


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
    ms = e0.elapsed_time(e1) / iters
    print(f"{name:4s} {ms * 1000:8.1f} us  {flops / ms / 1e9:7.1f} TFLOP/s (hd padded flops x{32 / hd:.2f})")


f1 = 2.0 * nwin * H * N * N * hd
run("fwd", fwd, 2 * f1)
run("bwd", bwd, 5 * f1)
