"""Micro-benchmark of the fp32 thin-end conv kernels (f16x3) at the BASELINE
regularizer grid (1 x 28 x 192 x 160): thin-input forward (SFE 4 -> 160) and
dgrad (final conv, masked), thin-output forward (final 160 -> 4) and dgrad (SFE),
both weight gradients; us per launch and the HBM rate of the 160-channel side
(550 MB fp32 read or written once).  DLCS_THIN_OUT_V2=1 times the thin-output
kernel with LDS-resident weights."""
import os
os.environ.setdefault("DLCS_DIAG", "1")         # the diagnostic switches below are live
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
import torch  # noqa: E402
from dl_cs.models import _ops as K  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
grid = (1, 28, 192, 160)
rows, C, e = 28 * 192 * 160, 160, 4
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
x4 = torch.zeros((rows, 8), device=dev)
x4[:, :e] = torch.randn((rows, e), device=dev, generator=g)
x160 = torch.randn((rows, C), device=dev, generator=g)
m = torch.randn((rows, C), device=dev, generator=g)
w_sfe = torch.randn((C, e, 3, 3, 3), device=dev, generator=g) / (27 * e) ** 0.5
w_fin = torch.randn((e, C, 3, 3, 3), device=dev, generator=g) / (27 * C) ** 0.5
b160, b4 = torch.zeros(C, device=dev), torch.zeros(e, device=dev)
wp = K.thin_pack_f16x3(K.conv_pack(w_sfe, torch.float32, 0), C, e, 0)
wdp = K.thin_pack_f16x3(K.conv_pack(w_fin, torch.float32, 1), C, e, 0)
wo = K.thin_pack_f16x3(K.conv_pack(w_fin, torch.float32, 0), e, C, 1)
wso = K.thin_pack_f16x3(K.conv_pack(w_sfe, torch.float32, 1), e, C, 1)
mx4, mx160 = K.absmax(x4[:, :e].contiguous()), K.absmax(x160)
big = rows * C * 4


def run(name, fn):
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
    print(f"{name:12s} {us:8.1f} us  {big / us / 1e3:7.1f} GB/s of the 160-channel side ({big / us / 1e3 / 8000:.2f} of 8 TB/s)")


run("thin_in", lambda: K.conv3d_thin_f16x3(x4, e, mx4, wp, C, C, grid, bias=b160))
run("thin_in_mask", lambda: K.conv3d_thin_f16x3(x4, e, mx4, wdp, C, C, grid, mask=m))
run("thin_out", lambda: K.conv3d_thin_f16x3(x160, C, mx160, wo, e, 8, grid, bias=b4))
run("thin_out_dg", lambda: K.conv3d_thin_f16x3(x160, C, mx160, wso, e, 8, grid))
dw1 = torch.zeros((27, C, K.pad32(e)), device=dev)
run("wgrad_sfe", lambda: K.conv3d_thin_wgrad_f16x3(x4, e, mx4, x160, C, mx160, grid, dw1))
dw2 = torch.zeros((27, K.pad32(e), C), device=dev)
run("wgrad_fin", lambda: K.conv3d_thin_wgrad_f16x3(x160, C, mx160, x4, e, mx4, grid, dw2))
# the planes kernels (conv3d_thin_planes.inc) and the split that feeds them
p160 = K.split2(x160)
run("split2", lambda: K.split2(x160, out=p160))
cs = torch.zeros(C, device=dev)
run("split2_cs", lambda: K.split2(x160, out=p160, colsum=cs))
run("thin_out_p", lambda: K.conv3d_thin_out_planes(p160, wo, e, 8, grid, bias=b4))
run("wgrad_sfe_p", lambda: K.conv3d_thin_wgrad_planes(p160, x4, e, mx4, 1, grid, dw1))
run("wgrad_fin_p", lambda: K.conv3d_thin_wgrad_planes(p160, x4, e, mx4, 0, grid, dw2))
