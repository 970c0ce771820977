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
dt = torch.float32 if (len(sys.argv) > 3 and sys.argv[3] == "fp32") else torch.bfloat16
PEAK = 157.3 if dt == torch.float32 else 2500.0
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
    print(f"{name:8s} {ms:7.3f} ms  {flops / ms / 1e9:7.1f} TFLOP/s  ({flops / ms / 1e9 / PEAK * 100:4.1f}% of {dt} peak)")


if which in ("all", "fwd"):
    run("fwd", lambda: K.conv3d(x, C, wf, C, C, grid, bias=bias, res=r, relu_out=1))
if which in ("all", "dgrad"):
    run("dgrad", lambda: K.conv3d(x, C, wd, C, C, grid, mask=r))
if which in ("all", "wgrad"):
    run("wgrad", lambda: K.conv3d_wgrad(x, C, 0, r, C, grid, dwp))

# fp32 on bf16 matrix cores (3-plane split): split + conv, and the conv alone
if which in ("all", "x6") and dt == torch.float32:
    wx = K.conv_pack_x6(w, 0)
    planes = K.split3(x)
    PEAK_SAVE = PEAK
    run("x6_fwd", lambda: K.conv3d_x6(planes, wx, grid, bias=bias, res=r, relu_out=1))
    run("x6_dgr", lambda: K.conv3d_x6(planes, wx, grid, mask=r))
    run("split3", lambda: K.split3(x, planes))
    gplanes = K.split3(r)
    run("x6_wgr", lambda: K.conv3d_wgrad_x6(planes, gplanes, grid, dwp))

# fp32 on fp16 matrix cores (2-plane split, 3 products): split + conv, and the conv alone
if which in ("all", "f16x3") and dt == torch.float32:
    wh = K.conv_pack_f16x3(w, 0)
    hp = K.split2(x)
    run("h3_fwd", lambda: K.conv3d_f16x3(hp, wh, grid, bias=bias, res=r, relu_out=1))
    run("h3_dgr", lambda: K.conv3d_f16x3(hp, wh, grid, mask=r))
    run("split2", lambda: K.split2(x, hp))
    gh = K.split2(r)
    run("h3_wgr", lambda: K.conv3d_wgrad_f16x3(hp, gh, grid, dwp))
    # K = 160 patch GEMM (unembed forward: 13440 tokens x 10240 outputs)
    tok = torch.randn((13440, 160), device=dev, generator=g)
    wu = torch.randn((10240, 160), device=dev, generator=g) / 160 ** 0.5
    ob = torch.empty((13440, 10240), device=dev)
    tp, wp = K.split2(tok), K.split2(wu)
    flops_save = flops
    flops = 3 * 2.0 * 13440 * 10240 * 160
    run("k160", lambda: K.gemm_k160_f16x3(tp, 13440, wp, 10240, ob, act=3))
    r1, r2 = torch.randn_like(ob), torch.randn_like(ob)
    run("k160res", lambda: K.gemm_k160_f16x3(tp, 13440, wp, 10240, ob, res=r1, res_scale=2.0, res2=r2))
    flops = flops_save

# thin ends: SFE 4 -> 160 and final 160 -> 4 (8-column rows on the thin side)
if which in ("all", "thin"):
    x8 = torch.zeros((rows, 8), device=dev, dtype=dt)
    x8[:, :4] = torch.randn((rows, 4), device=dev, generator=g).to(dt)
    w_sfe = torch.randn((C, 4, 3, 3, 3), device=dev, generator=g) / (27 * 4) ** 0.5
    w_fin = torch.randn((4, C, 3, 3, 3), device=dev, generator=g) / (27 * C) ** 0.5
    ws_f, ws_d = K.conv_pack(w_sfe, dt, 0), K.conv_pack(w_sfe, dt, 1)
    wf_f, wf_d = K.conv_pack(w_fin, dt, 0), K.conv_pack(w_fin, dt, 1)
    dw_s = torch.zeros((27, C, 32), device=dev)
    dw_f = torch.zeros((27, 32, C), device=dev)
    flops = 2.0 * rows * C * 4 * 27
    run("sfe_fwd", lambda: K.conv3d(x8, 4, ws_f, C, C, grid, bias=bias))
    run("sfe_dgr", lambda: K.conv3d(x, C, ws_d, 4, 8, grid))
    run("sfe_wgr", lambda: K.conv3d_wgrad(x8, 4, 0, x, C, grid, dw_s))
    run("fin_fwd", lambda: K.conv3d(x, C, wf_f, 4, 8, grid, out_dtype=torch.float32))
    run("fin_dgr", lambda: K.conv3d(x8, 4, wf_d, C, C, grid, mask=r))
    run("fin_wgr", lambda: K.conv3d_wgrad(x, C, 0, x8, 4, grid, dw_f))
