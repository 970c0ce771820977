"""Accuracy of the split path's 160 -> 160 conv input gradients on the bench.py
probe input (the config regularizer on the BASELINE slice's A^H y): each captured
dgrad (engine.DGRAD_CAPTURE) is recomputed in float64 on the CPU from its fp32
input gradient, and the f16x3 output and the f32 kernel's output are compared
with it (NRMSE over all, over the unmasked rows, and the relative bias).

    python tools/dgrad_diag.py [X]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "dl-swin-gan_amd")):
    sys.path.insert(0, p)


def to_ncdhw(t, grid, C):
    """patch-blocked rows [B, nT, nY, nX, 4, 4, 4][C] -> [B, C, D, H, W]"""
    B, D, H, W = grid
    t = t[:, :C].reshape(B, D // 4, H // 4, W // 4, 4, 4, 4, C)
    return t.permute(0, 7, 1, 4, 2, 5, 3, 6).reshape(B, C, D, H, W)


def nrmse(ref, x):
    return float(np.sqrt(np.mean((x - ref) ** 2)) / max(np.sqrt(np.mean(ref ** 2)), 1e-300))


def main():
    X = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    torch.set_num_threads(16)
    import bench
    from dl_cs.models import _ops as K
    from dl_cs.models import engine, swin3D
    swin3D.set_compute_dtype(torch.float32)
    dev = torch.device("cuda", 0)
    sys.argv = [sys.argv[0], "--nx", str(X)]
    args = bench.parse()
    model, _ = bench.build_model(args, dev)
    net = model.cnn_update[0]
    net.eval()
    x = bench.make_slice(args, 0, dev)["x0"].detach()
    engine.CAPTURE = []
    engine.DGRAD_CAPTURE = []
    try:
        y = net(x)
        g = torch.randn(y.shape, dtype=y.dtype, device=dev, generator=torch.Generator(dev).manual_seed(3))
        (y.real * g.real + y.imag * g.imag).sum().backward()
        caps = engine.DGRAD_CAPTURE
    finally:
        engine.CAPTURE = engine.DGRAD_CAPTURE = None
    for name, gin, mask, w, out in caps:
        if mask is None:
            # the unembed input gradient: d_tok [ntok, C] = g_a [ntok, 64 C] @ unemb [64 C, C]
            C = out.shape[1]
            ga = gin.reshape(-1, 64 * C)
            wm = w.detach().reshape(64 * C, C)
            ref = (ga.double().cpu() @ wm.double().cpu()).numpy()
            h = out.double().cpu().numpy()
            f32 = (ga.float() @ wm.float()).double().cpu().numpy()
            report(name, ref, {"h3r": h, "torch": f32}, axis=0)
            continue
        rows = gin.shape[0]
        # the grid: B = 1, D = T + 2 pad, H = Y, W = X of the captured slice
        B, E, T, Y, Xs = x.shape
        grid = (B, T + 8, Y, Xs)
        assert grid[0] * grid[1] * grid[2] * grid[3] == rows
        C = 160
        gd = to_ncdhw(gin.double().cpu(), grid, C)
        wd = w.detach().double().cpu()
        ref = torch.nn.functional.conv_transpose3d(gd, wd, padding=1)
        md = to_ncdhw((mask > 0).double().cpu(), grid, C)
        ref = (ref * md).numpy()
        h3 = to_ncdhw(out.double().cpu(), grid, C).numpy()
        f32 = K.conv3d(gin, C, K.conv_pack(w.detach(), torch.float32, 1), C, C, grid, mask=mask)
        f32 = to_ncdhw(f32.double().cpu(), grid, C).numpy()
        print(f"{name}: rows {rows} masked-in {(md.numpy() > 0).mean():.3f}  |g| max {gin.abs().max().item():.3e} "
              f"rms {gin.pow(2).mean().sqrt().item():.3e}")
        report(name, ref, {"f16x3": h3, "f32": f32}, axis=(0, 2, 3, 4))


def report(name, ref, outs, axis):
    """element NRMSE, and the error of the per-channel sums (a bias gradient, or any
    reduction over rows): a coherent error component survives those where the element
    error averages out"""
    cs = np.sum(ref, axis=axis)
    ca = np.sum(np.abs(ref), axis=axis)
    print(f"{name}: per-channel |sum| / sum|.| median {np.median(np.abs(cs) / ca):.3e}")
    for lab, v in outs.items():
        ce = np.sum(v - ref, axis=axis)
        print(f"  {lab:6s} nrmse {nrmse(ref, v):.3e}  colsum nrmse {nrmse(cs, cs + ce):.3e}  "
              f"mean err/mean|ref| {np.mean(v - ref) / np.mean(np.abs(ref)):+.3e}")


if __name__ == "__main__":
    main()
