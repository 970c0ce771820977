"""Accuracy of the f16x3 conv weight gradient vs float64, against PyTorch's own
fp32 (CPU) error, as a function of the accumulation chain length (voxel ranges
per launch: DLCS_WGH3_RANGES is read once per process, so run one process per
value):  python tools/wgrad_err.py RANGES [T Y X]

Also the forward conv and the dgrad at the same grid for comparison."""
import os
os.environ.setdefault("DLCS_DIAG", "1")         # the diagnostic switches below are live
import sys

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
from dl_cs.models import _ops as K  # noqa: E402


def blocked(v):
    """[1, C, T, Y, X] -> patch-blocked rows [T Y X, C] (engine layout)."""
    _, C, T, Y, X = v.shape
    return (v[0].reshape(C, T // 4, 4, Y // 4, 4, X // 4, 4).permute(1, 3, 5, 2, 4, 6, 0)
            .reshape(-1, C).contiguous())


def unblocked(r, T, Y, X):
    C = r.shape[1]
    return r.reshape(T // 4, Y // 4, X // 4, 4, 4, 4, C).permute(6, 0, 3, 1, 4, 2, 5).reshape(1, C, T, Y, X)


def nrmse(ref, x):
    ref, x = ref.double().flatten(), x.double().flatten()
    return float((x - ref).norm() / ref.norm())


def main():
    T, Y, X = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (28, 48, 48)
    torch.set_num_threads(16)
    g0 = torch.Generator().manual_seed(5)
    C = 160
    x = torch.relu(torch.randn((1, C, T, Y, X), generator=g0))
    go = torch.randn((1, C, T, Y, X), generator=g0)
    w = torch.randn((C, C, 3, 3, 3), generator=g0) / (27 * C) ** 0.5
    # float64 and fp32 references (CPU)
    x64, g64 = x.double().requires_grad_(), go.double()
    w64 = w.double().requires_grad_()
    y64 = F.conv3d(x64, w64, padding=1)
    (y64 * g64).sum().backward()
    x32, w32 = x.clone().requires_grad_(), w.clone().requires_grad_()
    y32 = F.conv3d(x32, w32, padding=1)
    (y32 * go).sum().backward()
    grid = (1, T, Y, X)
    dev = "cuda"
    xb, gb = blocked(x).to(dev), blocked(go).to(dev)
    xp, gp = K.split2(xb), K.split2(gb)
    dwp = torch.zeros((27, C, C), device=dev)
    K.conv3d_wgrad_f16x3(xp, gp, grid, dwp)
    dw = torch.zeros((C, C, 3, 3, 3), device=dev)
    K.conv_unpack_grad(dwp, dw, C, C)
    yh = K.conv3d_f16x3(xp, K.conv_pack_f16x3(w.to(dev), 0), grid)
    dxh = K.conv3d_f16x3(gp, K.conv_pack_f16x3(w.to(dev), 1), grid)
    torch.cuda.synchronize()
    r = os.environ.get("DLCS_WGH3_RANGES", "28")
    print(f"grid {T}x{Y}x{X} ranges {r}: wgrad f16x3 {nrmse(w64.grad, dw.cpu()):.3e}  torch fp32 "
          f"{nrmse(w64.grad, w32.grad):.3e} | fwd f16x3 {nrmse(y64, unblocked(yh.cpu(), T, Y, X)):.3e} torch "
          f"{nrmse(y64, y32):.3e} | dgrad f16x3 {nrmse(x64.grad, unblocked(dxh.cpu(), T, Y, X)):.3e} torch "
          f"{nrmse(x64.grad, x32.grad):.3e}")


if __name__ == "__main__":
    main()
