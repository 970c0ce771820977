"""Per-workgroup timestamps of the v5 forward conv (DLCS_CONV_STAMP=1): prologue,
main loop and epilogue cycles of each 256-voxel x 160-channel tile at the
BASELINE size.  Run on the GPU box:  DLCS_CONV_STAMP=1 python tools/conv_stamps.py"""
import os
os.environ.setdefault("DLCS_DIAG", "1")         # the diagnostic switches below are live
import ctypes
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
import torch  # noqa: E402
from dl_cs import _lib  # noqa: E402
from dl_cs.models import _ops as K  # noqa: E402

assert os.environ.get("DLCS_CONV_STAMP") == "1", "set DLCS_CONV_STAMP=1"
dt = torch.bfloat16
grid = (1, 28, 192, 160)
rows, C = 28 * 192 * 160, 160
x = torch.randn((rows, C), device="cuda").to(dt)
r = torch.randn((rows, C), device="cuda").to(dt)
w = torch.randn((C, C, 3, 3, 3), device="cuda") / (27 * C) ** 0.5
wf = K.conv_pack(w, dt, 0)
bias = torch.zeros(C, device="cuda")
for _ in range(5):
    K.conv3d(x, C, wf, C, C, grid, bias=bias, res=r, relu_out=1)
torch.cuda.synchronize()
L = _lib.lib()
buf = np.zeros(4096 * 4, dtype=np.uint64)
L.dlcs_debug_conv_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
assert L.dlcs_debug_conv_stamps(buf.ctypes.data, buf.size) == 0
st = buf.reshape(4096, 4)[:3360].astype(np.int64)
for name, d in (("prologue", st[:, 1] - st[:, 0]), ("main loop", st[:, 2] - st[:, 1]), ("epilogue", st[:, 3] - st[:, 2])):
    print(f"{name:10s} cycles: median {np.median(d):8.0f}  p10 {np.percentile(d, 10):8.0f}  p90 {np.percentile(d, 90):8.0f}")
