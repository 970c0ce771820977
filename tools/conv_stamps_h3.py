"""Per-workgroup cycle stamps of the fp32 f16x3 160 -> 160 forward conv at the
BASELINE grid (DIAG build): prologue (entry -> first barrier), each of the 70 barrier
steps, epilogue, and the gap from a workgroup's end to the start of the workgroup
dispatched 256 later (the same CU slot's next tile).  Shows where the kernel's time
goes beside the matrix work (70 steps x 120 MFMAs per wave x 16 cycles x 2 waves
per SIMD = 3840 cycles per step at full rate).
GPU box:  make -C dl-swin-gan_amd/csrc DIAG=1 &&
          DLCS_HIP_LIB=$PWD/dl-swin-gan_amd/dl_cs/libdlcs_hip_diag.so DLCS_DIAG=1 DLCS_CONV_STAMP=1 \
          python tools/conv_stamps_h3.py"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
import torch  # noqa: E402
from dl_cs import _lib  # noqa: E402
from dl_cs.models import _ops as K  # noqa: E402

assert os.environ.get("DLCS_CONV_STAMP") == "1" and os.environ.get("DLCS_DIAG") == "1"
L = _lib.lib()
assert hasattr(L, "dlcs_debug_h3_stamps"), "needs the DIAG build (libdlcs_hip_diag.so)"
grid = (1, 28, 192, 160)
rows, C = 28 * 192 * 160, 160
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn((rows, C), device="cuda", generator=g)
r = torch.randn((rows, C), device="cuda", generator=g)
w = torch.randn((C, C, 3, 3, 3), device="cuda", generator=g) / (27 * C) ** 0.5
xp = K.split2(x)
wf = K.conv_pack_f16x3(w, 0)
for _ in range(3):
    K.conv3d_f16x3(xp, wf, grid, res=r)
torch.cuda.synchronize()
n = 4096 * 73
buf = (ctypes.c_ulonglong * n)()
L.dlcs_debug_h3_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
assert L.dlcs_debug_h3_stamps(ctypes.addressof(buf), n) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 73).astype(np.int64)
nwg = 3328
st = st[:nwg]
t0 = st[:, 0].min()
pro = st[:, 1] - st[:, 0]
steps = np.diff(st[:, 1:72], axis=1)                      # 70 step durations
epi = st[:, 72] - st[:, 71]
tot = st[:, 72] - st[:, 0]
print(f"workgroups {nwg}; kernel span {(st[:, 72].max() - t0) / 1e3:.1f} k cycles")
print(f"per workgroup: total {tot.mean():.0f} cyc, prologue {pro.mean():.0f}, steps {steps.sum(1).mean():.0f} "
      f"({steps.mean():.0f} per step, median {np.median(steps):.0f}), epilogue {epi.mean():.0f}")
seam = steps[:, 13::14]
print(f"chunk-seam steps (13, 27, ...): {seam.mean():.0f} per step; other steps "
      f"{np.delete(steps, list(range(13, 70, 14)), axis=1).mean():.0f}")
print("mean step duration by position:", " ".join(f"{v:.0f}" for v in steps.mean(0)[:16]), "...")
nxt = st[256:, 0] - st[:-256, 72]
print(f"gap from a workgroup's end to workgroup b + 256's start: mean {nxt.mean():.0f} cyc, "
      f"median {np.median(nxt):.0f}, p10 {np.percentile(nxt, 10):.0f}")
ideal = 70 * 3840
print(f"matrix-only ideal per tile {ideal} cyc -> overhead {tot.mean() / ideal - 1:.1%} inside the workgroup")
