"""DIAG timing experiments on the fp32 (h3) window attention kernels at the BASELINE
geometry with region labels of the shifted blocks (10 of 30 windows mixed, as
compute_mask): DLCS_ATTN_EXP bits skip parts of the inner loops (outputs wrong).
Run with the DIAG library:
  DLCS_DIAG=1 DLCS_HIP_LIB=dl-swin-gan_amd/dl_cs/libdlcs_hip_diag.so python tools/attn_exp.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "dl-swin-gan_amd"), REPO]
import torch  # noqa: E402
from dl_cs.models import _ops as K  # noqa: E402
from oracle import windex  # noqa: E402

iters = 20
dt = torch.float32 if (len(sys.argv) < 2 or sys.argv[1] == "fp32") else torch.bfloat16
nwin, N, heads, hd, window = 30, 448, 8, 20, (7, 8, 8)
C, scale = heads * hd, hd ** -0.5
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn((nwin * N, 3 * C), device=dev, generator=g).to(dt)
table = torch.randn((13 * 15 * 15, heads), device=dev, generator=g) * 0.1
# the shifted block's region labels at the BASELINE token grid (7, 48, 40), shift (0, 4, 4), window order
lab = windex.region_labels(7, 48, 40, window, (0, 4, 4))
lab = lab.reshape(1, 7, 6, 8, 5, 8).transpose(0, 2, 4, 1, 3, 5).reshape(-1)
labels = torch.from_numpy(lab).int().to(dev)
dout = torch.randn((nwin * N, C), device=dev, generator=g).to(dt)
dtab = torch.zeros_like(table)
out, lse = K.attn_fwd(qkv, table, labels, nwin, N, heads, hd, window, scale)


def timed(fn):
    """GPU time per call: the calls captured in a HIP graph and replayed (the ctypes
    launch path costs more host time per call than these kernels take)."""
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(iters):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (3 * iters) * 1e3


fwd = lambda: K.attn_fwd(qkv, table, labels, nwin, N, heads, hd, window, scale)   # noqa: E731
bwd = lambda: K.attn_bwd(qkv, out, dout, lse, table, labels, dtab, nwin, N, heads, hd, window, scale)   # noqa: E731
cases = [("fwd", fwd, e, n) for e, n in ((0, "base"), (1, "no bias gather"), (2, "no PV mfma"), (4, "no S mfma"),
                                         (8, "no exp"), (16, "no P split"), (6, "no mfma"), (1 | 8 | 16, "no bias/exp/split"))]
cases += [("kv", bwd, 8192 | e, n) for e, n in ((0, "base"), (32, "no table bins"), (64, "no dK/dV mfma"),
                                                 (128, "no S/dP mfma"), (256, "no bias gather"), (192, "no mfma"),
                                                 (32 | 256, "no bins/gather"))]
cases += [("q", bwd, 16384 | e, n) for e, n in ((0, "base"), (1024, "no bias gather"), (2048, "no dQ mfma"),
                                                 (4096, "no S/dP mfma"), (2048 | 4096, "no mfma"))]
if len(sys.argv) > 2 and sys.argv[2] == "base":
    cases = [c for c in cases if c[3] == "base"]
for kind, fn, e, name in cases:
    os.environ["DLCS_ATTN_EXP"] = str(e)
    print(f"{kind:4s} {str(dt):14s} exp={e:6d} {name:22s} {timed(fn):8.1f} us", flush=True)
os.environ["DLCS_ATTN_EXP"] = "0"
