"""GPU time of dlcs_mhsa_fwd / dlcs_mhsa_bwd at the config-5 shapes (DiT: 16 heads of 24
over the 1,920 patches of each of 24 frames, and over the 24 frames of each patch;
Latte: 6 heads of 32, same token grid).  The f32-MFMA backward for an A/B:
  DLCS_DIAG=1 DLCS_MHSA_H3_BWD=0 DLCS_HIP_LIB=dl-swin-gan_amd/dl_cs/libdlcs_hip_diag.so python tools/mhsa_bench.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "dl-swin-gan_amd"), REPO]
import torch  # noqa: E402
from dl_cs import _lib  # noqa: E402
from dl_cs.models import _ops as K  # noqa: E402

iters = 10


def timed(fn):
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


dev = "cuda"
for name, nseq, N, heads, hd in (("dit spatial", 24, 1920, 16, 24), ("dit temporal", 1920, 24, 16, 24),
                                 ("latte spatial", 24, 1920, 6, 32), ("latte temporal", 1920, 24, 6, 32)):
    C = heads * hd
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn((nseq * N, 3 * C), device=dev, generator=g)
    dout = torch.randn((nseq * N, C), device=dev, generator=g)
    out = torch.empty((nseq * N, C), device=dev)
    lse = torch.empty((nseq, heads, N), device=dev)
    dq = torch.empty_like(qkv)
    nb = int(_lib.lib().dlcs_mhsa_bwd_workspace_bytes(nseq, N, heads))
    ws = torch.empty((nb // 4,), device=dev)
    sc = hd ** -0.5
    fwd = lambda: _lib.call("dlcs_mhsa_fwd", K.F32, K.p(qkv), K.p(out), K.p(lse), nseq, N, heads, hd, sc, K.S())  # noqa: E731
    bwd = lambda: _lib.call("dlcs_mhsa_bwd", K.F32, K.p(qkv), K.p(out), K.p(dout), K.p(lse), K.p(dq), nseq, N,  # noqa: E731
                            heads, hd, sc, K.p(ws), nb, K.S())
    tf = timed(fwd)
    tb = timed(bwd)
    print(f"{name:15s} nseq={nseq:5d} N={N:5d} heads={heads:2d} hd={hd}: fwd {tf:8.1f} us  bwd {tb:8.1f} us", flush=True)
