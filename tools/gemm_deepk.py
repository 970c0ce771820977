"""Times the two deep-K patch GEMMs of the regularizer at the BASELINE size
(embed fwd: tok += s . W_emb^T, K = 64 x 160; unembed dgrad: d_tok += g_a . W_unemb)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
import torch  # noqa: E402
from dl_cs.models import _ops as K  # noqa: E402

C, ntok = 160, 7 * 48 * 40
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
s = (torch.randn((ntok * 64, C), device=dev, generator=g) * 0.1).to(torch.bfloat16)
w = (torch.randn((C, 64 * C), device=dev, generator=g) * 0.01).to(torch.bfloat16)
wu = (torch.randn((64 * C, C), device=dev, generator=g) * 0.01).to(torch.bfloat16)
tok = torch.zeros((ntok, C), device=dev)
ref = (s.view(ntok, 64 * C).float() @ w.float().t())
K.gemm(s, w, tok, ntok, C, 64 * C, 64 * C, 64 * C, C, accumulate=1)
err = (tok - ref).norm() / ref.norm()
print(f"embed fwd rel err {float(err):.2e}")
for name, fn in (("embed_fwd", lambda: K.gemm(s, w, tok, ntok, C, 64 * C, 64 * C, 64 * C, C, accumulate=1)),
                 ("unembed_dgrad", lambda: K.gemm(s, wu, tok, ntok, C, 64 * C, 64 * C, C, C, b_trans=1, accumulate=1))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:14s} {e0.elapsed_time(e1) / 20 * 1e3:7.1f} us")
