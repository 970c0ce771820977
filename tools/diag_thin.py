"""Per-tap / per-channel error map of the thin-channel wgrad vs fp64 torch."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd")); sys.path.insert(0, os.path.join(REPO, "tests"))
import torch, torch.nn.functional as F
from test_gpu_kernels import _to_blocked, _from_blocked, _pad_cols
from dl_cs.models import _ops as K
cin, cout = int(sys.argv[1]), int(sys.argv[2])
B, D, H, W = 1, 8, 16, 12
g0 = torch.Generator().manual_seed(0)
x = torch.randn((B, cin, D, H, W), generator=g0); g = torch.randn((B, cout, D, H, W), generator=g0)
xr = _pad_cols(_to_blocked(x), max(8, cin)).cuda().bfloat16(); gr = _pad_cols(_to_blocked(g), max(8, cout)).cuda().bfloat16()
xq = _from_blocked(xr[:, :cin].float().cpu(), B, cin, D, H, W); gq = _from_blocked(gr[:, :cout].float().cpu(), B, cout, D, H, W)
dwp = torch.zeros((27, K.pad32(cout), K.pad32(cin)), device="cuda")
K.conv3d_wgrad(xr, cin, 0, gr, cout, (B, D, H, W), dwp)
gw = torch.zeros((cout, cin, 3, 3, 3), device="cuda"); K.conv_unpack_grad(dwp, gw, cout, cin)
w_ = torch.zeros((cout, cin, 3, 3, 3), dtype=torch.float64, requires_grad=True)
F.conv3d(xq.double(), w_, None, padding=1).backward(gq.double())
ref = w_.grad.reshape(cout, cin, 27); got = gw.cpu().double().reshape(cout, cin, 27)
e = (ref - got).abs() / ref.abs().mean()
print("per tap max rel err:", [round(float(v), 3) for v in e.amax(dim=(0, 1))])
print("per ci max:", [round(float(v), 3) for v in e.amax(dim=(0, 2))][:16])
print("per co max:", [round(float(v), 3) for v in e.amax(dim=(1, 2))][:160])
