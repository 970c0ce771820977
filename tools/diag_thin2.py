import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
import torch
from dl_cs.models import _ops as K
B, D, H, W = 1, 4, 4, 4
rows = 64
for ch in range(4):
    x = torch.zeros((rows, 8)); x[:, ch] = 1.0
    x[:, 4:] = 0
    g = torch.zeros((rows, 160)); g[:, 0] = 1.0
    dwp = torch.zeros((27, 160, 32), device="cuda")
    K.conv3d_wgrad(x.cuda().bfloat16(), 4, 0, g.cuda().bfloat16(), 160, (B, D, H, W), dwp)
    print("x ch", ch, "-> dW[13][0][:8]", dwp[13, 0, :8].tolist(), " dW[0][0][:4]", dwp[0, 0, :4].tolist())
