"""Diagnostic (not a test): localise fused-path error vs an fp64 oracle."""
import os, sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))  # run from the repo root
import conftest  # noqa
import torch, torch.nn.functional as F
from goldutil import nrmse
from oracle import dlcs_oracle as O, recipe
from oracle.shapes import swinnet_param_shapes
from dl_cs.models import swin3D, engine
swin3D.set_compute_dtype(torch.float32)

def from_blocked(r, B, C, D, H, W):
    t = r.reshape(B, D // 4, H // 4, W // 4, 4, 4, 4, C).permute(0, 1, 4, 2, 5, 3, 6, 7)
    return t.reshape(B, D, H, W, C).permute(0, 4, 1, 2, 3)

net = swin3D.SwinTransformer3DNet(num_swinblocks=1, in_chans=4, chans=160, kernel_size=3, window_size=(4, 4)); net.eval()
recipe.fill_module(net, 31); net = net.cuda()
P = {k: recipe.param_value(31, k, s).double() for k, s in swinnet_param_shapes().items()}
x = recipe.crandn(32, (1, 2, 20, 32, 32))
# oracle pieces (fp64)
u = torch.cat((x.real, x.imag), 1).double(); u = F.pad(u, (0, 0, 0, 0, 4, 4), mode="circular")
s = O.conv_block(P, "SFE.", u, act=False)
pre = "DFE.resswin_blocks.0.layers.0.transformer."
emb = F.conv3d(s, P[pre + "patch_embed.proj.weight"], P[pre + "patch_embed.proj.bias"], stride=4)
tok_ref = emb.permute(0, 2, 3, 4, 1).reshape(-1, 160)
a_ref = O.swin3d(P, pre, s)
# mine
Pm = net.engine_params()
W = engine.NetWeights(Pm, torch.float32, 6)
out, sv = engine.swinnet_forward(W, x.cuda())
B, C, D, H, Wd = 1, 160, 28, 32, 32
print("s   ", nrmse(s.numpy(), from_blocked(sv["s"].cpu(), B, C, D, H, Wd).double().numpy()))
print("tok0", nrmse(tok_ref.numpy(), sv["bsaved"][0]["x"].cpu().double().numpy()))
t = tok_ref.view(1, 7, 8, 8, 160)
mask = torch.from_numpy(__import__("oracle.windex", fromlist=["x"]).compute_mask(7, 8, 8, (7, 8, 8), (0, 0, 0))).double()
for i in range(6):
    t = O.swin_block(P, f"{pre}layers.0.blocks.{i}.", t, (0, 0, 0) if i % 2 == 0 else (3, 4, 4), mask, 8, (7, 8, 8))
    mine = sv["bsaved"][i + 1]["x"] if i < 5 else sv["tok_t"]
    print(f"blk{i}", nrmse(t.reshape(-1, 160).numpy(), mine.cpu().double().numpy()))
print("a   ", nrmse(a_ref.numpy(), from_blocked(sv["a"].cpu(), B, C, D, H, Wd).double().numpy()))
print("out ", nrmse(O.swinnet(P, x.to(torch.complex128)).numpy(), out.cpu().numpy()))
# ---- backward
Pg = {k: v.clone().requires_grad_() for k, v in P.items()}
xx = x.to(torch.complex128)
u2 = F.pad(torch.cat((xx.real, xx.imag), 1), (0, 0, 0, 0, 4, 4), mode="circular")
s2 = O.conv_block(Pg, "SFE.", u2, act=False)
a2 = O.swin3d(Pg, pre, s2); a2.retain_grad()
b2 = O.conv_block(Pg, "DFE.resswin_blocks.0.layers.1.", a2) + s2; b2.retain_grad()
h2 = s2 + O.conv_block(Pg, "DFE.layers.1.", b2) + s2; h2.retain_grad()
o2 = O.conv_block(Pg, "final_layer.", h2)[:, :, 4:24]
y2 = torch.complex(o2[:, :2], o2[:, 2:])
gr = recipe.crandn(33, y2.shape).to(torch.complex128)
(y2.real * gr.real + y2.imag * gr.imag).sum().backward()
grads = {n: torch.zeros_like(p) for n, p in W.p.items()}
grads["emb_packed"] = torch.zeros((C, 64 * C), device="cuda")
grads["unemb_packed"] = torch.zeros((64 * C, C), device="cuda")
dbg = {}
engine.swinnet_backward(W, sv, gr.to(torch.complex64).cuda(), grads, dbg=dbg)
print("g_h ", nrmse(h2.grad.numpy(), from_blocked(dbg["g_h"].cpu(), B, C, D, H, Wd).double().numpy()))
print("g_b ", nrmse(b2.grad.numpy(), from_blocked(dbg["g_b"].cpu(), B, C, D, H, Wd).double().numpy()))
print("g_a ", nrmse(a2.grad.numpy(), from_blocked(dbg["g_a"].cpu(), B, C, D, H, Wd).double().numpy()))
for k in ["patch_unembed.proj.bias", "blocks.5.mlp.fc2.bias", "blocks.5.norm2.bias", "blocks.0.norm1.weight", "swin_tail.weight", "patch_embed.proj.weight"]:
    rk = {"swin_tail.weight": "DFE.resswin_blocks.0.layers.1.layers.2.conv.weight"}.get(k, pre + k.replace("blocks.", "layers.0.blocks."))
    print(k, nrmse(Pg[rk].grad.numpy(), grads[k].cpu().double().numpy()))
am = from_blocked(sv["a"].cpu(), B, C, D, H, Wd).double()
print("sign mismatch a:", int(((am > 0) != (a_ref > 0)).sum()), "zeros mine/ref:", int((am == 0).sum()), int((a_ref == 0).sum()), "numel", am.numel())
gbm = from_blocked(dbg["g_b"].cpu(), B, C, D, H, Wd).double().requires_grad_(False)
am_ = am.clone().requires_grad_()
yy = F.conv3d(F.relu(am_), Pg["DFE.resswin_blocks.0.layers.1.layers.2.conv.weight"].detach(), None, padding=1)
yy.backward(gbm)
gam = from_blocked(dbg["g_a"].cpu(), B, C, D, H, Wd).double()
print("g_a vs torch(dgrad of my g_b, my a):", nrmse(am_.grad.numpy(), gam.numpy()))
print("g_a vs ref, where a>0 agrees:", nrmse((a2.grad * (a_ref > 0)).numpy(), (gam * (a_ref > 0)).numpy()))
err = (gam - a2.grad).abs()
print("err by t:", [float(err[:, :, t].max()) for t in range(0, 28, 3)])
print("err by channel blocks:", [float(err[:, c:c+32].max()) for c in range(0, 160, 32)])
