"""The reference's per-module forwards on the HIP path (standalone autograd
nodes, dl_cs/models/_standalone.py) at sizes the fused path does not tile,
vs torch fp32 / the oracle: ConvBlock and Conv3d (s3d:120-273), PatchEmbed3D
with its end padding (vst:440-479), PatchUnembed3D with the reference's crop
(vst:481-531), SwinTransformer3D (vst:735-756) and SwinTransformer3DNet at
non-multiple-of-4 sizes (s3d:394-435, module-by-module path).  fp32:
outputs NRMSE <= 1e-5, gradients <= 1e-5 (the ReLU-masked regularizer
parameter gradients are held to the float64 floor, goldutil.assert_f64_floor)."""
import pytest
import torch
import torch.nn.functional as F

from goldutil import nrmse
from oracle import dlcs_oracle as O
from oracle import recipe

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _fp32():
    from dl_cs.models import swin3D
    old = swin3D.get_compute_dtype()
    swin3D.set_compute_dtype(torch.float32)
    yield
    swin3D.set_compute_dtype(old)


def _grads_close(mod, ref_params, tol):
    for n, p in mod.named_parameters():
        if n in ref_params and ref_params[n].grad is not None:
            assert nrmse(ref_params[n].grad.numpy(), p.grad.cpu().numpy()) < tol, n


@pytest.mark.parametrize("cin,cout,act,shape", [(4, 160, "none", (1, 6, 9, 10)), (160, 160, "relu", (2, 5, 7, 9)),
                                                (160, 4, "relu", (1, 8, 12, 12)), (12, 20, "relu", (1, 3, 5, 6))])
def test_convblock(cin, cout, act, shape):
    from dl_cs.models import swin3D
    blk = swin3D.ConvBlock(cin, cout, 3, act_type=act)
    recipe.fill_module(blk, 5)
    blk = blk.to(DEV)
    B, D, H, W = shape
    x = recipe.randn(6, (B, cin, D, H, W))
    xg = x.to(DEV).requires_grad_()
    y = blk(xg)
    g = recipe.randn(7, y.shape)
    (y * g.to(DEV)).sum().backward()
    w = blk.layers[2].conv.weight.detach().cpu().clone().requires_grad_()
    b = blk.layers[2].conv.bias.detach().cpu().clone().requires_grad_()
    xo = x.clone().requires_grad_()
    yo = F.conv3d(F.relu(xo) if act == "relu" else xo, w, b, padding=1)
    (yo * g).sum().backward()
    assert nrmse(yo.detach().numpy(), y.detach().cpu().numpy()) < 1e-5
    assert nrmse(xo.grad.numpy(), xg.grad.cpu().numpy()) < 1e-5
    assert nrmse(w.grad.numpy(), blk.layers[2].conv.weight.grad.cpu().numpy()) < 1e-5
    assert nrmse(b.grad.numpy(), blk.layers[2].conv.bias.grad.cpu().numpy()) < 1e-5


@pytest.mark.parametrize("shape", [(1, 7, 48, 40), (2, 6, 10, 13)])
def test_patch_embed_unembed(shape):
    from dl_cs.models import video_swin_transformer_mri_downsample as vst
    C, E = 20, 24
    pe = vst.PatchEmbed3D(patch_size=(4, 4, 4), in_chans=C, embed_dim=E)
    pu = vst.PatchUnembed3D([4, 4, 4], in_channels=C, embed_dim=E)
    recipe.fill_module(pe, 8)
    recipe.fill_module(pu, 9)
    pe, pu = pe.to(DEV), pu.to(DEV)
    B, D, H, W = shape
    x = recipe.randn(10, (B, C, D, H, W))
    xg = x.to(DEV).requires_grad_()
    t = pe(xg)
    y = pu(t, x.shape)
    g = recipe.randn(11, y.shape)
    (y * g.to(DEV)).sum().backward()
    P = {k: v.detach().cpu().clone().requires_grad_() for k, v in
         [("pe.w", pe.proj.weight), ("pe.b", pe.proj.bias), ("pu.w", pu.proj.weight), ("pu.b", pu.proj.bias)]}
    xo = x.clone().requires_grad_()
    xp = F.pad(xo, (0, (-W) % 4, 0, (-H) % 4, 0, (-D) % 4))                   # vst:464-470
    to = F.conv3d(xp, P["pe.w"], P["pe.b"], stride=4)
    yf = F.conv_transpose3d(to, P["pu.w"], P["pu.b"], stride=4)
    from dl_cs.models._standalone import center_crop_like_reference
    yo = center_crop_like_reference(yf, x.shape)
    (yo * g).sum().backward()
    assert nrmse(to.detach().numpy(), t.detach().cpu().numpy()) < 1e-5
    assert nrmse(yo.detach().numpy(), y.detach().cpu().numpy()) < 1e-5
    assert nrmse(xo.grad.numpy(), xg.grad.cpu().numpy()) < 1e-5
    for k, p in (("pe.w", pe.proj.weight), ("pe.b", pe.proj.bias), ("pu.w", pu.proj.weight), ("pu.b", pu.proj.bias)):
        assert nrmse(P[k].grad.numpy(), p.grad.cpu().numpy()) < 1e-5, k


def test_swin_transformer3d_module():
    from dl_cs.models import video_swin_transformer_mri_downsample as vst
    m = vst.SwinTransformer3D(in_chans=160, embed_dim=160, depths=[6], num_heads=[8], window_size=(7, 8, 8))
    m.eval()
    recipe.fill_module(m, 12)
    m = m.to(DEV)
    x = recipe.randn(13, (1, 160, 28, 32, 30)) * 0.5
    xg = x.to(DEV).requires_grad_()
    y = m(xg)
    g = recipe.randn(14, y.shape)
    (y * g.to(DEV)).sum().backward()
    P = {k: v.detach().cpu().clone().requires_grad_(torch.is_floating_point(v) and "relative_position_index" not in k)
         for k, v in m.state_dict().items()}
    xo = x.clone().requires_grad_()
    yo = O.swin3d(P, "", xo)
    (yo * g).sum().backward()
    assert nrmse(yo.detach().numpy(), y.detach().cpu().numpy()) < 1e-5
    assert nrmse(xo.grad.numpy(), xg.grad.cpu().numpy()) < 1e-5
    _grads_close(m, P, 1e-4)


def test_swinnet_non_multiple_of_4():
    """SwinTransformer3DNet at Y = 30, X = 26 (not tiled by the fused path):
    the module-by-module HIP path vs the oracle, forward and backward."""
    from dl_cs.models import swin3D
    net = swin3D.SwinTransformer3DNet(num_swinblocks=1, in_chans=4, chans=160, kernel_size=3, window_size=(4, 4))
    net.eval()
    recipe.fill_module(net, 15)
    net = net.to(DEV)
    x = recipe.crandn(16, (1, 2, 20, 30, 26))
    xg = x.to(DEV).requires_grad_()
    y = net(xg)
    g = recipe.crandn(17, y.shape)
    (y.real * g.real.to(DEV) + y.imag * g.imag.to(DEV)).sum().backward()
    P = {k: v.detach().cpu().clone().requires_grad_(torch.is_floating_point(v) and "relative_position_index" not in k)
         for k, v in net.state_dict().items()}
    xo = x.clone().requires_grad_()
    yo = O.swinnet(P, xo)
    (yo.real * g.real + yo.imag * g.imag).sum().backward()
    assert nrmse(yo.detach().numpy(), y.detach().cpu().numpy()) < 1e-5
    from test_gpu_fullsize import swinnet_grads_f64
    from goldutil import assert_f64_floor
    dx64, pg64 = swinnet_grads_f64(net.state_dict(), x, g)
    floor = nrmse(dx64, xo.grad.numpy())
    err = nrmse(dx64, xg.grad.cpu().numpy())
    print(f"dx err vs f64 {err:.3g}, oracle32 floor {floor:.3g}")
    assert err < max(1e-5, 4 * floor), (err, floor)
    o32 = {n: v.grad.numpy() for n, v in P.items() if torch.is_tensor(v) and v.grad is not None}
    assert_f64_floor({n: p.grad for n, p in net.named_parameters() if p.grad is not None}, o32, pg64,
                     "swinnet 30x26 (module path)")
