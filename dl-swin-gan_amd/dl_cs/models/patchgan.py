"""Conv PatchGAN discriminator for Swin-GAN training (BASELINE config 3).

The reference names a Swin-GAN run (run_script.sh:29, :45-47, :144-155) but does
not ship its discriminator (`scripts/train_swin_gan.py` and
`configs/config_swingan.yaml` are missing), so this network
is build-defined and its parity is pinned only against this package's own CPU
restatement (oracle/dlcs_oracle.py::patchgan) -- "parity unpinned" against the
reference.

Architecture (3-D PatchGAN in the reference's own pre-activation ConvBlock
idiom, s3d:225-273, sized so every layer runs on the generator's tuned
kernels):

    x complex [B, E, T, Y, X] -> cat(re, im) channels [B, 2E, T, Y, X]  (s3d:394-406)
    c1 = Conv3d(2E -> F, k3, pad 1)          thin-input conv (fp32: dlcs_conv3d_thin_f16x3)
    c2 = Conv3d(F -> F, k3, pad 1)(relu c1)  160 -> 160 conv (fp32: dlcs_conv3d_k3_f16x3)
    p  = Conv3d(F -> F, k4, s4)(relu c2)     GEMM on the patch-blocked layout (fp32: dlcs_gemm_h3r)
    logits = Conv3d(F -> 1, k1)(relu p)      dlcs_gemm

In fp32 every conv and patch GEMM runs on the generator's fp16 / bf16 plane-split
kernels (fp32 accuracy on 16-bit matrix cores), its backward too.
    -> patch logits [B, 1, T/4, Y/4, X/4]  (each logit sees a 4x4x4 patch + 2-voxel halo)

ReLU (not LeakyReLU) because the conv epilogues fuse ReLU; F = NUM_FEATURES
(160 at config_swin).  Requires T, Y, X divisible by 4 (no time padding:
20 frames at BASELINE).  Forward and backward are hand-scheduled HIP launches
inside one torch.autograd.Function; the gradient w.r.t. x flows back to the
generator for the adversarial term.
"""
import weakref

import torch
from torch import nn
import torch.nn.functional as F

from .. import _lib
from . import _ops as K
from . import engine
from .swin3D import get_compute_dtype

PAD_CIN = 8          # channel stride of the 2E-channel volume (engine.PAD_CIN)


class PatchGANDiscriminator3D(nn.Module):
    NAMES = ("conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias",
             "patch.weight", "patch.bias", "head.weight", "head.bias")

    def __init__(self, in_chans=4, chans=160):
        super().__init__()
        self.in_chans, self.chans = in_chans, chans
        self.conv1 = nn.Conv3d(in_chans, chans, 3, padding=1)
        self.conv2 = nn.Conv3d(chans, chans, 3, padding=1)
        self.patch = nn.Conv3d(chans, chans, 4, stride=4)
        self.head = nn.Conv3d(chans, 1, 1)

    def forward(self, x):
        """x complex64 [B, E, T, Y, X] on the GPU -> fp32 logits [B, 1, T/4, Y/4, X/4]."""
        assert torch.is_complex(x)
        _lib.require_gpu(x)
        B, E, T, Y, X = x.shape
        if 2 * E != self.in_chans or T % 4 or Y % 4 or X % 4:
            raise NotImplementedError("PatchGANDiscriminator3D: need 2E == in_chans and T, Y, X % 4 == 0")
        params = [getattr(self, n.split(".")[0]).get_parameter(n.split(".")[1]) for n in self.NAMES]
        return _PatchGANFn.apply(x, get_compute_dtype(), *params)


def _split(dtype, C):
    """fp32 with C == 160: the convs and patch GEMMs on the generator's fp16-split
    kernels (engine.FP32_CONV == 'f16x3'; the thin-input conv1, the 160 -> 160 conv2,
    the row-scaled split-K patch GEMM (dlcs_gemm_h3r), the K = 160 GEMM of its input
    gradient)."""
    return dtype == torch.float32 and C == 160 and engine.X6


_PATCH_PACK = []        # [(weakref to patch.weight, version, data_ptr, h3r packing)], most recent first


def _patch_h3r(w, wp, C):
    """The h3r packing of the patch GEMM's B operand, reused while the parameter is
    unchanged (identity, storage and in-place version, as the generator's NetWeights)."""
    for r, ver, ptr, packed in _PATCH_PACK:
        if r() is w and ver == w._version and ptr == w.data_ptr():
            return packed
    (packed,) = K.h3r_pack([(wp.reshape(C, 64 * C), False)])
    _PATCH_PACK.insert(0, (weakref.ref(w), w._version, w.data_ptr(), packed))
    del _PATCH_PACK[4:]
    return packed


def _forward(x, dtype, P):
    B, E, T, Y, X = x.shape
    C = P["conv1.bias"].shape[0]
    cin = 2 * E
    grid = (B, T, Y, X)
    rows = B * T * Y * X
    ntok = rows // 64
    dev = x.device
    split = _split(dtype, C)
    u = K.swin_pre(x.contiguous(), dtype, 0, PAD_CIN)
    w1 = K.conv_pack(P["conv1.weight"], dtype, 0)
    # k4 s4 conv = GEMM on the patch-blocked rows: B operand [co][(kd, kh, kw, ci)]
    wp = K.permute(P["patch.weight"], (C, 4, 4, 4, C), (C * 64, 16, 4, 1, 64), dst_dtype=dtype)
    a3 = K.empty((ntok, C), dtype, dev)
    sv = dict(u=u, wp=wp, shape=(B, E, T, Y, X), grid=grid, C=C, cin=cin, rows=rows, ntok=ntok, split=split)
    if split:
        umax = K.absmax(u)
        pa1 = K.planes_alloc(rows, dev)
        a1 = K.conv3d_thin_f16x3(u, cin, umax, K.thin_pack_f16x3(w1, C, cin, 0), C, C, grid, bias=P["conv1.bias"],
                                 relu_out=1, out_max=K.planes_max(pa1, rows))            # relu(c1)
        p1 = K.split2(a1, out=pa1, have_max=True)
        a2 = K.conv3d_f16x3(p1, K.conv_pack_f16x3(P["conv2.weight"], 0), grid, bias=P["conv2.bias"],
                            relu_out=1)                                                    # relu(c2)
        if engine.H3R:
            wph = _patch_h3r(P["patch.weight"], wp, C)
            K.linear_h3r(a2.view(ntok, 64 * C), wph, C, out=a3, bias=P["patch.bias"])      # p (fixed-order split-K)
            torch.relu_(a3)                                                                # relu(p)
        else:                                               # DLCS_DIAG=1 DLCS_H3R=0: the f32 GEMM
            K.gemm(a2, wp, a3, ntok, C, 64 * C, 64 * C, 64 * C, C, bias=P["patch.bias"], act=3)
        sv.update(umax=umax, p1=p1)
    else:
        w2 = K.conv_pack(P["conv2.weight"], dtype, 0)
        a1 = K.conv3d(u, cin, w1, C, C, grid, bias=P["conv1.bias"], relu_out=1)          # relu(c1)
        a2 = K.conv3d(a1, C, w2, C, C, grid, bias=P["conv2.bias"], relu_out=1)           # relu(c2)
        K.gemm(a2, wp, a3, ntok, C, 64 * C, 64 * C, 64 * C, C, bias=P["patch.bias"], act=3)   # relu(p)
    wh = K.cast(P["head.weight"].reshape(1, C).contiguous(), dtype)
    logits = K.empty((ntok, 1), torch.float32, dev)
    K.gemm(a3, wh, logits, ntok, 1, C, C, C, 1, bias=P["head.bias"])
    sv.update(a1=a1, a2=a2, a3=a3, wh=wh)
    if engine.CAPTURE is not None:                   # test hook: the three ReLU decisions (blocked, blocked, tokens)
        engine.CAPTURE.append(dict(relu_inputs=[a1, a2], tokens=[a3], grid=grid, C=C))
    return logits.view(B, 1, T // 4, Y // 4, X // 4), sv


def _backward(dtype, P, sv, glog):
    C, cin, grid, rows, ntok = sv["C"], sv["cin"], sv["grid"], sv["rows"], sv["ntok"]
    dev = glog.device
    G = {n: torch.zeros_like(P[n]) for n in PatchGANDiscriminator3D.NAMES}
    g = K.cast(glog.reshape(ntok, 1).contiguous().float(), dtype)      # GEMM operands share one dtype
    # head: logits = a3 . wh^T + bh
    K.gemm(g, sv["a3"], G["head.weight"].view(1, C), 1, C, ntok, 1, C, C, a_trans=1, b_trans=1,
           accumulate=1, splitk=max(1, min(64, ntok // 256)))
    K.colsum(g, G["head.bias"])
    da3 = K.empty((ntok, C), dtype, dev)
    K.gemm(g, sv["wh"], da3, ntok, C, 1, 1, C, C, b_trans=1)
    K.relu_grad(da3, sv["a3"])                                          # d(pre-ReLU p)
    # patch GEMM: p = a2_patch . wp^T + bp
    dwp = torch.zeros((C, 64 * C), dtype=torch.float32, device=dev)
    a2_tok = sv["a2"].view(ntok, 64 * C)
    if K.dw_grouped_ok(ntok, [(da3, a2_tok)]):
        K.gemm_dw_grouped(ntok, [(da3, a2_tok, dwp, G["patch.bias"], 0)])
    else:
        K.gemm(da3, sv["a2"], dwp, C, 64 * C, ntok, C, 64 * C, 64 * C, a_trans=1, b_trans=1,
               accumulate=1, splitk=max(1, min(16, ntok // 256)))
        K.colsum(da3, G["patch.bias"])
    K.permute(dwp, (C, C, 4, 4, 4), (64 * C, 1, 16 * C, 4 * C, C), out=G["patch.weight"], accumulate=1)
    da2 = K.empty((rows, C), dtype, dev)
    if sv["split"]:
        # K = 160 patch input gradient on the fp16 split (B = wp^T as [64 C][C] planes)
        wpT = K.split2(sv["wp"].reshape(C, 64 * C).t().contiguous())
        K.gemm_k160_f16x3(K.split2(da3), ntok, wpT, 64 * C, da2.view(ntok, 64 * C))
    else:
        K.gemm(da3, sv["wp"], da2, ntok, 64 * C, C, C, 64 * C, 64 * C, b_trans=1)
    K.relu_grad(da2, sv["a2"])                                          # d c2

    def conv_grads(x_in, cin_, gout, cout, wname, bname):
        dwk = torch.zeros((27, K.pad32(cout), K.pad32(cin_)), dtype=torch.float32, device=dev)
        K.conv3d_wgrad(x_in, cin_, 0, gout, cout, grid, dwk)
        K.conv_unpack_grad(dwk, G[wname], cout, cin_)
        K.colsum(gout, G[bname], rows=rows, C=cout, ld=gout.shape[-1])

    w1 = K.conv_pack(P["conv1.weight"], dtype, 1)
    if sv["split"]:
        # conv2: c2 = conv(a1); dgrad masked by relu'(c1) -> d c1 (its max for the thin conv1 kernels)
        gp = K.split2(da2, colsum=G["conv2.bias"])
        dc1max = K.zeros((1,), torch.int32, dev)
        dc1 = K.conv3d_f16x3(gp, K.conv_pack_f16x3(P["conv2.weight"], 1), grid, mask=sv["a1"], out_max=K.p(dc1max))
        dwk = torch.zeros((27, C, C), dtype=torch.float32, device=dev)
        K.conv3d_wgrad_f16x3(sv["p1"], gp, grid, dwk)
        K.conv_unpack_grad(dwk, G["conv2.weight"], C, C)
        del gp
        # conv1 (thin input): c1 = conv(u)
        du = K.conv3d_thin_f16x3(dc1, C, dc1max, K.thin_pack_f16x3(w1, cin, C, 1), cin, PAD_CIN, grid)
        dwk = torch.zeros((27, C, K.pad32(cin)), dtype=torch.float32, device=dev)
        K.conv3d_thin_wgrad_f16x3(sv["u"], cin, sv["umax"], dc1, C, dc1max, grid, dwk, colsum=G["conv1.bias"])
        K.conv_unpack_grad(dwk, G["conv1.weight"], C, cin)
    else:
        # conv2: c2 = conv(a1); dgrad masked by relu'(c1) -> d c1
        w2 = K.conv_pack(P["conv2.weight"], dtype, 1)
        dc1 = K.conv3d(da2, C, w2, C, C, grid, mask=sv["a1"])
        conv_grads(sv["a1"], C, da2, C, "conv2.weight", "conv2.bias")
        # conv1: c1 = conv(u)
        du = K.conv3d(dc1, C, w1, cin, PAD_CIN, grid)
        conv_grads(sv["u"], cin, dc1, C, "conv1.weight", "conv1.bias")
    gx = K.swin_pre_bwd(du, sv["shape"], 0)
    return gx, G


class _PatchGANFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype, *plist):
        P = dict(zip(PatchGANDiscriminator3D.NAMES, plist))
        logits, sv = _forward(x.to(torch.complex64), dtype, P)
        ctx.state = (dtype, P, sv)
        return logits

    @staticmethod
    def backward(ctx, glog):
        dtype, P, sv = ctx.state
        ctx.state = None
        gx, G = _backward(dtype, P, sv, glog)
        return (gx, None) + tuple(G[n] for n in PatchGANDiscriminator3D.NAMES)


def d_loss(d_real, d_fake):
    """Discriminator loss: BCE-with-logits, real -> 1, fake -> 0 (mean over patches)."""
    return (F.binary_cross_entropy_with_logits(d_real, torch.ones_like(d_real)) +
            F.binary_cross_entropy_with_logits(d_fake, torch.zeros_like(d_fake)))


def g_adv_loss(d_fake):
    """Generator adversarial term: BCE-with-logits of D(G(y)) against 1."""
    return F.binary_cross_entropy_with_logits(d_fake, torch.ones_like(d_fake))
