"""3D ResNet regularizer of the reference's "dlespirit" unrolled network
(BASELINE config 1, configs/example.yaml), MI355X build.

Same classes, constructor arguments and state_dict keys as the reference
(r3d = dl_cs/models/resnet3d.py:163-317).  The whole network runs as one HIP
autograd node (_ResNetFn) on the generic Conv3d k3 kernels (dlcs_conv3d_k3 /
dlcs_conv3d_k3_wgrad, any channel count padded to 32) in the patch-blocked
channels-last layout of the Swin path.

The reference's pre-activation blocks use nn.ReLU(inplace=True) (r3d:39-55,
:200-208): a ResBlock's ReLU overwrites its input, so its residual adds
relu(input), not input (r3d:232-240), and the final layer's ReLU likewise
(r3d:308).  Every block output is therefore only ever consumed as relu(o), and
the HIP forward stores r = relu(o) straight from the producing conv's epilogue:

    u  = pre(x)                          cat(re, im), circular T pad (r3d:270-282)
    r0 = relu(conv0(u))                  init_layer, act 'none' (r3d:260, :305)
    t  = relu(conv_a(r_k))               ResBlock first ConvBlock + the second's ReLU
    r_{k+1} = relu(conv_b(t) + r_k)      ResBlock (r3d:232-240) + next block's ReLU
    out = conv_f(r_L) + u                final_layer + input (r3d:308)
    x'  = post(out)                      crop, complex (r3d:284-294)
"""
import torch
from torch import nn

from . import _ops as K
from .swin3D import ConvBlock, get_compute_dtype

PAD_CIN = 8


class ResBlock(nn.Module):
    """r3d:214-240 -- two pre-activation ConvBlocks and a residual connection."""

    def __init__(self, chans, kernel_size, act_type='relu', is_complex=False):
        super().__init__()
        self.layers = nn.Sequential(
            ConvBlock(chans, chans, kernel_size, act_type=act_type, is_complex=is_complex),
            ConvBlock(chans, chans, kernel_size, act_type=act_type, is_complex=is_complex))

    def forward(self, input):
        raise NotImplementedError("dl_cs: ResBlock runs inside ResNet's fused HIP node")


def _conv(x, cin, w, cout, out_ld, grid, **kw):
    return K.conv3d(x, cin, K.conv_pack(w, x.dtype, 0), cout, out_ld, grid, **kw)


def _dgrad(g, cout_w, w, cin_w, out_ld, grid, **kw):
    """dL/d(conv input) of a conv with weight w [cout_w, cin_w, 3, 3, 3] from g [rows, >= cout_w]."""
    return K.conv3d(g, cout_w, K.conv_pack(w, g.dtype, 1), cin_w, out_ld, grid, **kw)


def _wgrad(x, cin, g, cout, grid, gw, gb, rows):
    dwp = torch.zeros((27, K.pad32(cout), K.pad32(cin)), dtype=torch.float32, device=x.device)
    K.conv3d_wgrad(x, cin, 0, g, cout, grid, dwp)
    K.conv_unpack_grad(dwp, gw, cout, cin)
    K.colsum(g, gb, rows=rows, C=cout, ld=g.shape[-1])


def resnet_forward(P, names, x, nblocks, pad):
    """x complex64 [B, E, T, Y, X] -> (out complex64, saved)."""
    B, E, T, Y, X = x.shape
    Tp = T + 2 * pad
    if Tp % 4 or Y % 4 or X % 4:
        raise NotImplementedError("dl_cs HIP path: T+2*pad, Y and X must be multiples of 4")
    grid = (B, Tp, Y, X)
    cin = 2 * E
    F = P[names["init_w"]].shape[0]
    u = K.swin_pre(x.contiguous(), torch.float32, pad, PAD_CIN)
    r = [_conv(u, cin, P[names["init_w"]], F, F, grid, bias=P[names["init_b"]], relu_out=1)]
    ts = []
    for k in range(nblocks):
        wa, ba, wb, bb = (P[n] for n in names["blocks"][k])
        t = _conv(r[-1], F, wa, F, F, grid, bias=ba, relu_out=1)
        ts.append(t)
        r.append(_conv(t, F, wb, F, F, grid, bias=bb, res=r[-1], relu_out=1))
    o = _conv(r[-1], F, P[names["final_w"]], cin, PAD_CIN, grid, bias=P[names["final_b"]], res=u,
              out_dtype=torch.float32)
    out = K.swin_post(o, (B, E, T, Y, X), pad)
    from . import engine
    if engine.CAPTURE is not None:                   # test hook: ReLU decisions in the oracle's call order
        order = [t for k in range(nblocks) for t in (r[k], ts[k])] + [r[-1]]
        engine.CAPTURE.append(dict(relu_inputs=order, grid=grid, C=F))
    return out, dict(u=u, r=r, ts=ts, grid=grid, cin=cin, F=F, shape=(B, E, T, Y, X), pad=pad)


def resnet_backward(P, names, sv, gout, grads):
    grid, cin, F, pad = sv["grid"], sv["cin"], sv["F"], sv["pad"]
    rows = grid[0] * grid[1] * grid[2] * grid[3]
    r, ts, u = sv["r"], sv["ts"], sv["u"]
    go = K.swin_post_bwd(gout.contiguous(), torch.float32, pad, PAD_CIN)           # dL/d out (and the + u path)
    # final layer: out = conv_f(r_L) + b_f + u
    _wgrad(r[-1], F, go, cin, grid, grads[names["final_w"]], grads[names["final_b"]], rows)
    g = _dgrad(go, cin, P[names["final_w"]], F, F, grid, mask=r[-1])                # dL/d o_L (through relu)
    for k in reversed(range(len(ts))):
        wa, ba, wb, bb = (P[n] for n in names["blocks"][k])
        gwa, gba, gwb, gbb = (grads[n] for n in names["blocks"][k])
        # o_{k+1} = conv_b(t_k) + b_b + r_k ;  t_k = relu(conv_a(r_k) + b_a)
        _wgrad(ts[k], F, g, F, grid, gwb, gbb, rows)
        gt = _dgrad(g, F, wb, F, F, grid, mask=ts[k])
        _wgrad(r[k], F, gt, F, grid, gwa, gba, rows)
        gr = _dgrad(gt, F, wa, F, F, grid, res=g)                                  # dL/d r_k (conv + residual)
        g = K.relu_grad(gr, r[k])                                                  # dL/d o_k
    # init layer: o_0 = conv0(u) + b0 ;  du = conv0^T(g) + go (the final residual)
    _wgrad(u, cin, g, F, grid, grads[names["init_w"]], grads[names["init_b"]], rows)
    du = _dgrad(g, F, P[names["init_w"]], cin, PAD_CIN, grid, res=go, out_dtype=torch.float32)
    return K.swin_pre_bwd(du, sv["shape"], pad)


class _ResNetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, meta, *plist):
        P = dict(zip(meta["order"], plist))
        out, sv = resnet_forward(P, meta["names"], x.to(torch.complex64), meta["nblocks"], meta["pad"])
        ctx.state = (P, sv, meta)
        return out

    @staticmethod
    def backward(ctx, gout):
        P, sv, meta = ctx.state
        grads = {n: torch.zeros_like(p) for n, p in P.items()}
        gx = resnet_backward(P, meta["names"], sv, gout.to(torch.complex64), grads)
        ctx.state = None
        return (gx, None) + tuple(grads[n] for n in meta["order"])


class ResNet(nn.Module):
    """r3d:243-317 -- init ConvBlock (no activation), num_resblocks ResBlocks,
    final pre-activation ConvBlock back to in_chans, plus the input residual."""

    def __init__(self, num_resblocks, in_chans, chans, kernel_size, act_type='relu', use_complex_layers=False,
                 circular_pad=True):
        super().__init__()
        if use_complex_layers:
            raise NotImplementedError("dl_cs HIP ResNet: COMPLEX: False (configs/example.yaml)")
        if kernel_size != 3 or act_type != 'relu' or not circular_pad:
            raise NotImplementedError("dl_cs HIP ResNet: kernel 3, relu, circular pad (configs/example.yaml)")
        self.use_complex_layers = use_complex_layers
        self.circular_pad = circular_pad
        self.pad_size = (2 * num_resblocks + 2) * (kernel_size - 1) // 2                  # r3d:253
        self.init_layer = ConvBlock(in_chans, chans, kernel_size, act_type='none')
        self.res_blocks = nn.ModuleList([ResBlock(chans, kernel_size, act_type=act_type)
                                         for _ in range(num_resblocks)])
        self.final_layer = ConvBlock(chans, in_chans, kernel_size, act_type=act_type)

    def _names(self):
        c = lambda pre: (f"{pre}.layers.2.conv.weight", f"{pre}.layers.2.conv.bias")
        blocks = []
        for k in range(len(self.res_blocks)):
            blocks.append(c(f"res_blocks.{k}.layers.0") + c(f"res_blocks.{k}.layers.1"))
        iw, ib = c("init_layer")
        fw, fb = c("final_layer")
        return dict(init_w=iw, init_b=ib, final_w=fw, final_b=fb, blocks=blocks)

    def forward(self, input):
        if get_compute_dtype() != torch.float32:
            raise NotImplementedError("dl_cs HIP ResNet: fp32 (the generic conv kernels; no bf16 wgrad at 64 ch)")
        if not input.is_cuda:
            raise RuntimeError("dl_cs HIP ResNet needs GPU tensors (no CPU fallback in the product path)")
        params = dict(self.named_parameters())
        order = list(params.keys())
        meta = dict(order=order, names=self._names(), nblocks=len(self.res_blocks), pad=self.pad_size)
        return _ResNetFn.apply(input, meta, *[params[n] for n in order])
