"""Swin regularizer R_i of the unrolled reconstruction, MI355X build.

Mirrors the reference module tree (s3d = dl_cs/models/swin3D.py) so the
state_dict keys -- including the DFE.layers / DFE.resswin_blocks aliases
(s3d:350-357) -- are identical, but SwinTransformer3DNet.forward runs the
whole regularizer (SFE conv -> Swin -> ResSwin conv -> DFE conv -> final conv,
s3d:420-435) as ONE autograd node whose forward and hand-scheduled backward
are HIP kernels (dl_cs.models.engine).
"""
import os
import weakref

import torch
from torch import nn

from . import engine
from .video_swin_transformer_mri_downsample import SwinTransformer3D
from .. import _lib

_COMPUTE_DTYPE = {"bf16": torch.bfloat16, "fp32": torch.float32}.get(
    os.environ.get("DLCS_COMPUTE_DTYPE", "fp32"), torch.float32)


def set_compute_dtype(dtype):
    """Storage dtype of activations / GEMM operands (fp32 accumulation always):
    torch.float32 (parity build) or torch.bfloat16 (fast path)."""
    global _COMPUTE_DTYPE
    assert dtype in (torch.float32, torch.bfloat16)
    _COMPUTE_DTYPE = dtype


def get_compute_dtype():
    return _COMPUTE_DTYPE


# Direct gradient sink (set by dl_cs.distributed.GradBuckets): when on and every
# parameter of a SwinTransformer3DNet already has an fp32 .grad, the fused
# backward accumulates straight into those .grad buffers and returns None for
# the parameters -- no per-parameter zero-filled gradient tensors and no
# AccumulateGrad adds.  GRAD_READY callbacks then get the module once its
# gradients are complete (the all-reduce trigger).  Off by default, so
# torch.autograd.grad() and other functional uses see ordinary gradients.
DIRECT_GRADS = False
GRAD_READY = []


class Normalization(nn.Module):
    """s3d:16-36 (only 'none' is on the Swin path: config_swin NORM: none)."""

    def __init__(self, in_chans, type):
        super().__init__()
        if type == 'none':
            self.norm = nn.Identity()
        elif type == 'instance':
            self.norm = nn.InstanceNorm3d(in_chans, affine=False)
        elif type == 'batch':
            self.norm = nn.BatchNorm3d(in_chans, affine=False)
        else:
            raise ValueError('Invalid normalization type: %s' % type)

    def forward(self, input):
        return self.norm(input)


class Activation(nn.Module):
    """s3d:39-61."""

    def __init__(self, type):
        super().__init__()
        self.type = type
        if type == 'none':
            self.activ = nn.Identity()
        elif type == 'relu':
            self.activ = nn.ReLU(inplace=True)
        elif type == 'leaky_relu':
            self.activ = nn.LeakyReLU(inplace=True)
        elif type == 'sigmoid':
            self.activ = nn.Sigmoid()
        else:
            raise ValueError('Invalid activation type: %s' % type)

    def forward(self, input):
        return self.activ(input)


class Conv3d(nn.Module):
    """s3d:120-134 -- nn.Conv3d with 'same' padding; forward is dlcs_conv3d_k3
    (standalone module path, _standalone.ConvBlockFn)."""

    def __init__(self, in_chans, out_chans, kernel_size):
        super().__init__()
        padding = (kernel_size - 1) // 2
        self.conv = nn.Conv3d(in_chans, out_chans, kernel_size, padding=padding)

    def forward(self, input):
        from ._standalone import conv_block
        return conv_block(input, self.conv, relu=False)


class ConvBlock(nn.Module):
    """s3d:225-273 -- Norm -> Act -> Conv3d (pre-activation)."""

    def __init__(self, in_chans, out_chans, kernel_size, act_type='relu', norm_type='none', is_complex=False):
        super().__init__()
        if is_complex:
            raise NotImplementedError("ComplexConv3d is not on the config_swin path (COMPLEX: False)")
        self.in_chans = in_chans
        self.out_chans = out_chans
        self.is_complex = is_complex
        self.name = 'Conv3D'
        self.act_type = act_type
        self.layers = nn.Sequential(Normalization(in_chans, norm_type), Activation(act_type),
                                    Conv3d(in_chans, out_chans, kernel_size=kernel_size))

    def forward(self, input):
        """Norm (Identity) -> ReLU / none -> Conv3d k3 in one HIP autograd node
        (the ReLU is the conv's prologue; its backward the dgrad's mask)."""
        from ._standalone import conv_block
        norm, act = self.layers[0].norm, self.layers[1].type
        if not isinstance(norm, nn.Identity) or act not in ('relu', 'none'):
            raise NotImplementedError("HIP ConvBlock: norm 'none', activation relu / none (config_swin)")
        return conv_block(input, self.layers[2].conv, relu=(act == 'relu'))

    def __repr__(self):
        return f'{self.name}(in_chans={self.in_chans}, out_chans={self.out_chans})'


class SwinTransformer3DBlock(nn.Module):
    """s3d:304-325 -- hard-coded SwinTransformer3D(depths=[6], heads=[8], window (7,8,8))."""

    def __init__(self, in_chans, chans, window_size, num_heads, num_layers, is_complex=False):
        super().__init__()
        self.is_complex = is_complex
        self.transformer = SwinTransformer3D(in_chans=in_chans, embed_dim=chans, depths=[6], num_heads=[8],
                                             window_size=(7, 8, 8))

    def forward(self, input):
        return self.transformer(input)


class ResSwinTransformer3DBlock(nn.Module):
    """s3d:327-340 -- Swin -> ConvBlock, + input."""

    def __init__(self, in_chans, chans, window_size, num_heads, num_layers, act_type='relu', is_complex=False):
        super().__init__()
        self.layers = nn.Sequential(
            SwinTransformer3DBlock(in_chans, chans, window_size, num_heads, num_layers, is_complex=is_complex),
            ConvBlock(chans, chans, kernel_size=3, act_type=act_type, is_complex=is_complex))

    def forward(self, input):
        return self.layers(input) + input                                    # s3d:339-340


class DeepFeatureExtraction(nn.Module):
    """s3d:342-368 -- the ResSwin blocks are registered twice (resswin_blocks and
    layers), exactly as in the reference, so checkpoints load unchanged."""

    def __init__(self, in_chans, chans, window_size, num_heads, num_layers, num_swinblocks, act_type='relu',
                 is_complex=False):
        super().__init__()
        self.resswin_blocks = nn.ModuleList([])
        for _ in range(num_swinblocks):
            self.resswin_blocks += [ResSwinTransformer3DBlock(in_chans, chans, window_size, num_heads, num_layers,
                                                              act_type=act_type, is_complex=is_complex)]
        self.layers = nn.Sequential(*self.resswin_blocks,
                                    ConvBlock(chans, chans, kernel_size=3, act_type=act_type, is_complex=is_complex))

    def forward(self, input):
        return self.layers(input) + input                                    # s3d:368


class SwinTransformer3DNet(nn.Module):
    """s3d:371-435 -- SwinMR regularizer; forward runs on libdlcs_hip."""

    def __init__(self, num_swinblocks, in_chans, chans, kernel_size, window_size, act_type='relu', num_heads=[4],
                 num_layers=[4], use_complex_layers=False, circular_pad=True):
        super().__init__()
        if use_complex_layers:
            # The reference builds this net (s3d:378-387) but cannot run it: the complex
            # tensor reaches SwinTransformer3D's real nn.Conv3d patch embedding (vst:440-479),
            # where torch raises "Input type (c10::complex<float>) and bias type (float)
            # should be the same".  config_swin sets COMPLEX: False.
            raise NotImplementedError("use_complex_layers=True: the reference's forward fails at PatchEmbed3D "
                                      "(real Conv3d on a complex tensor); config_swin uses COMPLEX: False")
        if kernel_size != 3 or act_type != 'relu' or not circular_pad or num_swinblocks < 1:
            raise NotImplementedError("HIP path: kernel_size=3, NUM_SWINBLOCKS >= 1, relu, circular_pad")
        self.use_complex_layers = use_complex_layers
        self.circular_pad = circular_pad
        self.pad_size = (2 * num_swinblocks + 2) * (kernel_size - 1) // 2                # s3d:380
        self.SFE = ConvBlock(in_chans, chans, kernel_size=3, act_type='none', is_complex=use_complex_layers)
        self.DFE = DeepFeatureExtraction(chans, chans, window_size, num_heads, num_layers, num_swinblocks,
                                         act_type=act_type, is_complex=use_complex_layers)
        self.final_layer = ConvBlock(chans, in_chans, kernel_size=3, act_type=act_type, is_complex=use_complex_layers)

    # engine short name -> parameter; ResSwin block k's parameters carry the prefix
    # "rs<k>." (swin_tail = its ConvBlock, s3d:336; the SwinTransformer3D's patch
    # embed / unembed and blocks); dfe_tail = the DFE's closing ConvBlock (s3d:356)
    def engine_params(self):
        P = {
            "SFE.layers.2.conv.weight": self.SFE.layers[2].conv.weight,
            "SFE.layers.2.conv.bias": self.SFE.layers[2].conv.bias,
            "dfe_tail.weight": self.DFE.layers[-1].layers[2].conv.weight,
            "dfe_tail.bias": self.DFE.layers[-1].layers[2].conv.bias,
            "final_layer.layers.2.conv.weight": self.final_layer.layers[2].conv.weight,
            "final_layer.layers.2.conv.bias": self.final_layer.layers[2].conv.bias,
        }
        for k, rs in enumerate(self.DFE.resswin_blocks):
            tr = rs.layers[0].transformer
            pre = f"rs{k}."
            P.update({
                pre + "swin_tail.weight": rs.layers[1].layers[2].conv.weight,
                pre + "swin_tail.bias": rs.layers[1].layers[2].conv.bias,
                pre + "patch_embed.proj.weight": tr.patch_embed.proj.weight,
                pre + "patch_embed.proj.bias": tr.patch_embed.proj.bias,
                pre + "patch_unembed.proj.weight": tr.patch_unembed.proj.weight,
                pre + "patch_unembed.proj.bias": tr.patch_unembed.proj.bias,
            })
            for i, blk in enumerate(tr.layers[0].blocks):
                for n, p in blk.named_parameters():
                    if n in engine.BlockWeights.NAMES:
                        P[f"{pre}blocks.{i}.{n}"] = p
        return P

    def _transformers(self):
        return [rs.layers[0].transformer for rs in self.DFE.resswin_blocks]

    def _has_drop_path(self):
        from .video_swin_transformer_mri_downsample import DropPath
        return any(isinstance(b.drop_path, DropPath) and b.drop_path.drop_prob > 0
                   for tr in self._transformers() for b in tr.layers[0].blocks)

    def _forward_modules(self, x):
        """s3d:394-435 module by module (every compute step a HIP autograd node):
        the path for T + 2 pad, Y or X not multiples of 4, which the fused
        path's patch-blocked tiling needs."""
        import torch.nn.functional as F
        p = self.pad_size
        u = torch.cat((x.real, x.imag), dim=1)                               # s3d:399
        u = F.pad(u, (0, 0, 0, 0, p, p), mode='circular')                    # s3d:402-404
        s = self.SFE(u)
        h = s + self.DFE(s)                                                  # s3d:425-427
        o = self.final_layer(h)[:, :, p:u.shape[2] - p]                      # s3d:408-410
        E = o.shape[1] // 2
        return torch.complex(o[:, :E].contiguous(), o[:, E:].contiguous())   # s3d:412-416

    def forward(self, x):
        """x: complex64 [B, E, T, Y, X] on the GPU -> complex64 [B, E, T, Y, X]."""
        assert torch.is_complex(x)
        _lib.require_gpu(x)
        if (x.shape[2] + 2 * self.pad_size) % 4 or x.shape[3] % 4 or x.shape[4] % 4:
            return self._forward_modules(x)
        if self.training and x.shape[0] > 1 and self._has_drop_path():
            # timm DropPath draws per sample: one fused pass per sample, each with its own draws
            return torch.cat([self.forward(x[i:i + 1]) for i in range(x.shape[0])], dim=0)
        P = self.engine_params()
        names = list(P.keys())
        trs = self._transformers()
        tr = trs[0]
        drop = [[blk.drop_scales() for blk in t.layers[0].blocks] for t in trs] if self.training else None
        meta = dict(names=names, heads=tr.num_heads[0], window=tuple(tr.window_size), pad=self.pad_size,
                    depth=len(tr.layers[0].blocks), nstages=len(trs), drop=drop, dtype=get_compute_dtype(),
                    module=self)
        return _SwinNetFn.apply(x, meta, *[P[n] for n in names])


_W_CACHE = weakref.WeakKeyDictionary()   # module -> [(key, engine.NetWeights)], one per compute dtype


def clear_weight_cache(module=None):
    """Drop the packed weights kept between calls (of `module`, or of every network) and
    the weight norms their plane bounds are derived from (engine._CONV_NORMS).  Needed
    only after changing a parameter through ``.data``, which bypasses the version
    counter both caches check."""
    if module is None:
        _W_CACHE.clear()
    else:
        _W_CACHE.pop(module, None)
    engine.clear_norm_cache()


def _net_weights(params, meta):
    """engine.NetWeights of this parameter set, reused while no parameter has changed: the
    unrolls of one training step (and every eval call between optimizer steps) share one
    packing of the weights.  Keyed by each parameter's identity, storage and in-place
    version counter (an optimizer step, load_state_dict or any in-place update bumps it).
    The cache lives on the module (a weak key: it dies with the network) and holds one
    packing per compute dtype -- a stale packing of the same dtype is dropped as soon as
    its replacement is built (a backward still in flight keeps its own reference)."""
    key = (meta["dtype"], meta["depth"], meta["nstages"],
           tuple((id(p), p.data_ptr(), p._version) for p in params.values()))
    lst = _W_CACHE.setdefault(meta["module"], [])
    for k, W in lst:
        if k == key:
            return W
    W = engine.NetWeights(params, meta["dtype"], meta["depth"], meta["nstages"])
    lst[:] = [(k, w) for k, w in lst if k[0] != key[0]]
    lst.insert(0, (key, W))
    return W


class _SwinNetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, meta, *plist):
        params = dict(zip(meta["names"], plist))
        W = _net_weights(params, meta)
        out, sv = engine.swinnet_forward(W, x.to(torch.complex64), heads=meta["heads"], window=meta["window"],
                                         pad=meta["pad"], drop_scales=meta["drop"])
        ctx.state = (W, sv, meta)
        return out

    @staticmethod
    def backward(ctx, gout):
        W, sv, meta = ctx.state
        dev = gout.device
        C = W.p["SFE.layers.2.conv.bias"].shape[0]
        direct = DIRECT_GRADS and all(
            p.grad is not None and p.grad.dtype == torch.float32 and p.grad.is_contiguous() and
            p.grad.shape == p.shape for p in W.p.values())
        if DIRECT_GRADS and GRAD_READY and not direct:
            raise RuntimeError("dl_cs: GradBuckets is active but a parameter's .grad no longer points into its "
                               "bucket (optimizer.zero_grad(set_to_none=True)?); call GradBuckets.zero() "
                               "before each backward instead")
        if direct:
            grads = {n: p.grad for n, p in W.p.items()}
        else:
            grads = {n: torch.zeros_like(p) for n, p in W.p.items()}
        for k in range(meta["nstages"]):
            grads[f"rs{k}.emb_packed"] = torch.zeros((C, 64 * C), dtype=torch.float32, device=dev)
            grads[f"rs{k}.unemb_packed"] = torch.zeros((64 * C, C), dtype=torch.float32, device=dev)
        gx = engine.swinnet_backward(W, sv, gout.to(torch.complex64), grads)
        engine.unpack_patch_grads(grads, C, meta["nstages"])
        ctx.state = None
        if direct:
            for cb in GRAD_READY:
                cb(meta["module"])
            return (gx, None) + (None,) * len(meta["names"])
        return (gx, None) + tuple(grads[n] for n in meta["names"])
