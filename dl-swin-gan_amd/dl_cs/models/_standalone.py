"""Module-at-a-time HIP path: the reference's per-module forwards (s3d ConvBlock /
Conv3d, vst PatchEmbed3D / PatchUnembed3D / SwinTransformer3D) callable on
their own, each a torch.autograd.Function over the same kernels the fused
SwinTransformer3DNet path uses (conv3d_k3 fwd / dgrad / wgrad, the patch GEMMs,
colsum), with NCDHW tensors converted to and from the patch-blocked layout by
dlcs_block_layout.

Any spatial size works: the blocked grid is zero-padded to multiples of 4,
which is exact for the k3 / pad 1 convolution (the padded voxels are the
convolution's own zero padding, and their output gradients are zero), and is
exactly PatchEmbed3D's end padding (vst:464-470).  This is also the path
SwinTransformer3DNet takes for sizes the fused path does not tile.
"""
import math

import torch

from .. import _lib
from . import _ops as K


def _pad4(n):
    return (n + 3) // 4 * 4


def _pad8(n):
    return (n + 7) // 8 * 8


def to_blocked(x, ld, dtype):
    """[B, C, D, H, W] -> blocked rows [B * nT * nY * nX * 64, ld] (zero padded)."""
    B, C, D, H, W = x.shape
    x = x.contiguous()
    rows = B * (_pad4(D) // 4) * (_pad4(H) // 4) * (_pad4(W) // 4) * 64
    out = torch.empty((rows, ld), dtype=dtype, device=x.device)
    _lib.call("dlcs_block_layout", K.code(x), K.code(out), _lib.ptr(x), _lib.ptr(out), B, C, D, H, W, ld, 0,
              _lib.stream())
    return out


def from_blocked(rows, shape, dtype=torch.float32):
    """blocked rows [.., ld] -> [B, C, D, H, W] (cropped to the shape)."""
    B, C, D, H, W = shape
    out = torch.empty(shape, dtype=dtype, device=rows.device)
    _lib.call("dlcs_block_layout", K.code(rows), K.code(out), _lib.ptr(rows), _lib.ptr(out), B, C, D, H, W,
              rows.shape[-1], 1, _lib.stream())
    return out


def _dtype():
    from .swin3D import get_compute_dtype
    return get_compute_dtype()


class ConvBlockFn(torch.autograd.Function):
    """(ReLU ->) Conv3d(k3, pad 1) + bias  (s3d:225-273 with Identity norm, s3d:120-134)."""

    @staticmethod
    def forward(ctx, x, w, b, relu):
        dtype = _dtype()
        B, Cin, D, H, W = x.shape
        Cout = w.shape[0]
        grid = (B, _pad4(D), _pad4(H), _pad4(W))
        cin_ld, out_ld = max(8, _pad8(Cin)), max(8, _pad8(Cout))
        u = to_blocked(x.float(), cin_ld, dtype)
        o = K.conv3d(u, Cin, K.conv_pack(w, dtype, 0), Cout, out_ld, grid, bias=b, relu_in=int(relu),
                     out_dtype=torch.float32)
        ctx.save_for_backward(u, w)
        ctx.meta = (relu, x.shape, grid, cin_ld, out_ld, dtype)
        return from_blocked(o, (B, Cout, D, H, W))

    @staticmethod
    def backward(ctx, gy):
        u, w = ctx.saved_tensors
        relu, shp, grid, cin_ld, out_ld, dtype = ctx.meta
        B, Cin, D, H, W = shp
        Cout = w.shape[0]
        g = to_blocked(gy.float(), out_ld, dtype)
        dx = K.conv3d(g, Cout, K.conv_pack(w, dtype, 1), Cin, cin_ld, grid, mask=u if relu else None,
                      out_dtype=torch.float32)
        dwp = torch.zeros((27, K.pad32(Cout), K.pad32(Cin)), dtype=torch.float32, device=gy.device)
        K.conv3d_wgrad(u, Cin, int(relu), g, Cout, grid, dwp)
        gw = torch.zeros_like(w)
        K.conv_unpack_grad(dwp, gw, Cout, Cin)
        gb = torch.zeros((Cout,), dtype=torch.float32, device=gy.device)
        K.colsum(g, gb, rows=g.shape[0], C=Cout, ld=out_ld)
        return from_blocked(dx, shp), gw, gb, None


def conv_block(x, conv, relu):
    """nn.Conv3d(k3, pad 1) parameters `conv` applied to real x [B, C, D, H, W] on the GPU."""
    _lib.require_gpu(x)
    if conv.kernel_size != (3, 3, 3) or conv.padding != (1, 1, 1) or conv.stride != (1, 1, 1):
        raise NotImplementedError("HIP conv3d: kernel 3, padding 1, stride 1 (s3d:120-134)")
    b = conv.bias if conv.bias is not None else torch.zeros(conv.out_channels, device=x.device)
    return ConvBlockFn.apply(x, conv.weight, b, bool(relu))


class PatchEmbedFn(torch.autograd.Function):
    """Conv3d(k4, s4) of [B, C, D, H, W] (end-padded to multiples of 4) -> [B, E, nT, nY, nX]
    as one GEMM on the blocked rows (vst:460-479)."""

    @staticmethod
    def forward(ctx, x, w, b):
        dtype = _dtype()
        B, C, D, H, W = x.shape
        E = w.shape[0]
        nT, nY, nX = _pad4(D) // 4, _pad4(H) // 4, _pad4(W) // 4
        ntok = B * nT * nY * nX
        u = to_blocked(x.float(), C, dtype).view(ntok, 64 * C)
        emb = K.permute(w, (E, 4, 4, 4, C), (C * 64, 16, 4, 1, 64), dst_dtype=dtype)    # [e][(kd,kh,kw,c)]
        tok = torch.empty((ntok, E), dtype=torch.float32, device=x.device)
        K.gemm(u, emb, tok, ntok, E, 64 * C, 64 * C, 64 * C, E, bias=b)
        ctx.save_for_backward(u, emb)
        ctx.meta = (x.shape, (B, nT, nY, nX), w.shape, dtype)
        return K.permute(tok, (B, E, nT, nY, nX), (nT * nY * nX * E, 1, nY * nX * E, nX * E, E))

    @staticmethod
    def backward(ctx, gy):
        u, emb = ctx.saved_tensors
        shp, (B, nT, nY, nX), wshape, dtype = ctx.meta
        E, C = wshape[0], wshape[1]
        ntok = B * nT * nY * nX
        g = K.permute(gy.float().contiguous(), (B, nT, nY, nX, E),
                      (E * nT * nY * nX, nY * nX, nX, 1, nT * nY * nX), dst_dtype=dtype).view(ntok, E)
        du = torch.empty((ntok, 64 * C), dtype=torch.float32, device=gy.device)
        K.gemm(g, emb, du, ntok, 64 * C, E, E, 64 * C, 64 * C, b_trans=1)
        gx = from_blocked(du.view(ntok * 64, C), shp)
        dwp = torch.zeros((E, 64 * C), dtype=torch.float32, device=gy.device)
        K.gemm(g, u, dwp, E, 64 * C, ntok, E, 64 * C, 64 * C, a_trans=1, b_trans=1, accumulate=1,
               splitk=max(1, min(16, ntok // 256)))
        gw = torch.zeros(wshape, dtype=torch.float32, device=gy.device)
        K.permute(dwp, (E, C, 4, 4, 4), (64 * C, 1, 16 * C, 4 * C, C), out=gw, accumulate=1)
        gb = torch.zeros((E,), dtype=torch.float32, device=gy.device)
        K.colsum(g, gb)
        return gx, gw, gb


class PatchUnembedFn(torch.autograd.Function):
    """ConvTranspose3d(k4, s4) [B, E, nT, nY, nX] -> [B, C, 4nT, 4nY, 4nX] as one GEMM
    writing blocked rows (vst:503-508); the crop to pre_size is the caller's."""

    @staticmethod
    def forward(ctx, x, w, b):
        dtype = _dtype()
        B, E, nT, nY, nX = x.shape
        C = w.shape[1]
        ntok = B * nT * nY * nX
        tok = K.permute(x.float().contiguous(), (B, nT, nY, nX, E),
                        (E * nT * nY * nX, nY * nX, nX, 1, nT * nY * nX), dst_dtype=dtype).view(ntok, E)
        unemb = K.permute(w, (4, 4, 4, C, E), (16, 4, 1, 64, C * 64), dst_dtype=dtype)   # [(kd,kh,kw,c)][e]
        bias = K.fill_bias(torch.empty((64 * C,), dtype=torch.float32, device=x.device), b, 1, 64 * C, C)
        full = torch.empty((ntok, 64 * C), dtype=torch.float32, device=x.device)
        K.gemm(tok, unemb, full, ntok, 64 * C, E, E, E, 64 * C, bias=bias)
        ctx.save_for_backward(tok, unemb)
        ctx.meta = (x.shape, C, dtype)
        return from_blocked(full.view(ntok * 64, C), (B, C, 4 * nT, 4 * nY, 4 * nX))

    @staticmethod
    def backward(ctx, gy):
        tok, unemb = ctx.saved_tensors
        (B, E, nT, nY, nX), C, dtype = ctx.meta
        ntok = B * nT * nY * nX
        g = to_blocked(gy.float(), C, dtype).view(ntok, 64 * C)
        dt = torch.empty((ntok, E), dtype=torch.float32, device=gy.device)
        K.gemm(g, unemb, dt, ntok, E, 64 * C, 64 * C, E, E, b_trans=1)
        gx = K.permute(dt, (B, E, nT, nY, nX), (nT * nY * nX * E, 1, nY * nX * E, nX * E, E))
        dwp = torch.zeros((64 * C, E), dtype=torch.float32, device=gy.device)
        K.gemm(g, tok, dwp, 64 * C, E, ntok, 64 * C, E, E, a_trans=1, b_trans=1, accumulate=1,
               splitk=max(1, min(16, ntok // 256)))
        gw = torch.zeros((E, C, 4, 4, 4), dtype=torch.float32, device=gy.device)
        K.permute(dwp, (E, C, 4, 4, 4), (1, E, 16 * C * E, 4 * C * E, C * E), out=gw, accumulate=1)
        gb = torch.zeros((C,), dtype=torch.float32, device=gy.device)
        K.colsum(g.view(ntok * 64, C), gb)
        return gx, gw, gb


def center_crop_like_reference(x, pre_size):
    """vst:517-524 -- crop ceil(diff/2) from the start and floor(diff/2) from the end."""
    cs = x.shape
    diff = [cs[j] - pre_size[j] for j in range(5)]
    return x[:, :, math.ceil(diff[2] / 2):cs[2] - math.floor(diff[2] / 2),
             math.ceil(diff[3] / 2):cs[3] - math.floor(diff[3] / 2),
             math.ceil(diff[4] / 2):cs[4] - math.floor(diff[4] / 2)]
