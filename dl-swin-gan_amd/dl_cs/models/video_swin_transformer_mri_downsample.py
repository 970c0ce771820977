"""Video-Swin backbone of the regularizer, MI355X build.

Same public names, constructor arguments and state_dict schema as the
reference module (vst = dl_cs/models/video_swin_transformer_mri_downsample.py);
the arithmetic runs in libdlcs_hip:

* window_partition / window_reverse / cyclic shift -> dlcs_window_index tables
  + dlcs_gather_rows (and, inside the fused path, the LayerNorm gather and the
  proj-GEMM scatter epilogue);
* WindowAttention3D -> dlcs_gemm (qkv, proj) + dlcs_window_attn_fwd/_bwd;
* Mlp -> dlcs_gemm with fused bias + GELU(erf) epilogues;
* SwinTransformerBlock3D / BasicLayer -> engine.block_forward / block_backward.

The full SwinTransformer3D (patch embed -> 6 blocks -> unembed) is executed as
part of SwinTransformer3DNet's fused forward (dl_cs.models.swin3D).
"""
import math
from typing import Callable, List, Optional

import torch
from torch import nn

from . import _ops as K
from . import engine
from ._window import get_window_size  # noqa: F401  (vst:72-85, re-exported)
from .. import _lib


def _trunc_normal_(t, std=0.02, a=-2.0, b=2.0):
    """timm trunc_normal_ (vst:11, :136): N(0, std) truncated to [a, b]."""
    with torch.no_grad():
        nn.init.trunc_normal_(t, mean=0.0, std=std, a=a, b=b)
    return t


class DropPath(nn.Module):
    """Stochastic depth (timm DropPath, vst:210): identity in eval mode, else an
    independent keep decision per sample (timm's mask shape [B, 1, ...]) with
    survivors scaled by 1/keep.  The fused path draws one sample's decision on
    the host and folds it into the GEMM epilogue's alpha (see drop_scales);
    SwinTransformer3DNet runs a batch > 1 one sample at a time in training so
    every sample gets its own draw."""

    def __init__(self, drop_prob=0.0):
        super().__init__()
        self.drop_prob = drop_prob

    def sample_scale(self):
        """One sample's factor: 0 (dropped) or 1/keep."""
        if not self.training or self.drop_prob == 0.0:
            return 1.0
        keep = 1.0 - self.drop_prob
        return (1.0 / keep) if torch.rand(()).item() < keep else 0.0

    def forward(self, x):
        if not self.training or self.drop_prob == 0.0:
            return x
        keep = 1.0 - self.drop_prob
        shape = (x.shape[0],) + (1,) * (x.ndim - 1)
        mask = (torch.rand(shape, device=x.device) < keep).to(x.dtype)
        return x * mask / keep


class Mlp(nn.Module):
    """vst:20-38 -- fc2(drop(GELU(fc1 x)))."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)

    def forward(self, x):
        _lib.require_gpu(x)
        return _MlpFn.apply(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias)


class _MlpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        shp = x.shape
        xf = x.reshape(-1, shp[-1]).float().contiguous()
        h = K.empty((xf.shape[0], w1.shape[0]), torch.float32, x.device)
        a = K.linear(xf, w1, b1, act=1, aux_out=h)
        y = K.linear(a, w2, b2)
        ctx.save_for_backward(xf, h, a, w1, w2)
        ctx.shp = shp
        return y.reshape(*shp[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, gy):
        xf, h, a, w1, w2 = ctx.saved_tensors
        g = gy.reshape(-1, gy.shape[-1]).float().contiguous()
        dw1, db1 = torch.zeros_like(w1), torch.zeros(w1.shape[0], device=g.device)
        dw2, db2 = torch.zeros_like(w2), torch.zeros(w2.shape[0], device=g.device)
        dh = K.linear_dx(g, w2, act=2, aux=h)
        K.linear_dw(g, a, dw2)
        K.colsum(g, db2)
        dx = K.linear_dx(dh, w1)
        K.linear_dw(dh, xf, dw1)
        K.colsum(dh, db1)
        return dx.reshape(ctx.shp), dw1, db1, dw2, db2


def _window_perm(B, D, H, W, window_size, device):
    ws = tuple(window_size)
    part, rev, _, nrows = K.window_tables(B, D, H, W, ws, (0, 0, 0), device, False)
    return part, rev, nrows


class _GatherFn(torch.autograd.Function):
    """Row permutation y[r] = x[idx[r]] (idx < 0 -> 0); backward scatters with inv."""

    @staticmethod
    def forward(ctx, x, idx, inv, nrows):
        ctx.save_for_backward(idx, inv)
        ctx.nin = x.shape[0]
        return K.gather_rows(x.contiguous(), idx, nrows, x.dtype)

    @staticmethod
    def backward(ctx, g):
        idx, inv = ctx.saved_tensors
        return K.gather_rows(g.contiguous(), inv, ctx.nin, g.dtype), None, None, None


def window_partition(x, window_size):
    """vst:41-52 -- (B, D, H, W, C) -> (B*num_windows, Wd*Wh*Ww, C)."""
    _lib.require_gpu(x)
    B, D, H, W, C = x.shape
    part, rev, nrows = _window_perm(B, D, H, W, window_size, x.device)
    y = _GatherFn.apply(x.reshape(-1, C), part, rev, nrows)
    N = window_size[0] * window_size[1] * window_size[2]
    return y.view(-1, N, C)


def window_reverse(windows, window_size, B, D, H, W):
    """vst:55-67 -- (B*num_windows, Wd, Wh, Ww, C) -> (B, D, H, W, C)."""
    _lib.require_gpu(windows)
    C = windows.shape[-1]
    part, rev, nrows = _window_perm(B, D, H, W, window_size, windows.device)
    y = _GatherFn.apply(windows.reshape(-1, C), rev, part, B * D * H * W)
    return y.view(B, D, H, W, C)


def compute_mask(D, H, W, window_size, shift_size, device):
    """vst:342-355 -- additive shift mask [nW, N, N] in {0, -100}.  Region labels
    come from the dlcs_window_index kernel; the fused path consumes the labels
    directly and never builds this tensor."""
    ws, ss = tuple(window_size), tuple(shift_size)
    _, _, lab, nrows = K.window_tables(1, D, H, W, ws, ss, torch.device(device), True)
    N = ws[0] * ws[1] * ws[2]
    lab = lab.view(nrows // N, N)
    return (lab.unsqueeze(1) != lab.unsqueeze(2)).float() * -100.0


def _relative_position_index(window_size):
    """vst:114-129 (integer, identical construction order)."""
    wd, wh, ww = window_size
    coords = torch.stack(torch.meshgrid(torch.arange(wd), torch.arange(wh), torch.arange(ww), indexing="ij"))
    cf = torch.flatten(coords, 1)
    rel = (cf[:, :, None] - cf[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += wd - 1
    rel[:, :, 1] += wh - 1
    rel[:, :, 2] += ww - 1
    rel[:, :, 0] *= (2 * wh - 1) * (2 * ww - 1)
    rel[:, :, 1] *= (2 * ww - 1)
    return rel.sum(-1)


class WindowAttention3D(nn.Module):
    """vst:88-170 -- window MSA with relative position bias (dlcs_window_attn_*)."""

    def __init__(self, dim, window_size, num_heads, qkv_bias=False, qk_scale=None, attn_drop=0., proj_drop=0.):
        super().__init__()
        self.dim = dim
        self.window_size = window_size
        self.num_heads = num_heads
        head_dim = dim // num_heads
        self.scale = qk_scale or head_dim ** -0.5
        self.relative_position_bias_table = nn.Parameter(
            torch.zeros((2 * window_size[0] - 1) * (2 * window_size[1] - 1) * (2 * window_size[2] - 1), num_heads))
        self.register_buffer("relative_position_index", _relative_position_index(window_size))
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        _trunc_normal_(self.relative_position_bias_table, std=.02)
        self.softmax = nn.Softmax(dim=-1)

    def forward(self, x, mask=None):
        """x: (num_windows*B, N, C); mask: (nW, N, N) additive or None."""
        _lib.require_gpu(x)
        qkv_b = self.qkv.bias if self.qkv.bias is not None else torch.zeros(3 * self.dim, device=x.device)
        return _WindowAttnFn.apply(x, self.qkv.weight, qkv_b, self.proj.weight, self.proj.bias,
                                   self.relative_position_bias_table, mask, self)


class _WindowAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wqkv, bqkv, wproj, bproj, table, mask, mod):
        B_, N, C = x.shape
        heads = mod.num_heads
        hd = C // heads
        xf = x.reshape(-1, C).float().contiguous()
        qkv = K.linear(xf, wqkv, bqkv)
        m = mask.float().contiguous() if mask is not None else None
        att, lse = K.attn_fwd(qkv, table, None, B_, N, heads, hd, mod.window_size, mod.scale,
                              mask=m, mask_nw=(m.shape[0] if m is not None else 0))
        y = K.linear(att, wproj, bproj)
        ctx.save_for_backward(xf, qkv, att, lse, wqkv, wproj, table)
        ctx.m, ctx.meta = m, (B_, N, C, heads, hd, tuple(mod.window_size), mod.scale)
        return y.view(B_, N, C)

    @staticmethod
    def backward(ctx, gy):
        xf, qkv, att, lse, wqkv, wproj, table = ctx.saved_tensors
        B_, N, C, heads, hd, window, scale = ctx.meta
        g = gy.reshape(-1, C).float().contiguous()
        dwp, dbp = torch.zeros_like(wproj), torch.zeros(C, device=g.device)
        dwq, dbq = torch.zeros_like(wqkv), torch.zeros(3 * C, device=g.device)
        dtab = torch.zeros_like(table)
        datt = K.linear_dx(g, wproj)
        K.linear_dw(g, att, dwp)
        K.colsum(g, dbp)
        m = ctx.m
        dqkv = K.attn_bwd(qkv, att, datt, lse, table, None, dtab, B_, N, heads, hd, window, scale,
                          mask=m, mask_nw=(m.shape[0] if m is not None else 0))
        dx = K.linear_dx(dqkv, wqkv)
        K.linear_dw(dqkv, xf, dwq)
        K.colsum(dqkv, dbq)
        return dx.view(B_, N, C), dwq, dbq, dwp, dbp, dtab, None, None


class SwinTransformerBlock3D(nn.Module):
    """vst:173-273 -- pre-LN shifted-window block (engine.block_forward)."""

    def __init__(self, dim, num_heads, window_size=(2, 7, 7), shift_size=(0, 0, 0),
                 mlp_ratio=4., qkv_bias=True, qk_scale=None, drop=0., attn_drop=0., drop_path=0.,
                 act_layer=nn.GELU, norm_layer=nn.LayerNorm, use_checkpoint=False):
        super().__init__()
        self.dim = dim
        self.num_heads = num_heads
        self.window_size = window_size
        self.shift_size = shift_size
        self.mlp_ratio = mlp_ratio
        self.use_checkpoint = use_checkpoint
        assert 0 <= self.shift_size[0] < self.window_size[0], "shift_size must in 0-window_size"
        assert 0 <= self.shift_size[1] < self.window_size[1], "shift_size must in 0-window_size"
        assert 0 <= self.shift_size[2] < self.window_size[2], "shift_size must in 0-window_size"
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention3D(dim, window_size=self.window_size, num_heads=num_heads,
                                      qkv_bias=qkv_bias, qk_scale=qk_scale, attn_drop=attn_drop, proj_drop=drop)
        self.drop_path = DropPath(drop_path) if drop_path > 0. else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop)

    def drop_scales(self):
        if isinstance(self.drop_path, DropPath):
            return (self.drop_path.sample_scale(), self.drop_path.sample_scale())
        return (1.0, 1.0)

    def param_dict(self):
        return {n: p for n, p in self.named_parameters() if n in engine.BlockWeights.NAMES}

    def forward(self, x, mask_matrix):
        """x: (B, D, H, W, C) fp32 on the GPU; mask_matrix: (nW, N, N) additive."""
        _lib.require_gpu(x)
        if self.training and x.shape[0] > 1 and isinstance(self.drop_path, DropPath) and self.drop_path.drop_prob > 0:
            # timm DropPath draws per sample: one pass per sample
            return torch.cat([self.forward(x[i:i + 1], mask_matrix) for i in range(x.shape[0])], dim=0)
        names = engine.BlockWeights.NAMES
        params = self.param_dict()
        return _BlockFn.apply(x, mask_matrix, self, *[params[n] for n in names])


class _BlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mask, blk, *plist):
        B, D, H, W, C = x.shape
        names = engine.BlockWeights.NAMES
        params = dict(zip(names, plist))
        bw = engine.BlockWeights(params, torch.float32)
        geo = engine.SwinGeometry(B, D, H, W, blk.window_size, any(s > 0 for s in blk.shift_size), x.device)
        geo_shift = tuple(blk.shift_size)
        if geo.shifted and tuple(s for s in geo.ss) != engine.get_window_size_tuple((D, H, W), blk.window_size,
                                                                                     geo_shift)[1]:
            raise NotImplementedError("shift_size must be window_size // 2 (as BasicLayer builds it)")
        m = mask.float().contiguous() if (mask is not None and geo.shifted) else None
        x2, sv = engine.block_forward(bw, geo, x.reshape(-1, C).float().contiguous(), torch.float32,
                                      blk.num_heads, drop_scale=blk.drop_scales(),
                                      mask=m, mask_nw=(m.shape[0] if m is not None else 0))
        ctx.state = (bw, geo, sv, blk.num_heads, x.shape)
        return x2.view(B, D, H, W, C)

    @staticmethod
    def backward(ctx, gy):
        bw, geo, sv, heads, shp = ctx.state
        grads = {n: torch.zeros_like(p) for n, p in bw.p.items()}
        gx = engine.block_backward(bw, geo, sv, gy.reshape(-1, shp[-1]).float().contiguous(), grads,
                                   torch.float32, heads)
        ctx.state = None
        return (gx.view(shp), None, None) + tuple(grads[n] for n in engine.BlockWeights.NAMES)


class PatchMerging(nn.Module):
    """vst:276-309 (unused at depths=[6]; kept for the state_dict schema of other depths)."""

    def __init__(self, dim, norm_layer=nn.LayerNorm):
        super().__init__()
        self.dim = dim
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = norm_layer(4 * dim)

    def forward(self, x):
        raise NotImplementedError("PatchMerging is not on the depths=[6] hot path")


class PatchExpand(nn.Module):
    """vst:311-338 (unused at depths=[6])."""

    def __init__(self, dim, norm_layer=nn.LayerNorm):
        super().__init__()
        self.dim = dim
        self.expand = nn.Linear(dim, 2 * dim, bias=False)
        self.norm = norm_layer(dim // 2)

    def forward(self, x, input_resolution):
        raise NotImplementedError("PatchExpand is not on the depths=[6] hot path")


class BasicLayer(nn.Module):
    """vst:358-437 -- one stage of `depth` blocks with alternating (0,0,0) /
    window//2 shifts; runs inside the fused SwinTransformer3DNet path."""

    def __init__(self, dim, depth, num_heads, window_size=(1, 7, 7), mlp_ratio=4., qkv_bias=False,
                 qk_scale=None, drop=0., attn_drop=0., drop_path=0., norm_layer=nn.LayerNorm,
                 downsample=None, use_checkpoint=False):
        super().__init__()
        self.window_size = window_size
        self.shift_size = tuple(i // 2 for i in window_size)
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        self.blocks = nn.ModuleList([
            SwinTransformerBlock3D(
                dim=dim, num_heads=num_heads, window_size=window_size,
                shift_size=(0, 0, 0) if (i % 2 == 0) else self.shift_size,
                mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop, attn_drop=attn_drop,
                drop_path=drop_path[i] if isinstance(drop_path, list) else drop_path,
                norm_layer=norm_layer, use_checkpoint=use_checkpoint)
            for i in range(depth)])
        self.downsample = downsample
        if self.downsample is not None:
            self.downsample = downsample(dim=dim, norm_layer=norm_layer)

    def forward(self, x):
        """x: (B, C, D, H, W) -> (B, C, D, H, W), blocks on the HIP path."""
        B, C, D, H, W = x.shape
        window_size, shift_size = get_window_size((D, H, W), self.window_size, self.shift_size)
        Dp, Hp, Wp = [int(math.ceil(n / w)) * w for n, w in zip((D, H, W), window_size)]
        mask = compute_mask(Dp, Hp, Wp, window_size, shift_size, x.device)
        t = x.permute(0, 2, 3, 4, 1).contiguous()
        for blk in self.blocks:
            t = blk(t, mask)
        if self.downsample is not None:
            t = self.downsample(t)
        return t.permute(0, 4, 1, 2, 3)


class PatchEmbed3D(nn.Module):
    """vst:440-479 -- k4s4 Conv3d; a GEMM on the patch-blocked layout in the fused path."""

    def __init__(self, patch_size=(2, 4, 4), in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        self.patch_size = patch_size
        self.in_chans = in_chans
        self.embed_dim = embed_dim
        self.proj = nn.Conv3d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None

    def forward(self, x):
        """vst:460-479: end-pad to the patch size, k4s4 conv (one HIP GEMM)."""
        from ._standalone import PatchEmbedFn
        _lib.require_gpu(x)
        if tuple(self.patch_size) != (4, 4, 4) or self.norm is not None:
            raise NotImplementedError("HIP PatchEmbed3D: patch (4, 4, 4), patch_norm False (config_swin)")
        return PatchEmbedFn.apply(x, self.proj.weight, self.proj.bias)


class PatchUnembed3D(nn.Module):
    """vst:481-531 -- k4s4 ConvTranspose3d; a GEMM on the patch-blocked layout in the fused path."""

    def __init__(self, patch_size: List[int], in_channels: int = 3, embed_dim: int = 96,
                 norm_layer: Optional[Callable[..., nn.Module]] = None) -> None:
        super().__init__()
        self.tuple_patch_size = (patch_size[0], patch_size[1], patch_size[2])
        self.proj = nn.ConvTranspose3d(embed_dim, in_channels, kernel_size=self.tuple_patch_size,
                                       stride=self.tuple_patch_size)
        self.norm = norm_layer(in_channels) if norm_layer is not None else nn.Identity()

    def forward(self, x, pre_size):
        """vst:510-531: k4s4 transposed conv (one HIP GEMM), crop to pre_size, norm."""
        from ._standalone import PatchUnembedFn, center_crop_like_reference
        _lib.require_gpu(x)
        if self.tuple_patch_size != (4, 4, 4):
            raise NotImplementedError("HIP PatchUnembed3D: patch (4, 4, 4)")
        y = center_crop_like_reference(PatchUnembedFn.apply(x, self.proj.weight, self.proj.bias), pre_size)
        if not isinstance(self.norm, nn.Identity):
            y = self.norm(y.permute(0, 2, 3, 4, 1)).permute(0, 4, 1, 2, 3)
        return y


class SwinTransformer3D(nn.Module):
    """vst:534-761 -- Swin backbone (patch embed -> BasicLayer(s) -> unembed).
    At depths=[6] it is executed by SwinTransformer3DNet's fused kernel path."""

    def __init__(self, pretrained=None, pretrained2d=True, patch_size=(4, 4, 4), in_chans=3, embed_dim=96,
                 depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24], window_size=(2, 7, 7), mlp_ratio=4.,
                 qkv_bias=True, qk_scale=None, drop_rate=0., attn_drop_rate=0., drop_path_rate=0.2,
                 norm_layer=nn.LayerNorm, patch_norm=False, frozen_stages=-1, use_checkpoint=False):
        super().__init__()
        self.pretrained = pretrained
        self.pretrained2d = pretrained2d
        self.num_layers = len(depths)
        self.embed_dim = embed_dim
        self.patch_norm = patch_norm
        self.frozen_stages = frozen_stages
        self.window_size = window_size
        self.patch_size = patch_size
        self.num_heads = num_heads
        self.patch_embed = PatchEmbed3D(patch_size=patch_size, in_chans=in_chans, embed_dim=embed_dim,
                                        norm_layer=norm_layer if self.patch_norm else None)
        self.patch_unembed = PatchUnembed3D(patch_size=patch_size, embed_dim=embed_dim,
                                            norm_layer=norm_layer if self.patch_norm else None,
                                            in_channels=in_chans)
        self.pos_drop = nn.Dropout(p=drop_rate)
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, sum(depths))]        # vst:603
        self.layers = nn.ModuleList()
        for i_layer in range(self.num_layers):
            self.layers.append(BasicLayer(
                dim=int(embed_dim * 2 ** i_layer), depth=depths[i_layer], num_heads=num_heads[i_layer],
                window_size=window_size, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale,
                drop=drop_rate, attn_drop=attn_drop_rate,
                drop_path=dpr[sum(depths[:i_layer]):sum(depths[:i_layer + 1])], norm_layer=norm_layer,
                downsample=PatchMerging if i_layer < self.num_layers - 1 else None,
                use_checkpoint=use_checkpoint))
        self.layers_up = nn.ModuleList()
        for i_layer in range(self.num_layers - 1):
            self.layers_up.append(PatchExpand(dim=int(embed_dim * 2 ** (self.num_layers - i_layer - 1))))
        self.num_features = int(embed_dim * 2 ** (self.num_layers - 1))
        self.norm = norm_layer(self.num_features)          # vst:633, never called in forward

    def forward(self, x):
        """vst:735-756 -- patch embed -> stages -> patch unembed to the input size."""
        x_size = [x.size()]
        x = self.pos_drop(self.patch_embed(x))
        for ii, layer in enumerate(self.layers):
            if ii < self.num_layers - 1:
                x_size.append(x.size())
            x = layer(x.contiguous())
        if self.num_layers > 1:
            raise NotImplementedError("HIP SwinTransformer3D: one stage (depths=[6], swin3D.py:315)")
        return self.patch_unembed(x, x_size[0])
