"""DiT denoiser networks (BASELINE config 5: configs/config_dit.yaml), MI355X build.

Same classes, constructor arguments and state_dict keys as the reference
(dit = dl_cs/models/DiT.py): DiTResNet (dit:1284-1350, the regularizer of
every unrolledDiT driver), DiTNet (dit:1199-1282) and the DiT backbone
(dit:411-632) with DiTBlockFactor blocks (dit:311-350), FinalLayer
(dit:388-408), TimestepEmbedder / LabelEmbedder / PosEmbed (dit:184-305) and
timm's Attention / Mlp (restated in dl_cs.models._timm: timm is not vendored by
the reference).  DiTResNet.forward / DiTNet.forward run the whole network as ONE
autograd node whose forward and hand-scheduled backward are HIP kernels
(dl_cs.models.dit_engine); the sub-modules are parameter containers.

Configurations outside the HIP path raise NotImplementedError: complex layers,
NUM_RESBLOCKS != 0 is allowed (it only changes the time padding), learn_sigma,
grids whose padded T is not a multiple of 4 or whose Y, X are not multiples of
4, head dims > 32, and the bf16 compute dtype (the DiT path is fp32).
"""
import collections.abc
import itertools
import math
from math import prod

import numpy as np
import torch
from torch import nn

from ._timm import Attention, Mlp
from .swin3D import ConvBlock


def modulate(x, shift, scale):
    """dit:22-23"""
    return x * (1 + scale.unsqueeze(1)) + shift.unsqueeze(1)


def to_3tuple(x):
    """dit:25-28"""
    if isinstance(x, collections.abc.Iterable):
        return x
    return (x, x, x)


def calc_num_patch(x, patch_size):
    """dit:30-53 -> (num_patch, grid_size, pad) of a [B, C, D, H, W] tensor."""
    patch_size = to_3tuple(patch_size)
    _, _, D, H, W = x.size()
    pad = np.array([(p - n % p) % p for n, p in zip((D, H, W), patch_size)])
    grid = np.array([(n + q) // p for n, q, p in zip((D, H, W), pad, patch_size)])
    return int(grid.prod()), grid, pad


def factorize(x, patchify_size, flag):
    """dit:55-65"""
    b, d, f, h, w = patchify_size
    if flag == 0:
        return x.reshape(b * f, h * w, d)
    return x.reshape(b, f, h, w, d).permute(0, 2, 3, 1, 4).reshape(b * h * w, f, d)


def unfactorize(x, patchify_size, flag):
    """dit:67-76"""
    b, d, f, h, w = patchify_size
    if flag == 0:
        return x.reshape(b, f * h * w, d)
    return x.reshape(b, h, w, f, d).permute(0, 3, 1, 2, 4).reshape(b, f * h * w, d)


def _fused_only(name):
    raise NotImplementedError(f"dl_cs: {name} runs inside the DiT network's fused HIP node "
                              "(DiTResNet / DiTNet forward)")


class PatchEmbed3D(nn.Module):
    """dit:78-138 -- Conv3d(k = s = patch) (a GEMM over the patch-blocked layout)."""

    def __init__(self, image_size=(224, 224, 20), patch_size=(2, 4, 4), in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        self.patch_size = to_3tuple(patch_size)
        self.image_size = to_3tuple(image_size)
        self.in_chans = in_chans
        self.embed_dim = embed_dim
        self.proj = nn.Conv3d(in_chans, embed_dim, kernel_size=self.patch_size, stride=self.patch_size)
        if norm_layer is not None:
            raise NotImplementedError("dl_cs DiT: PatchEmbed3D norm_layer=None (dit:435)")
        self.norm = None

    def forward(self, x):
        _fused_only("PatchEmbed3D")


class PatchUnembed3D(nn.Module):
    """dit:140-182 -- constructed by DiT (dit:440) but never called by its forward."""

    def __init__(self, patch_size=(2, 4, 4), in_channels=3, embed_dim=96, norm_layer=None):
        super().__init__()
        self.patch_size = to_3tuple(patch_size)
        self.proj = nn.ConvTranspose3d(embed_dim, in_channels, kernel_size=self.patch_size, stride=self.patch_size)
        self.norm = nn.Identity()

    def forward(self, x, pre_size):
        _fused_only("PatchUnembed3D")


class TimestepEmbedder(nn.Module):
    """dit:184-221"""

    def __init__(self, hidden_size, frequency_embedding_size=256):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(frequency_embedding_size, hidden_size, bias=True), nn.SiLU(),
                                 nn.Linear(hidden_size, hidden_size, bias=True))
        self.frequency_embedding_size = frequency_embedding_size

    @staticmethod
    def timestep_embedding(t, dim, max_period=10000):
        """dit:198-216 (the HIP path computes it with dlcs_timestep_embedding)."""
        half = dim // 2
        freqs = torch.exp(-math.log(max_period) * torch.arange(start=0, end=half, dtype=torch.float32) / half
                          ).to(device=t.device)
        args = t[:, None].float() * freqs[None]
        emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
        if dim % 2:
            emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
        return emb

    def forward(self, t):
        _fused_only("TimestepEmbedder")


class LabelEmbedder(nn.Module):
    """dit:224-251 -- label table with a classifier-free-guidance null row."""

    def __init__(self, num_classes, hidden_size, dropout_prob):
        super().__init__()
        use_cfg_embedding = dropout_prob > 0
        self.embedding_table = nn.Embedding(num_classes + use_cfg_embedding, hidden_size)
        self.num_classes = num_classes
        self.dropout_prob = dropout_prob

    def token_drop(self, labels, force_drop_ids=None):
        """dit:235-244"""
        if force_drop_ids is None:
            drop_ids = torch.rand(labels.shape[0], device=labels.device) < self.dropout_prob
        else:
            drop_ids = force_drop_ids == 1
        return torch.where(drop_ids, self.num_classes, labels)

    def effective_labels(self, labels, train, force_drop_ids=None):
        """dit:246-249 -- the label rows the forward reads."""
        if (train and self.dropout_prob > 0) or (force_drop_ids is not None):
            labels = self.token_drop(labels, force_drop_ids)
        return labels

    def forward(self, labels, train, force_drop_ids=None):
        _fused_only("LabelEmbedder")


def _sincos_1d(embed_dim, pos):
    """dit:771-789"""
    omega = np.arange(embed_dim // 2, dtype=np.float64)
    omega /= embed_dim / 2.
    omega = 1. / 10000 ** omega
    out = np.einsum('m,d->md', pos.reshape(-1), omega)
    return np.concatenate([np.sin(out), np.cos(out)], axis=1)


def get_3d_sincos_pos_embed_from_grid(embed_dim, grid):
    """dit:730-741"""
    assert embed_dim % 2 == 0
    return np.concatenate([_sincos_1d(embed_dim // 3, grid[0]), _sincos_1d(embed_dim // 3, grid[1]),
                           _sincos_1d(embed_dim // 3, grid[2])], axis=1)


def get_3d_sincos_pos_embed(embed_dim, grid_size, cls_token=False, extra_tokens=0):
    """dit:711-728 (meshgrid's default 'xy' indexing, as the reference)."""
    g = np.meshgrid(np.arange(grid_size[0], dtype=np.float32), np.arange(grid_size[1], dtype=np.float32),
                    np.arange(grid_size[2], dtype=np.float32))
    grid = np.stack(g, axis=0).reshape(3, 1, grid_size[0], grid_size[1], grid_size[2])
    pos_embed = get_3d_sincos_pos_embed_from_grid(embed_dim, grid)
    if cls_token and extra_tokens > 0:
        pos_embed = np.concatenate([np.zeros([extra_tokens, embed_dim]), pos_embed], axis=0)
    return pos_embed


class PosEmbed(nn.Module):
    """dit:253-305 -- frozen sin-cos table over the maximal grid, rows picked per grid."""

    def __init__(self, patch_size, hidden_size, max_grid_size=(128, 128, 15)):
        super().__init__()
        self.patch_size = patch_size
        self.hidden_size = hidden_size
        self.max_grid_size = max_grid_size
        self.pos_embed_table = nn.Parameter(torch.zeros(1, prod(self.max_grid_size), self.hidden_size),
                                            requires_grad=False)
        pos = get_3d_sincos_pos_embed(self.hidden_size, self.max_grid_size)
        self.pos_embed_table.data.copy_(torch.from_numpy(pos).float().unsqueeze(0))

    def index(self, grid_size):
        """dit:274 -- the reference's loop binds w to the frame index and f to the
        width index: row = f + h * max_F + w * max_F * max_H, in token order."""
        Fd, H, W = (int(v) for v in grid_size)
        mF, mH, _ = self.max_grid_size
        if Fd > self.max_grid_size[2] or W > mF or H > mH:
            raise ValueError(f"token grid {grid_size} exceeds PosEmbed max_grid_size {self.max_grid_size}")
        return np.array([f + h * mF + w * mF * mH for w, h, f in itertools.product(range(Fd), range(H), range(W))],
                        dtype=np.int64)

    def forward(self, grid_size):
        return self.pos_embed_table[:, self.index(grid_size), :]


class DiTBlockFactor(nn.Module):
    """dit:311-350 -- adaLN-Zero block with factorised (per-position over frames,
    then per-frame over positions) self-attention sharing one Attention."""

    def __init__(self, hidden_size, num_heads, mlp_ratio=4.0, **block_kwargs):
        super().__init__()
        self.norm1 = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        self.norm2 = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        self.attn = Attention(hidden_size, num_heads=num_heads, qkv_bias=True, **block_kwargs)
        self.norm3 = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        mlp_hidden_dim = int(hidden_size * mlp_ratio)
        approx_gelu = lambda: nn.GELU(approximate="tanh")  # noqa: E731
        self.mlp = Mlp(in_features=hidden_size, hidden_features=mlp_hidden_dim, act_layer=approx_gelu, drop=0)
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(hidden_size, 9 * hidden_size, bias=True))

    def forward(self, x, c, patchify_size):
        _fused_only("DiTBlockFactor")


class DiTBlock(nn.Module):
    """dit:353-385 -- the unfactorised adaLN-Zero block (schema only: DiT builds
    DiTBlockFactor, dit:448-451)."""

    def __init__(self, hidden_size, num_heads, mlp_ratio=4.0, **block_kwargs):
        super().__init__()
        self.norm1 = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        self.attn = Attention(hidden_size, num_heads=num_heads, qkv_bias=True, **block_kwargs)
        self.norm2 = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        mlp_hidden_dim = int(hidden_size * mlp_ratio)
        approx_gelu = lambda: nn.GELU(approximate="tanh")  # noqa: E731
        self.mlp = Mlp(in_features=hidden_size, hidden_features=mlp_hidden_dim, act_layer=approx_gelu, drop=0)
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(hidden_size, 6 * hidden_size, bias=True))

    def forward(self, x, c):
        _fused_only("DiTBlock")


class FinalLayer(nn.Module):
    """dit:388-408"""

    def __init__(self, hidden_size, patch_size, out_channels):
        super().__init__()
        patch_size = to_3tuple(patch_size)
        self.norm_final = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        self.linear = nn.Linear(hidden_size, patch_size[0] * patch_size[1] * patch_size[2] * out_channels, bias=True)
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(hidden_size, 2 * hidden_size, bias=True))

    def forward(self, x, c):
        _fused_only("FinalLayer")


class DiT(nn.Module):
    """dit:411-632 -- Diffusion transformer backbone (DiTBlockFactor blocks)."""

    def __init__(self, input_size=(28, 180, 64), patch_size=(2, 4, 4), in_channels=4, hidden_size=1152, depth=28,
                 num_heads=16, mlp_ratio=4.0, class_dropout_prob=0.1, num_classes=1, learn_sigma=False):
        super().__init__()
        self.learn_sigma = learn_sigma
        self.in_channels = in_channels
        self.out_channels = in_channels * 2 if learn_sigma else in_channels
        self.patch_size = patch_size
        self.num_heads = num_heads
        self.x_embedder = PatchEmbed3D(input_size, patch_size, in_channels, hidden_size, norm_layer=None)
        self.t_embedder = TimestepEmbedder(hidden_size)
        self.y_embedder = LabelEmbedder(num_classes, hidden_size, class_dropout_prob)
        self.x_unembedder = PatchUnembed3D(patch_size=patch_size, in_channels=in_channels, embed_dim=hidden_size,
                                           norm_layer=None)
        self.pos_embedder = PosEmbed(patch_size, hidden_size)
        self.blocks = nn.ModuleList([DiTBlockFactor(hidden_size, num_heads, mlp_ratio=mlp_ratio)
                                     for _ in range(depth)])
        self.final_layer = FinalLayer(hidden_size, patch_size, self.out_channels)
        self.initialize_weights()

    def initialize_weights(self):
        """dit:455-498"""
        def _basic_init(module):
            if isinstance(module, nn.Linear):
                torch.nn.init.xavier_uniform_(module.weight)
                if module.bias is not None:
                    nn.init.constant_(module.bias, 0)
        self.apply(_basic_init)
        w = self.x_embedder.proj.weight.data
        nn.init.xavier_uniform_(w.view([w.shape[0], -1]))
        nn.init.constant_(self.x_embedder.proj.bias, 0)
        nn.init.normal_(self.y_embedder.embedding_table.weight, std=0.02)
        nn.init.normal_(self.t_embedder.mlp[0].weight, std=0.02)
        nn.init.normal_(self.t_embedder.mlp[2].weight, std=0.02)
        for block in self.blocks:
            nn.init.constant_(block.adaLN_modulation[-1].weight, 0)
            nn.init.constant_(block.adaLN_modulation[-1].bias, 0)
        nn.init.constant_(self.final_layer.adaLN_modulation[-1].weight, 0)
        nn.init.constant_(self.final_layer.adaLN_modulation[-1].bias, 0)
        nn.init.constant_(self.final_layer.linear.weight, 0)
        nn.init.constant_(self.final_layer.linear.bias, 0)

    def forward(self, x, t, y):
        """dit:546-632 on a real [N, C, F, H, W] tensor (C = in_channels)."""
        from . import dit_engine
        return dit_engine.dit_forward_real(self, x, t, y)


def DiT_XL_2(**kwargs):
    return DiT(depth=28, hidden_size=1152, patch_size=2, num_heads=16, **kwargs)


def DiT_S_2(**kwargs):
    return DiT(depth=12, hidden_size=384, patch_size=2, num_heads=6, **kwargs)


def DiT_Cust(**kwargs):
    return DiT(depth=6, hidden_size=384, patch_size=2, num_heads=6, **kwargs)


DiT_models = {'DiT-XL/2': DiT_XL_2, 'DiT-S/2': DiT_S_2, 'DiT-Cust': DiT_Cust}


class _DiTRegularizer(nn.Module):
    """Shared pre / post processing of DiTNet and DiTResNet (dit:1225-1249, :1307-1331)."""

    def _check(self, use_complex_layers, learn_sigma):
        if use_complex_layers:
            raise NotImplementedError("dl_cs DiT: CONV_BLOCK.COMPLEX False (config_dit.yaml)")
        if learn_sigma:
            raise NotImplementedError("dl_cs DiT: LEARN_SIGMA False (config_dit.yaml)")

    def forward(self, x, t, c):
        from . import dit_engine
        return dit_engine.dit_regularizer_forward(self, x, t, c)


class DiTNet(_DiTRegularizer):
    """dit:1199-1282 -- the DiT straight on the 2E real channels."""

    residual_convs = False

    def __init__(self, num_blocks, in_chans, chans, kernel_size, act_type='relu', num_heads=6, num_layers=12,
                 use_complex_layers=False, circular_pad=True, learn_sigma=False):
        super().__init__()
        self._check(use_complex_layers, learn_sigma)
        self.use_complex_layers = use_complex_layers
        self.circular_pad = circular_pad
        self.pad_size = (2 * num_blocks + 2) * (kernel_size - 1) // 2
        self.SFE = ConvBlock(in_chans, chans, kernel_size=3, act_type='none', is_complex=use_complex_layers)
        self.DiT = DiT(depth=num_layers, hidden_size=chans, patch_size=(2, 4, 4), num_heads=num_heads,
                       in_channels=in_chans, learn_sigma=learn_sigma)
        self.final_layer = ConvBlock(chans, in_chans, kernel_size=3, act_type=act_type, is_complex=use_complex_layers)


class DiTResNet(_DiTRegularizer):
    """dit:1284-1350 -- SFE conv -> DiT (in_channels = chans) -> ReLU + conv of
    (DiT output + SFE output) -> crop, complex."""

    residual_convs = True

    def __init__(self, num_blocks, in_chans, chans, kernel_size, act_type='relu', num_heads=6, num_layers=12,
                 use_complex_layers=False, circular_pad=True, learn_sigma=False):
        super().__init__()
        self._check(use_complex_layers, learn_sigma)
        self.use_complex_layers = use_complex_layers
        self.circular_pad = circular_pad
        self.pad_size = (2 * num_blocks + 2) * (kernel_size - 1) // 2
        self.SFE = ConvBlock(in_chans, chans, kernel_size=3, act_type='none', is_complex=use_complex_layers)
        self.DiT = DiT(depth=num_layers, hidden_size=chans, patch_size=(2, 4, 4), num_heads=num_heads,
                       in_channels=chans, learn_sigma=learn_sigma)
        self.final_layer = ConvBlock(chans, in_chans, kernel_size=3, act_type=act_type, is_complex=use_complex_layers)
