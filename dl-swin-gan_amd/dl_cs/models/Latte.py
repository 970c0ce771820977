"""Latte video-diffusion denoiser (BASELINE config 5: configs/config_latte.yaml), MI355X build.

Same classes, constructor arguments and state_dict keys as the reference
(lat = dl_cs/models/Latte.py): LatteNet (lat:861-937, the regularizer of every
unrolledLatte driver) around the Latte backbone (lat:338-587): a per-frame 2-D
patch embed (PatchEmbed2D, lat:89-147), fixed 2-D sin-cos position and 1-D
sin-cos frame tables (PosEmbed lat:161-191, TempEmbed lat:149-159), and
TransformerBlocks (lat:294-316) alternating spatial attention (the tokens of
one frame) and temporal attention (the frames of one patch position), adaLN-Zero
conditioned on the timestep embedding, then FinalLayer (lat:318-336) and
unpatchify2 (lat:450-475).  LatteNet.forward runs the whole network as ONE
autograd node whose forward and hand-scheduled backward are HIP kernels
(dl_cs.models.latte_engine); the sub-modules are parameter containers.  LatteNet
declares an SFE and a final ConvBlock that its forward never calls (lat:875,
:880, :926-937): they are kept for the state_dict schema.

Configurations outside the HIP path raise NotImplementedError: complex layers,
learn_sigma, extras != 1 (label / text conditioning is not reachable from
LatteNet), grids whose padded T is not a multiple of 4 or whose Y, X are not
multiples of 4, head dims > 32, an odd layer count, and the bf16 compute dtype.
"""
import collections.abc
import itertools
import math

import numpy as np
import torch
from torch import nn

from ._timm import Mlp
from .DiT import LabelEmbedder, TimestepEmbedder
from .swin3D import ConvBlock


def modulate(x, shift, scale):
    """lat:33-34"""
    return x * (1 + scale.unsqueeze(1)) + shift.unsqueeze(1)


def to_2tuple(x):
    """lat:36-39"""
    if isinstance(x, collections.abc.Iterable):
        return x
    return (x, x)


def _fused_only(name):
    raise NotImplementedError(f"dl_cs: {name} runs inside the Latte network's fused HIP node (LatteNet forward)")


class Attention(nn.Module):
    """lat:45-87 -- qkv Linear, heads, softmax(q k^T scale) v, proj (attention_mode
    'math'; 'xformers' / 'flash' compute the same function)."""

    def __init__(self, dim, num_heads=8, qkv_bias=False, attn_drop=0., proj_drop=0., use_lora=False,
                 attention_mode='math'):
        super().__init__()
        assert dim % num_heads == 0, 'dim should be divisible by num_heads'
        self.num_heads = num_heads
        self.scale = (dim // num_heads) ** -0.5
        self.attention_mode = attention_mode
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)

    def forward(self, x):
        _fused_only("Attention")


class PatchEmbed2D(nn.Module):
    """lat:89-147 -- Conv2d(k = s = patch) per frame (a GEMM over the 16-row 2-D
    patches of the patch-blocked layout)."""

    def __init__(self, image_size=(224, 224), patch_size=(2, 2), in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        self.patch_size = to_2tuple(patch_size)
        self.image_size = to_2tuple(image_size)
        self.in_chans = in_chans
        self.embed_dim = embed_dim
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=self.patch_size, stride=self.patch_size)
        if norm_layer is not None:
            raise NotImplementedError("dl_cs Latte: PatchEmbed2D norm_layer=None (lat:369)")
        self.norm = None

    def forward(self, x):
        _fused_only("PatchEmbed2D")


def get_1d_sincos_pos_embed_from_grid(embed_dim, pos):
    """lat:622-640"""
    assert embed_dim % 2 == 0
    omega = np.arange(embed_dim // 2, dtype=np.float64)
    omega /= embed_dim / 2.
    omega = 1. / 10000 ** omega
    out = np.einsum('m,d->md', np.asarray(pos).reshape(-1), omega)
    return np.concatenate([np.sin(out), np.cos(out)], axis=1)


def get_1d_sincos_temp_embed(embed_dim, length):
    """lat:589-591"""
    return get_1d_sincos_pos_embed_from_grid(embed_dim, torch.arange(0, length).unsqueeze(1).numpy())


def get_2d_sincos_pos_embed(embed_dim, grid_size, cls_token=False, extra_tokens=0):
    """lat:593-608 (meshgrid's default 'xy' indexing, as the reference)."""
    grid = np.meshgrid(np.arange(grid_size[1], dtype=np.float32), np.arange(grid_size[0], dtype=np.float32))
    grid = np.stack(grid, axis=0).reshape([2, 1, grid_size[0], grid_size[1]])
    assert embed_dim % 2 == 0
    emb = np.concatenate([get_1d_sincos_pos_embed_from_grid(embed_dim // 2, grid[0]),
                          get_1d_sincos_pos_embed_from_grid(embed_dim // 2, grid[1])], axis=1)
    if cls_token and extra_tokens > 0:
        emb = np.concatenate([np.zeros([extra_tokens, embed_dim]), emb], axis=0)
    return emb


class TempEmbed(nn.Module):
    """lat:149-159 -- frozen 1-D sin-cos table over frames."""

    def __init__(self, hidden_size, max_frames=100):
        super().__init__()
        self.temp_embed_table = nn.Parameter(torch.zeros(1, max_frames, hidden_size), requires_grad=False)
        self.temp_embed_table.data.copy_(torch.from_numpy(get_1d_sincos_temp_embed(hidden_size, max_frames))
                                         .float().unsqueeze(0))

    def forward(self, frames):
        return self.temp_embed_table[:, :frames, :]


class PosEmbed(nn.Module):
    """lat:161-191 -- frozen 2-D sin-cos table over the maximal patch grid."""

    def __init__(self, patch_size, hidden_size, max_grid_size=(128, 128)):
        super().__init__()
        self.patch_size = patch_size
        self.hidden_size = hidden_size
        self.max_grid_size = max_grid_size
        self.pos_embed_table = nn.Parameter(torch.zeros(1, math.prod(self.max_grid_size), self.hidden_size),
                                            requires_grad=False)
        self.pos_embed_table.data.copy_(torch.from_numpy(get_2d_sincos_pos_embed(hidden_size, max_grid_size))
                                        .float().unsqueeze(0))

    def index(self, grid_size):
        """lat:183 -- the reference binds w to the row index and h to the column
        index: row = h + w * max_H over product(range(H), range(W)), in token order
        (token p = row * W + col)."""
        H, W = (int(v) for v in grid_size)
        max_H, max_W = self.max_grid_size
        if H > max_W or W > max_H:
            raise ValueError(f"patch grid {grid_size} exceeds PosEmbed max_grid_size {self.max_grid_size}")
        return np.array([h + w * max_H for w, h in itertools.product(range(H), range(W))], dtype=np.int64)

    def forward(self, grid_size):
        return self.pos_embed_table[:, self.index(grid_size)]


class TransformerBlock(nn.Module):
    """lat:294-316 -- adaLN-Zero block: x += g_msa attn(modulate(LN x)); x += g_mlp mlp(modulate(LN x))."""

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
        _fused_only("TransformerBlock")


class FinalLayer(nn.Module):
    """lat:318-336"""

    def __init__(self, hidden_size, patch_size, out_channels):
        super().__init__()
        self.norm_final = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        self.linear = nn.Linear(hidden_size, patch_size[0] * patch_size[1] * out_channels, bias=True)
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(hidden_size, 2 * hidden_size, bias=True))

    def forward(self, x, c):
        _fused_only("FinalLayer")


class Latte(nn.Module):
    """lat:338-587 -- the video diffusion transformer (spatial / temporal block pairs)."""

    def __init__(self, input_size=32, patch_size=2, in_channels=4, hidden_size=1152, depth=28, num_heads=16,
                 mlp_ratio=4.0, num_frames=16, class_dropout_prob=0.1, num_classes=1000, learn_sigma=True, extras=1,
                 attention_mode='math'):
        super().__init__()
        self.learn_sigma = learn_sigma
        self.in_channels = in_channels
        self.out_channels = in_channels * 2 if learn_sigma else in_channels
        self.patch_size = patch_size
        self.num_heads = num_heads
        self.extras = extras
        self.num_frames = num_frames
        self.x_embedder = PatchEmbed2D(patch_size=patch_size, in_chans=in_channels, embed_dim=hidden_size)
        self.t_embedder = TimestepEmbedder(hidden_size)
        if self.extras == 2:
            self.y_embedder = LabelEmbedder(num_classes, hidden_size, class_dropout_prob)
        if self.extras == 78:
            self.text_embedding_projection = nn.Sequential(nn.SiLU(), nn.Linear(77 * 768, hidden_size, bias=True))
        self.pos_embedder = PosEmbed(patch_size=patch_size, hidden_size=hidden_size)
        self.temp_embedder = TempEmbed(hidden_size=hidden_size)
        self.hidden_size = hidden_size
        self.blocks = nn.ModuleList([TransformerBlock(hidden_size, num_heads, mlp_ratio=mlp_ratio,
                                                      attention_mode=attention_mode) for _ in range(depth)])
        self.final_layer = FinalLayer(hidden_size, to_2tuple(patch_size), self.out_channels)
        self.initialize_weights()

    def initialize_weights(self):
        """lat:395-433"""
        def _basic_init(module):
            if isinstance(module, nn.Linear):
                torch.nn.init.xavier_uniform_(module.weight)
                if module.bias is not None:
                    nn.init.constant_(module.bias, 0)
        self.apply(_basic_init)
        w = self.x_embedder.proj.weight.data
        nn.init.xavier_uniform_(w.view([w.shape[0], -1]))
        nn.init.constant_(self.x_embedder.proj.bias, 0)
        if self.extras == 2:
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

    def forward(self, x, t, y=None, text_embedding=None, use_fp16=False):
        _fused_only("Latte (call LatteNet)")


class LatteNet(nn.Module):
    """lat:861-937 -- circular time pad, Latte on the 2E real channels, crop, complex."""

    def __init__(self, num_blocks, in_chans, chans, kernel_size, act_type='relu', num_heads=6, num_layers=12,
                 use_complex_layers=False, circular_pad=True, learn_sigma=False):
        super().__init__()
        if use_complex_layers:
            raise NotImplementedError("dl_cs Latte: CONV_BLOCK.COMPLEX False (config_latte.yaml)")
        if learn_sigma:
            raise NotImplementedError("dl_cs Latte: LEARN_SIGMA False (config_latte.yaml)")
        self.use_complex_layers = use_complex_layers
        self.circular_pad = circular_pad
        self.pad_size = (2 * num_blocks + 2) * (kernel_size - 1) // 2
        self.SFE = ConvBlock(in_chans, chans, kernel_size=3, act_type='none', is_complex=use_complex_layers)
        self.Latte = Latte(depth=num_layers, hidden_size=chans, patch_size=(4, 4), num_heads=num_heads,
                           in_channels=in_chans, learn_sigma=learn_sigma)
        self.final_layer = ConvBlock(chans, in_chans, kernel_size=3, act_type=act_type, is_complex=use_complex_layers)

    def forward(self, x, t, c):
        from . import latte_engine
        return latte_engine.latte_forward(self, x, t, c)
