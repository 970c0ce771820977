"""The two timm modules the DiT denoiser builds (dit = dl_cs/models/DiT.py:18
imports timm.models.vision_transformer.{Attention, Mlp}); timm is a third-party
dependency the reference does not vendor (unpinned), so its published module
structure is restated here for the state_dict schema (qkv / proj, fc1 / fc2).
The arithmetic runs inside the DiT network's fused HIP node (dit_engine:
dlcs_mhsa_fwd / _bwd and dlcs_gemm); calling these modules on their own raises."""
from torch import nn


class Attention(nn.Module):
    """timm Attention: qkv Linear -> [3, heads, head_dim] -> softmax(q k^T * head_dim^-0.5) v -> proj."""

    def __init__(self, dim, num_heads=8, qkv_bias=False, qk_norm=False, attn_drop=0.0, proj_drop=0.0,
                 norm_layer=nn.LayerNorm):
        super().__init__()
        assert dim % num_heads == 0, 'dim should be divisible by num_heads'
        if qk_norm or attn_drop or proj_drop:
            raise NotImplementedError("dl_cs Attention: qk_norm False, dropout 0 (DiTBlockFactor, dit:319)")
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.q_norm = nn.Identity()
        self.k_norm = nn.Identity()
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)

    def forward(self, x):
        raise NotImplementedError("dl_cs: Attention runs inside the DiT network's fused HIP node")


class Mlp(nn.Module):
    """timm Mlp: fc1 -> act -> fc2 (dropout 0, no norm)."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, norm_layer=None,
                 bias=True, drop=0.0, use_conv=False):
        super().__init__()
        if drop or norm_layer is not None or use_conv:
            raise NotImplementedError("dl_cs Mlp: drop 0, no norm, Linear layers (dit:323)")
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features, bias=bias)
        self.act = act_layer()
        self.drop1 = nn.Dropout(drop)
        self.norm = nn.Identity()
        self.fc2 = nn.Linear(hidden_features, out_features, bias=bias)
        self.drop2 = nn.Dropout(drop)

    def forward(self, x):
        raise NotImplementedError("dl_cs: Mlp runs inside the DiT network's fused HIP node")
