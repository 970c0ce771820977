"""Reference state_dict key schema for SwinTransformer3DNet (TEST INFRASTRUCTURE).

Key names follow the reference's module tree (s3d:371-391, vst:534-633): the
deep-feature-extraction blocks are registered twice (DFE.resswin_blocks.i and
DFE.layers.i, s3d:350-357); only the first alias is listed by named_parameters.
"""


def swin3d_param_shapes(prefix, C=160, depth=6, heads=8, window=(7, 8, 8), patch=(4, 4, 4),
                        mlp_ratio=4):
    nrel = (2 * window[0] - 1) * (2 * window[1] - 1) * (2 * window[2] - 1)
    out = {
        prefix + "patch_embed.proj.weight": (C, C) + patch,
        prefix + "patch_embed.proj.bias": (C,),
        prefix + "patch_unembed.proj.weight": (C, C) + patch,
        prefix + "patch_unembed.proj.bias": (C,),
    }
    for i in range(depth):
        b = f"{prefix}layers.0.blocks.{i}."
        out.update({
            b + "norm1.weight": (C,), b + "norm1.bias": (C,),
            b + "attn.relative_position_bias_table": (nrel, heads),
            b + "attn.qkv.weight": (3 * C, C), b + "attn.qkv.bias": (3 * C,),
            b + "attn.proj.weight": (C, C), b + "attn.proj.bias": (C,),
            b + "norm2.weight": (C,), b + "norm2.bias": (C,),
            b + "mlp.fc1.weight": (mlp_ratio * C, C), b + "mlp.fc1.bias": (mlp_ratio * C,),
            b + "mlp.fc2.weight": (C, mlp_ratio * C), b + "mlp.fc2.bias": (C,),
        })
    out[prefix + "norm.weight"] = (C,)
    out[prefix + "norm.bias"] = (C,)
    return out


def swinnet_param_shapes(in_chans=4, C=160, num_swinblocks=1, with_aliases=False):
    out = {"SFE.layers.2.conv.weight": (C, in_chans, 3, 3, 3), "SFE.layers.2.conv.bias": (C,)}
    aliases = ["DFE.resswin_blocks"] + (["DFE.layers"] if with_aliases else [])
    for a in aliases:
        for i in range(num_swinblocks):
            p = f"{a}.{i}.layers."
            out.update(swin3d_param_shapes(p + "0.transformer.", C=C))
            out[p + "1.layers.2.conv.weight"] = (C, C, 3, 3, 3)
            out[p + "1.layers.2.conv.bias"] = (C,)
    out[f"DFE.layers.{num_swinblocks}.layers.2.conv.weight"] = (C, C, 3, 3, 3)
    out[f"DFE.layers.{num_swinblocks}.layers.2.conv.bias"] = (C,)
    out["final_layer.layers.2.conv.weight"] = (in_chans, C, 3, 3, 3)
    out["final_layer.layers.2.conv.bias"] = (in_chans,)
    return out
