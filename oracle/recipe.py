"""Deterministic weight / input recipes (TEST INFRASTRUCTURE, see oracle/__init__).

The same recipe is applied to the reference modules (golden generation, survey
container only) and to the oracle / HIP implementation (tests, GPU box), so the
goldens need not carry the 6.7 M parameters of each regularizer.

Parameters are filled by *name*: the value of a tensor depends only on
``(seed, key)``, never on registration order.  Keys are visited in sorted order,
so for aliased parameters (``DFE.layers.0.*`` is the same module as
``DFE.resswin_blocks.0.*``, swin3D.py:350-357) the lexicographically last alias
wins in every implementation that shares the same aliasing.
"""
import math
import zlib

import torch


def _gen(seed, key):
    g = torch.Generator(device="cpu")
    g.manual_seed((int(seed) * 1000003 + zlib.crc32(key.encode())) & 0x7FFFFFFFFFFF)
    return g


def param_value(seed, key, shape):
    """Value of parameter ``key`` (reference state_dict name) under ``seed``."""
    g = _gen(seed, key)
    u = torch.rand(shape, generator=g, dtype=torch.float64) * 2.0 - 1.0   # U(-1, 1)
    leaf = key.rsplit(".", 1)[-1]
    if "relative_position_bias_table" in key:
        v = 0.5 * u
    elif len(shape) >= 2:
        fan_in = 1
        for s in shape[1:]:
            fan_in *= s
        v = u / math.sqrt(fan_in)          # std = 1/sqrt(3 fan_in): PyTorch default scale
    elif ("norm" in key) and leaf == "weight":
        v = 1.0 + 0.1 * u
    else:                                   # biases, LayerNorm shifts
        v = 0.05 * u
    return v.to(torch.float32)


SKIP = ("relative_position_index", "step_size", "lamda", "pos_embed_table", "temp_embed_table")


def fill_state_dict(sd, seed):
    """Return a new {key: tensor} with every float parameter replaced by the recipe."""
    out = {}
    for k in sorted(sd.keys()):
        v = sd[k]
        if any(s in k for s in SKIP) or not torch.is_floating_point(v):
            out[k] = v.clone()
        else:
            out[k] = param_value(seed, k, tuple(v.shape))
    return out


def fill_module(module, seed):
    """In-place recipe fill of an nn.Module (reference or HIP implementation)."""
    sd = module.state_dict(keep_vars=True)
    with torch.no_grad():
        for k in sorted(sd.keys()):
            v = sd[k]
            if any(s in k for s in SKIP) or not torch.is_floating_point(v):
                continue
            v.copy_(param_value(seed, k, tuple(v.shape)).to(v.device))
    return module


def randn(seed, shape, dtype=torch.float32):
    g = torch.Generator(device="cpu")
    g.manual_seed(int(seed))
    return torch.randn(shape, generator=g, dtype=torch.float64).to(dtype)


def crandn(seed, shape):
    g = torch.Generator(device="cpu")
    g.manual_seed(int(seed))
    re = torch.randn(shape, generator=g, dtype=torch.float64)
    im = torch.randn(shape, generator=g, dtype=torch.float64)
    return torch.complex(re, im).to(torch.complex64)


def sense_maps(seed, B, E, C, Y, X):
    """ESPIRiT-like maps c64 [B,E,C,1,Y,X], normalised per pixel: sum_{e,c}|S|^2 = 1."""
    m = crandn(seed, (B, E, C, 1, Y, X)).to(torch.complex128)
    nrm = torch.sqrt((m.abs() ** 2).sum(dim=(1, 2), keepdim=True))
    return (m / nrm).to(torch.complex64)


def binary_mask(seed, shape, density=0.3):
    g = torch.Generator(device="cpu")
    g.manual_seed(int(seed))
    return (torch.rand(shape, generator=g, dtype=torch.float64) < density).to(torch.float32)
