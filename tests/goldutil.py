"""Comparison helpers for golden fixtures (full tensors or norm + fixed sample)."""
import numpy as np

NSAMPLE = 4096


def sample_index(numel):
    """Must match tests/golden/make_golden.py::sample_index."""
    rng = np.random.default_rng(numel)
    return np.sort(rng.choice(numel, size=min(NSAMPLE, numel), replace=False))


def _np(x):
    if hasattr(x, "detach"):
        x = x.detach().cpu()
        if x.is_complex():
            x = x.to(__import__("torch").complex128)
        else:
            x = x.double()
        x = x.numpy()
    return np.asarray(x)


def nrmse(ref, x):
    ref = np.asarray(ref).astype(np.complex128).reshape(-1)
    x = np.asarray(x).astype(np.complex128).reshape(-1)
    den = np.linalg.norm(ref)
    return float(np.linalg.norm(x - ref) / (den if den > 0 else 1.0))


def golden_err(g, key, x):
    """NRMSE of tensor x against golden entry ``key`` (full or sampled form)."""
    a = _np(x)
    if key in g:
        assert a.shape == g[key].shape, (key, a.shape, g[key].shape)
        return nrmse(g[key], a)
    shape = tuple(g[key + "@shape"])
    assert a.shape == shape, (key, a.shape, shape)
    flat = a.reshape(-1)
    e_sample = nrmse(g[key + "@sample"], flat[sample_index(flat.size)])
    ref_norm = float(g[key + "@norm"])
    e_norm = abs(float(np.linalg.norm(flat.astype(np.complex128))) - ref_norm) / max(ref_norm, 1e-30)
    return max(e_sample, e_norm)


def has(g, key):
    return key in g or (key + "@sample") in g


def grad_keys(g, prefix):
    out = set()
    for k in g:
        if k.startswith(prefix + "grad::"):
            out.add(k[len(prefix + "grad::"):].split("@")[0])
    return sorted(out)
