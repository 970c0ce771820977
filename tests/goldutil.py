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


def oracle_grads(loss_fn, sd, dtype, trainable=None):
    """Parameter gradients of loss_fn(P, cast) evaluated by the CPU oracle at
    `dtype` (torch.float32 or torch.float64) on the weights of state dict `sd`;
    cast(t) converts an input tensor to the matching real / complex dtype."""
    import torch
    cd = torch.complex128 if dtype == torch.float64 else torch.complex64

    def cast(t):
        t = t.detach().cpu()
        return t.to(cd) if t.is_complex() else (t.to(dtype) if t.is_floating_point() else t)

    P = {}
    for k, v in sd.items():
        v = v.detach().cpu()
        if torch.is_floating_point(v):
            v = v.to(dtype).clone().requires_grad_(trainable is None or bool(trainable(k)))
        P[k] = v
    loss_fn(P, cast).backward()
    return {k: v.grad.numpy() for k, v in P.items() if torch.is_tensor(v) and v.grad is not None}


def assert_f64_floor(hip, o32, o64, label, min_tol=1e-5, factor=4.0):
    """Per gradient tensor n (in all three dicts):
         NRMSE(hip[n] vs o64[n]) <= max(min_tol, factor * NRMSE(o32[n] vs o64[n])),
    i.e. the HIP build is held to the fp32 oracle's own distance from a float64
    evaluation (the floor set by ReLU masks / L1 signs that flip for values within
    fp32 rounding of 0), not to a fixed loose tolerance.  Prints the measured floors."""
    rows = []
    for n in sorted(set(hip) & set(o32) & set(o64)):
        h = hip[n].detach().cpu().numpy() if hasattr(hip[n], "detach") else np.asarray(hip[n])
        floor = nrmse(o64[n], o32[n])
        err = nrmse(o64[n], h)
        rows.append((err / max(min_tol, factor * floor), err, floor, n))
    assert rows, f"{label}: no gradients compared"
    rows.sort(reverse=True)
    r = rows[0]
    print(f"{label}: {len(rows)} grads vs f64; worst err/bound {r[0]:.3g} ({r[3]}: err {r[1]:.3g}, "
          f"oracle32 floor {r[2]:.3g}); largest floor {max(x[2] for x in rows):.3g}, "
          f"largest err {max(x[1] for x in rows):.3g}")
    bad = [x for x in rows if x[0] > 1.0]
    assert not bad, bad[:5]
