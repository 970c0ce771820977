"""SENSE forward / adjoint and the orthonormal 2D FFT on MI355X.

Drop-in for the reference's ``dl_cs.mri.transforms`` (tr:12-110): same class
names, constructor arguments, call signatures and assertions.  GPU tensors run
the hand-written HIP kernels of libdlcs_hip (``dlcs_sense_fwd`` /
``dlcs_sense_adj`` / ``dlcs_fft2``) and never anything else.  CPU tensors --
the reference calls SenseModel inside CPU DataLoader workers
(preprocess.py:140-164) -- take an explicit host path (``_host_forward`` /
``_host_adjoint``, torch.fft on the CPU); mixing devices raises.
"""
from typing import Optional

import torch
from torch import nn

from .. import _lib
from .. import diag as _diag


# Optional live profiling (bench.py): when PROFILE is a list, every SENSE
# forward / adjoint / normal operator appends (start_event, end_event,
# algorithmic_bytes, entry point, SenseModel-call bytes) recorded on the
# launching stream; algorithmic bytes = every operand this entry point needs
# read or written once (for the row-sparse operators: only the sampled k-space
# lines); SenseModel-call bytes = SURVEY.md §8(d)'s accounting of the
# reference's dense calls the entry point replaces (_call_bytes).
PROFILE = None


def _call_bytes(B, E, C, T, Y, X):
    """Bytes of one reference SenseModel call (A or A^H) per SURVEY.md §8(d):
    image in and out (complex64, 2 x 8 B), maps (complex64, read by the call and
    by its conjugate pass: 2 x 8 B per coil pixel), float mask and the coil
    k-space once -- 55.54 MB at the headline [1, 8, 20, 192, 160]."""
    return (16 * B * E * T * Y * X + 16 * B * E * C * Y * X + 4 * B * T * Y * X + 8 * B * C * T * Y * X)


def _timed_call(name, nbytes, calls, *args):
    if PROFILE is None:
        return _lib.call(name, *args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _lib.call(name, *args)
    e1.record()
    PROFILE.append((e0, e1, nbytes, name, calls))


def _c64(t):
    return t if t.dtype == torch.complex64 else t.to(torch.complex64)


def _workspace(B, C, T, Y, X, device):
    n = B * C * T * Y * X
    return torch.empty(n, dtype=torch.complex64, device=device)


def _weights_arg(weights, B, C, T, Y, X):
    """weights (tr:58 docstring: [B, coils, t, y, x]; in practice the mask [B,1,T,Y,X])."""
    if weights is None or isinstance(weights, float):
        return None, 1
    w = weights
    if w.dtype != torch.float32:
        w = w.real.float() if torch.is_complex(w) else w.float()
    if w.dim() == 4:
        w = w.unsqueeze(1)
    wc = w.shape[1]
    if wc not in (1, C):
        raise ValueError(f"weights coil dim must be 1 or {C}, got {wc}")
    w = w.expand(B, wc, T, Y, X).contiguous()
    return w, wc


def sense_fwd_raw(x, maps, weights):
    B, E, T, Y, X = x.shape
    C = maps.shape[2]
    x = _c64(x).contiguous()
    m = _c64(maps).reshape(B, E, C, Y, X).contiguous()
    w, wc = _weights_arg(weights, B, C, T, Y, X)
    y = torch.empty((B, C, T, Y, X), dtype=torch.complex64, device=x.device)
    ws = _workspace(B, C, T, Y, X, x.device)
    nbytes = (x.numel() + m.numel() + y.numel()) * 8 + (w.numel() * 4 if w is not None else 0)
    _timed_call("dlcs_sense_fwd", nbytes, _call_bytes(B, E, C, T, Y, X),
                _lib.ptr(x), _lib.ptr(m), _lib.ptr(w), wc, _lib.ptr(y),
                B, E, C, T, Y, X, _lib.ptr(ws), ws.numel() * 8, _lib.stream())
    return y


def sense_adj_raw(y, maps, weights, base=None, sub=None, step=1.0):
    """x = A^H y, or base + step * (A^H y - sub) when base is given (urs:109)."""
    B, C, T, Y, X = y.shape
    E = maps.shape[1]
    y = _c64(y).contiguous()
    m = _c64(maps).reshape(B, E, C, Y, X).contiguous()
    w, wc = _weights_arg(weights, B, C, T, Y, X)
    out = torch.empty((B, E, T, Y, X), dtype=torch.complex64, device=y.device)
    if base is not None:
        base = _c64(base).contiguous()
    if sub is not None:
        sub = _c64(sub).contiguous()
    if w is not None and _rows_enabled() and Y in _FAST_LEN and X in _FAST_LEN and E <= 2:
        # row-sparse adjoint: y is read only on the mask's sampled ky lines
        tab, jmax, lines = _rowtab(weights, w, wc, B, T, Y, X)
        jcap, lines = _jcap(jmax, Y), _lines(lines, B, wc, T, Y)
        nb = int(_lib.lib().dlcs_sense_rows_workspace_bytes(B, C, T, jcap, X))
        ws = torch.empty((nb + 7) // 8, dtype=torch.complex64, device=y.device)
        # algorithmic bytes: the sampled lines of y and of the weights, maps and out once (+ base / sub)
        nbytes = (lines * X * (8 * (C if wc == 1 else 1) + 4) + m.numel() * 8 +
                  out.numel() * 8 * (1 + (base is not None) + (sub is not None)))
        _timed_call("dlcs_sense_adj_rows", nbytes, _call_bytes(B, E, C, T, Y, X),
                    _lib.ptr(y), _lib.ptr(m), _lib.ptr(w), wc, _lib.ptr(tab), jcap,
                    _lib.ptr(out), _lib.ptr(base), _lib.ptr(sub), float(step), B, E, C, T, Y, X,
                    _lib.ptr(ws), ws.numel() * 8, _lib.stream())
        return out
    ws = _workspace(B, C, T, Y, X, y.device)
    nbytes = (y.numel() + m.numel() + out.numel() * (1 + (base is not None) + (sub is not None))) * 8 + \
        (w.numel() * 4 if w is not None else 0)
    _timed_call("dlcs_sense_adj", nbytes, _call_bytes(B, E, C, T, Y, X),
                _lib.ptr(y), _lib.ptr(m), _lib.ptr(w), wc, _lib.ptr(out),
                _lib.ptr(base), _lib.ptr(sub), float(step), B, E, C, T, Y, X,
                _lib.ptr(ws), ws.numel() * 8, _lib.stream())
    return out


class _SenseForwardFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, maps, weights):
        ctx.save_for_backward(maps, weights if torch.is_tensor(weights) else None)
        return sense_fwd_raw(x, maps, weights)

    @staticmethod
    def backward(ctx, gy):
        maps, weights = ctx.saved_tensors
        return sense_adj_raw(gy.contiguous(), maps, weights), None, None


class _SenseAdjointFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, maps, weights):
        ctx.save_for_backward(maps, weights if torch.is_tensor(weights) else None)
        return sense_adj_raw(y, maps, weights)

    @staticmethod
    def backward(ctx, gx):
        maps, weights = ctx.saved_tensors
        return sense_fwd_raw(gx.contiguous(), maps, weights), None, None


_FAST_LEN = (64, 80, 96, 128, 160, 192)
_ROWTAB = []          # [(weights tensor kept alive, version, geometry, table, jmax, lines)], most recent first


def _rows_enabled():
    import os
    return _diag.knob("DLCS_SENSE_ROWS", "1") != "0"


def _rowtab(key, w, wc, B, T, Y, X):
    """Row table of the weights tensor ``key`` (``w``: its float [B,Wc,T,Y,X]
    form) by dlcs_sense_rowtab: built once per mask and geometry, cached by the
    tensor object, its in-place version counter and the (B, Wc, T, Y, X) it was
    broadcast to (a [1,1,T,Y,X] mask reused with a larger batch gets its own
    table; the entry keeps the tensor alive).  The first use of a mask reads
    nothing back (jmax None: the kernels take the row capacity Y, their counts
    come from the device table), so a caller that builds a new mask per batch
    (preprocessing, the DiT A^H with 1 - mask) never waits on the host; the
    second use of the same mask reads its line counts once (jmax sizes the
    compressed-line workspace, lines the bench's byte count)."""
    geom = (B, wc, T, Y, X)
    for i, (wt, ver, g, tab, jmax, lines) in enumerate(_ROWTAB):
        if wt is key and ver == key._version and g == geom:
            if jmax is None:
                head = tab[:4 + B * wc * T].cpu()
                jmax, lines = int(head[0]), int(head[4:].sum())
                _ROWTAB[i] = (wt, ver, g, tab, jmax, lines)
            return tab, jmax, lines
    L = _lib.lib()
    nb = int(L.dlcs_sense_rowtab_bytes(B, wc, T, Y))
    tab = torch.empty((nb + 3) // 4, dtype=torch.int32, device=w.device)
    _lib.call("dlcs_sense_rowtab", _lib.ptr(w), wc, B, T, Y, X, _lib.ptr(tab), tab.numel() * 4, _lib.stream())
    _ROWTAB.insert(0, (key, key._version, geom, tab, None, None))
    del _ROWTAB[4:]
    return tab, None, None


def _jcap(jmax, Y):
    """Row capacity of the compressed-line workspace: the mask's max sampled lines
    per frame once known, else every line."""
    return Y if jmax is None else max(jmax, 1)


def _lines(lines, B, wc, T, Y):
    return B * wc * T * Y if lines is None else lines


def sense_normal_raw(x, maps, weights, sub=None, base_scale=1.0, step=1.0):
    """base_scale * x + step * (A^H A x - sub).  With a mask whose frames sample
    a subset of the phase-encode lines (the cine k-t masks), the row-sparse
    operator dlcs_sense_normal_rows (FFT_Y, the sampled lines through FFT_X /
    W^2 / IFFT_X, zero-filled IFFT_Y with the coil sum and the epilogue);
    otherwise dlcs_sense_normal (forward row pass, one fused FFT_Y / weights^2 /
    IFFT_Y column pass, adjoint row pass with the epilogue).  DLCS_SENSE_ROWS=0
    forces the latter."""
    B, E, T, Y, X = x.shape
    C = maps.shape[2]
    x = _c64(x).contiguous()
    m = _c64(maps).reshape(B, E, C, Y, X).contiguous()
    w, wc = _weights_arg(weights, B, C, T, Y, X)
    out = torch.empty_like(x)
    if sub is not None:
        sub = _c64(sub).contiguous()
    if (w is not None and _rows_enabled() and Y in _FAST_LEN and X in _FAST_LEN and E <= 2):
        tab, jmax, lines = _rowtab(weights, w, wc, B, T, Y, X)
        jcap, lines = _jcap(jmax, Y), _lines(lines, B, wc, T, Y)
        nb = int(_lib.lib().dlcs_sense_rows_workspace_bytes(B, C, T, jcap, X))
        ws = torch.empty((nb + 7) // 8, dtype=torch.complex64, device=x.device)
        # algorithmic bytes: x, A^H y, out, maps once; the sampled weight lines
        nbytes = (x.numel() * (2 + (sub is not None)) + m.numel()) * 8 + lines * X * 4
        _timed_call("dlcs_sense_normal_rows", nbytes, 2 * _call_bytes(B, E, C, T, Y, X),
                    _lib.ptr(x), _lib.ptr(m), _lib.ptr(w), wc, _lib.ptr(tab),
                    jcap, _lib.ptr(out), _lib.ptr(sub), float(base_scale), float(step), B, E, C, T, Y, X,
                    _lib.ptr(ws), ws.numel() * 8, _lib.stream())
        return out
    ws = _workspace(B, C, T, Y, X, x.device)
    nbytes = (x.numel() * (2 + (sub is not None)) + m.numel()) * 8 + (w.numel() * 4 if w is not None else 0)
    _timed_call("dlcs_sense_normal", nbytes, 2 * _call_bytes(B, E, C, T, Y, X),
                _lib.ptr(x), _lib.ptr(m), _lib.ptr(w), wc, _lib.ptr(out),
                _lib.ptr(sub), float(base_scale), float(step), B, E, C, T, Y, X,
                _lib.ptr(ws), ws.numel() * 8, _lib.stream())
    return out


class _NormalDCFn(torch.autograd.Function):
    """out = x + s * (A^H A x - ATy), the PGD data-consistency update (urs:109),
    as one dlcs_sense_normal call.  A^H A is Hermitian, so d out / d x applied
    to g is g + s * A^H A g (the same call with sub = 0)."""

    @staticmethod
    def forward(ctx, x, aty, step, maps, weights):
        s = float(step)
        ctx.s = s
        # the weights object itself (never requires grad): its cached row table is keyed by it
        ctx.weights = weights
        ctx.save_for_backward(maps)
        return sense_normal_raw(x, maps, weights, sub=aty, base_scale=1.0, step=s)

    @staticmethod
    def backward(ctx, g):
        (maps,), weights = ctx.saved_tensors, ctx.weights
        g = g.contiguous()
        gx = None
        if ctx.needs_input_grad[0]:
            gx = sense_normal_raw(g, maps, weights, sub=None, base_scale=1.0, step=ctx.s)
        gaty = -ctx.s * g if ctx.needs_input_grad[1] else None
        return gx, gaty, None, None, None


def normal_dc(x, aty, step, maps, weights):
    return _NormalDCFn.apply(x, aty, step, maps, weights)


class _NormalFn(torch.autograd.Function):
    """(A^H A + lamda I) m with a fixed lamda (HQS, urs:151); self-adjoint, so
    the backward is the same operator on the incoming gradient."""

    @staticmethod
    def forward(ctx, m, lamda, maps, weights):
        ctx.lamda = float(lamda)
        ctx.weights = weights
        ctx.save_for_backward(maps)
        return sense_normal_raw(m, maps, weights, base_scale=ctx.lamda, step=1.0)

    @staticmethod
    def backward(ctx, g):
        (maps,), weights = ctx.saved_tensors, ctx.weights
        return sense_normal_raw(g.contiguous(), maps, weights, base_scale=ctx.lamda, step=1.0), None, None, None


def sense_cg_raw(x, b, maps, weights, lamda, num_iter):
    """num_iter CG steps on (A^H A + lamda I) x = b from x (alg:50-73), every
    scalar on the device (dlcs_sense_cg); returns a new tensor."""
    B, E, T, Y, X = x.shape
    C = maps.shape[2]
    out = _c64(x).contiguous().clone()
    b = _c64(b).contiguous()
    m = _c64(maps).reshape(B, E, C, Y, X).contiguous()
    w, wc = _weights_arg(weights, B, C, T, Y, X)
    nb = int(_lib.lib().dlcs_sense_cg_workspace_bytes(B, E, C, T, Y, X))
    ws = torch.empty((nb + 7) // 8, dtype=torch.float64, device=x.device)
    if w is not None and _rows_enabled() and Y in _FAST_LEN and X in _FAST_LEN and E <= 2:
        tab, jmax, _ = _rowtab(weights, w, wc, B, T, Y, X)
        _lib.call("dlcs_sense_cg_rows", _lib.ptr(out), _lib.ptr(b), _lib.ptr(m), _lib.ptr(w), wc, _lib.ptr(tab),
                  _jcap(jmax, Y), float(lamda), int(num_iter), B, E, C, T, Y, X, _lib.ptr(ws), ws.numel() * 8,
                  _lib.stream())
        return out
    _lib.call("dlcs_sense_cg", _lib.ptr(out), _lib.ptr(b), _lib.ptr(m), _lib.ptr(w), wc, float(lamda),
              int(num_iter), B, E, C, T, Y, X, _lib.ptr(ws), ws.numel() * 8, _lib.stream())
    return out


class FFT(nn.Module):
    """tr:12-46 -- N-D FFT over the last ``ndims`` dims, orthonormal by default.
    The HIP path covers ndims == 2 with norm 'ortho' (what SenseModel uses)."""

    def __init__(self, ndims: int, norm: Optional[str] = "ortho") -> None:
        super().__init__()
        self.ndims = ndims
        self.norm = norm
        self.fft_dims = [i for i in range(-1, -1 - ndims, -1)]

    def forward(self, data: torch.Tensor, adjoint: Optional[bool] = False,
                centered: Optional[bool] = False):
        assert torch.is_complex(data)  # force complex (tr:33)
        if self.ndims != 2 or self.norm != "ortho":
            raise NotImplementedError("HIP FFT path: ndims=2, norm='ortho'")
        if _on_host(data):
            if centered:
                data = torch.fft.ifftshift(data, dim=self.fft_dims)
            out = _host_fft2(data, bool(adjoint))
            return torch.fft.fftshift(out, dim=self.fft_dims) if centered else out
        _lib.require_gpu(data)
        if centered:
            data = torch.fft.ifftshift(data, dim=self.fft_dims)
        out = _FFT2Fn.apply(data, bool(adjoint))
        if centered:
            out = torch.fft.fftshift(out, dim=self.fft_dims)
        return out


def fft2_raw(x, inverse):
    shp = x.shape
    Y, X = shp[-2], shp[-1]
    xc = _c64(x).contiguous()
    n = xc.numel() // (Y * X)
    out = torch.empty_like(xc)
    ws = torch.empty(xc.numel(), dtype=torch.complex64, device=x.device)
    _lib.call("dlcs_fft2", _lib.ptr(xc), _lib.ptr(out), n, Y, X, int(inverse),
              _lib.ptr(ws), ws.numel() * 8, _lib.stream())
    return out


class _FFT2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, inverse):
        ctx.inverse = inverse
        return fft2_raw(x, inverse)

    @staticmethod
    def backward(ctx, g):
        # unitary: the adjoint of the orthonormal FFT is its inverse
        return fft2_raw(g.contiguous(), not ctx.inverse), None


def _host_fft2(x, inverse):
    """Orthonormal uncentred 2-D FFT of CPU tensors over the last two dims."""
    return torch.fft.ifft2(x, norm="ortho") if inverse else torch.fft.fft2(x, norm="ortho")


def _host_forward(x, maps, weights):
    """CPU SENSE forward: y[b,c] = W * F2(sum_e S[b,e,c] x[b,e])."""
    k = _host_fft2(torch.einsum("betyx,becyx->bctyx", x, maps[:, :, :, 0]), False)
    return k if weights is None else k * weights


def _host_adjoint(y, maps, weights):
    """CPU SENSE adjoint: x[b,e] = sum_c conj(S[b,e,c]) F2^-1(W * y[b,c])."""
    img = _host_fft2(y if weights is None else y * weights, True)
    return torch.einsum("bctyx,becyx->betyx", img, maps[:, :, :, 0].conj())


def _on_host(*tensors):
    """True if every tensor is on the CPU, False if every one is on the GPU."""
    devs = {t.is_cuda for t in tensors if torch.is_tensor(t)}
    if len(devs) > 1:
        raise _lib.DlcsError("SenseModel / FFT operands must be all on the GPU or all on the CPU")
    return devs == {False}


class SenseModel(nn.Module):
    """tr:49-110 -- y = (W F S) x and x = (S^H F^H W) y.

    maps: complex64 [B, E, C, 1, Y, X]; weights: [B, 1, T, Y, X] mask (or
    [B, C, T, Y, X]) or None.  Keeps references to maps / weights (tr:73, :80-82).
    """

    def __init__(self, maps: torch.Tensor, weights: Optional[torch.Tensor] = None) -> None:
        super().__init__()
        assert torch.is_complex(maps)  # force complex (tr:70)
        self.maps = maps
        ndims = len(list(maps[0, 0, 0, ...].squeeze().shape))
        self.fft = FFT(ndims)
        self.weights = 1.0 if weights is None else weights

    def _w(self):
        return None if isinstance(self.weights, float) else self.weights

    def _adjoint_op(self, data):
        return _SenseAdjointFn.apply(data, self.maps, self._w())

    def _forward_op(self, data):
        return _SenseForwardFn.apply(data, self.maps, self._w())

    def normal_dc(self, x, aty, step):
        """Fused x + step * (A^H A x - aty)  (the PGD update, urs:109)."""
        _lib.require_gpu(x, aty, self.maps)
        return normal_dc(x, aty, step, self.maps, self._w())

    def normal(self, m, lamda):
        """(A^H A + lamda I) m with a fixed scalar lamda (HQS normal equations, urs:151)."""
        _lib.require_gpu(m, self.maps)
        return _NormalFn.apply(m, lamda, self.maps, self._w())

    def cg(self, x, b, lamda, num_iter):
        """ConjugateGradient(A^H A + lamda I, num_iter)(x, b) (alg:50-73) as one
        device-resident solve; no autograd (inference / no-grad callers)."""
        _lib.require_gpu(x, b, self.maps)
        return sense_cg_raw(x, b, self.maps, self._w(), lamda, num_iter)

    def forward(self, data: torch.Tensor, adjoint: Optional[bool] = False) -> torch.Tensor:
        assert torch.is_complex(data)  # tr:104
        if _on_host(data, self.maps, self._w()):
            op = _host_adjoint if adjoint else _host_forward
            return op(data, self.maps, self._w())
        _lib.require_gpu(data, self.maps)
        if adjoint:
            return self._adjoint_op(data)
        return self._forward_op(data)
