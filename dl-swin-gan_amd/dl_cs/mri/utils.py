"""MRI tensor helpers (ut = dl_cs/mri/utils.py of the reference).

center_crop is on the hot path (s3d:410) as a view.  The k-t helpers used by
the cine preprocessing (time_average, sliding_window) run
as HIP kernels for GPU tensors (dlcs_kt_window_average, prep.hip) and as
vectorised torch code for CPU tensors (DataLoader workers).
"""
import torch

from .. import _lib


def fftmod(out):
    """ut:7-19 -- in-place k-space modulation: the reference flips the sign of
    even columns, then even rows, then everything, i.e. multiplies pixel (y, x)
    by -(-1)^(y + x)."""
    Y, X = out.shape[-2], out.shape[-1]
    iy = torch.arange(Y, device=out.device).view(Y, 1)
    ix = torch.arange(X, device=out.device).view(1, X)
    sign = (((iy + ix) % 2) * 2 - 1).to(out.real.dtype if torch.is_complex(out) else out.dtype)
    out.mul_(sign)
    return out


def root_sum_of_squares(x, dim=0):
    """ut:22-26"""
    return torch.linalg.vector_norm(x, dim=dim)


def get_mask(data, eps=1e-12):
    """ut:69-79 -- 1 where |data| > eps."""
    assert torch.is_complex(data)
    return (torch.abs(data) > eps).to(torch.float32)


def _kt_kernel_ok(data, dim):
    return data.is_cuda and torch.is_complex(data) and data.dim() == 5 and dim in (2, -3)


def _kt_kernel(data, window, full):
    B, C, T, Y, X = data.shape
    x = data.to(torch.complex64).contiguous()
    out = torch.empty((B, C, 1 if full else T, Y, X), dtype=torch.complex64, device=data.device)
    _lib.call("dlcs_kt_window_average", _lib.ptr(x), _lib.ptr(out), B * C, T, Y * X, window, int(full),
              _lib.stream())
    return out


def time_average(data, dim, eps=1e-6, keepdim=True):
    """ut:29-34 -- sum over `dim` / (number of sampled entries + eps)."""
    if _kt_kernel_ok(data, dim) and keepdim and eps == 1e-6:
        return _kt_kernel(data, data.shape[dim], True)
    count = get_mask(data).sum(dim, keepdim=keepdim)
    return data.sum(dim, keepdim=keepdim) / (count + eps)


def sliding_window(data, dim, window_size):
    """ut:37-49 -- circular sliding-window time average: frame t averages frames
    (t - window_size // 2 + j) mod T, j < window_size (the view-sharing
    initial guess, preprocess.py:160-164)."""
    T = data.shape[dim]
    assert 0 < window_size <= T
    if _kt_kernel_ok(data, dim):
        return _kt_kernel(data, window_size, False)
    d = dim % data.dim()
    idx = (torch.arange(T).view(T, 1) - window_size // 2 + torch.arange(window_size).view(1, window_size)) % T
    win = data.index_select(d, idx.reshape(-1).to(data.device))
    win = win.reshape(data.shape[:d] + (T, window_size) + data.shape[d + 1:])
    count = get_mask(win).sum(d + 1)
    return win.sum(d + 1) / (count + 1e-6)


def center_crop(data, shapes, dims):
    """ut:52-66 -- centred crop along `dims` (a view)."""
    for size, dim in zip(shapes, dims):
        n = data.shape[dim]
        assert 0 < size <= n
        data = data.narrow(dim, (n - size) // 2, size)
    return data
