"""MRI tensor helpers (ut = dl_cs/mri/utils.py).  center_crop is on the hot
path (s3d:410) as a view; the others are data-preparation helpers (SURVEY 8(f)
rank 1, not yet ported to kernels) kept for API compatibility."""
import torch


def fftmod(out):
    """ut:7-19 -- multiply every other line by -1 (k-space modulation)."""
    out[..., ::2] *= -1
    out[..., ::2, :] *= -1
    out *= -1
    return out


def root_sum_of_squares(x, dim=0):
    return torch.sqrt(torch.sum(torch.abs(x) ** 2, dim=dim))


def get_mask(data, eps=1e-12):
    """ut:69-79"""
    assert torch.is_complex(data)
    return (torch.abs(data) > eps).to(torch.float32)


def time_average(data, dim, eps=1e-6, keepdim=True):
    """ut:29-34"""
    mask = get_mask(data)
    return data.sum(dim, keepdim=keepdim) / (mask.sum(dim, keepdim=keepdim) + eps)


def sliding_window(data, dim, window_size):
    """ut:37-49 -- circular sliding-window time average (view-sharing init)."""
    assert 0 < window_size <= data.shape[dim]
    windows = []
    for i in range(data.shape[dim]):
        data_slide = torch.roll(data, int(window_size / 2) - i, dim)
        windows.append(time_average(data_slide.narrow(dim, 0, window_size), dim))
    return torch.cat(windows, dim=dim)


def center_crop(data, shapes, dims):
    """ut:52-66"""
    for i, dim in enumerate(dims):
        assert 0 < shapes[i] <= data.shape[dim]
        idx_start = (data.shape[dim] - shapes[i]) // 2
        data = data.narrow(dim, idx_start, shapes[i])
    return data
