"""Cine preprocessing (pp = dl_cs/data/preprocess.py of the reference; SURVEY
8(f) rank 1).

CinePreprocess turns one fully-sampled slice (k-space [C, T, Y, X], ESPIRiT maps
[E, C, 1, Y, X], target [E, T, Y, X]) into the training tuple
(masked k-space, mask, maps, initial image, scale, target) exactly as the
reference does: FFT-domain crop / flip augmentation, SENSE-adjoint target,
VDkt undersampling, 95th-percentile scaling from the time-averaged image, and
the sliding-window initial guess (pp:54-180).

With device='cuda' every per-voxel step runs on the GPU through libdlcs_hip --
dlcs_fft2 (augmentation round trip), dlcs_crop_flip, dlcs_sense_adj (target,
scale image, initial guess), dlcs_cplx_mask_scale, dlcs_kt_window_average,
dlcs_kth_largest_abs -- and the scale never leaves the device.  The host keeps
only the random choices (crop centres, flips, the VDkt mask), drawn from the
same numpy RandomState stream in the same order as the reference, so a seeded
call (use_seed=True: seed = the file name's characters) reproduces the
reference's output.  With device=None the same steps run on CPU tensors (the
reference's DataLoader-worker placement).
"""
import numpy as np
import torch

from .. import _lib
from ..mri import subsample as ss
from ..mri import transforms as T
from ..mri import utils


class Preprocess:
    """pp:11-28 -- abstract preprocessing module."""

    def __init__(self, config, use_seed=False):
        self.config = config
        self.use_seed = use_seed
        self.rng = np.random.RandomState()

    def _augment(self, kspace, maps, target, seed):
        raise ValueError('Not implemented for abstract data class!')

    def __call__(self, kspace, maps, target, fname):
        raise ValueError('Not implemented for abstract data class!')


def _crop_flip(x, y0, ny, x0, nx, flip_t, flip_y, flip_x, has_t=True):
    """Crop the last two dims to [y0, y0+ny) x [x0, x0+nx), then flip t (dim -3,
    when has_t) / y / x."""
    if x.is_cuda:
        Y, X = x.shape[-2], x.shape[-1]
        Tn = x.shape[-3] if has_t else 1
        P = x.numel() // (Tn * Y * X)
        src = x.to(torch.complex64).contiguous()
        out = torch.empty(x.shape[:-2] + (ny, nx), dtype=torch.complex64, device=x.device)
        _lib.call("dlcs_crop_flip", _lib.ptr(src), _lib.ptr(out), P, Tn, Y, X, y0, ny, x0, nx,
                  int(bool(flip_t and has_t)), int(bool(flip_y)), int(bool(flip_x)), _lib.stream())
        return out
    out = x[..., y0:y0 + ny, x0:x0 + nx]
    dims = [d for d, f in ((-3, flip_t and has_t), (-2, flip_y), (-1, flip_x)) if f]
    return torch.flip(out, dims=dims) if dims else out.clone()


def _mask_scale(x, mask=None, scale=None, divide=True):
    """x * mask (broadcast over coils) and / scale (a 0-d tensor on x's device)."""
    if x.is_cuda:
        xc = x.contiguous()
        y = torch.empty_like(xc)
        TYX = x.shape[-3] * x.shape[-2] * x.shape[-1]
        P = x.numel() // TYX
        m = mask.to(torch.float32).contiguous() if mask is not None else None
        mp = (m.numel() // TYX) if m is not None else 0
        _lib.call("dlcs_cplx_mask_scale", _lib.ptr(xc), _lib.ptr(m), _lib.ptr(y), P, TYX, mp,
                  _lib.ptr(scale), int(divide), _lib.stream())
        return y
    y = x * mask if mask is not None else x
    if scale is not None:
        y = y / scale if divide else y * scale
    return y


def percentile_scale(image, frac=0.05):
    """min(topk(|image|, round(frac * numel))) -- the 95th-percentile magnitude
    (pp:149-153) -- as a 0-d tensor on image's device."""
    n = image.numel()
    k = int(round(frac * n))
    if image.is_cuda:
        x = image.to(torch.complex64).contiguous()
        out = torch.empty((), dtype=torch.float32, device=image.device)
        _lib.call("dlcs_kth_largest_abs", _lib.ptr(x), n, k, _lib.ptr(out), _lib.stream())
        return out
    return torch.min(torch.topk(torch.abs(image).reshape(-1), k).values)


class CinePreprocess(Preprocess):
    """pp:31-180 -- training-time cine preprocessing (augment, simulate
    undersampling, normalise, sliding-window initial guess)."""

    def __init__(self, config, lr_decom=False, use_seed=False, device=None):
        super().__init__(config, use_seed)
        if lr_decom:
            raise NotImplementedError("DSLR low-rank decomposition is not on the Swin path")
        us = config.AUG_TRAIN.UNDERSAMPLE
        self.mask_func = ss.VDktMaskFunc(us.ACCELERATIONS, sim_partial_kx=us.PARTIAL_KX,
                                         sim_partial_ky=us.PARTIAL_KY)
        self.device = torch.device(device) if device is not None else None

    def _crop_window(self, n, size):
        """Random crop start along an axis of length n (pp:61-74 / :86-99)."""
        centre = int(self.rng.normal(loc=n // 2 + 1, scale=size // 2))
        centre = int(np.clip(centre, a_min=size // 2, a_max=n - size // 2 - 1))
        return centre - size // 2 + 1

    def _augment(self, kspace, maps, target, seed):
        """pp:54-126 -- crop along readout / phase encode and random flips, applied
        to the multicoil images (IFFT of k-space) and maps / target alike."""
        self.rng.seed(seed)
        F = T.FFT(ndims=2)
        images = F(kspace, adjoint=True)
        Y, X = images.shape[-2], images.shape[-1]
        y0, ny, x0, nx = 0, Y, 0, X
        crop_x = self.config.AUG_TRAIN.CROP_READOUT
        if crop_x > 0:
            x0, nx = self._crop_window(X, crop_x), crop_x
        crop_y = self.config.AUG_TRAIN.ZPAD_PE
        if crop_y > 0:
            y0, ny = self._crop_window(Y, crop_y), crop_y
        fx = self.rng.rand() > 0.5
        fy = self.rng.rand() > 0.5
        ft = self.rng.rand() > 0.5
        images = _crop_flip(images, y0, ny, x0, nx, ft, fy, fx)
        maps = _crop_flip(maps, y0, ny, x0, nx, False, fy, fx, has_t=False)
        target = _crop_flip(target, y0, ny, x0, nx, ft, fy, fx)
        return F(images), maps, target

    def _to(self, a):
        t = a if torch.is_tensor(a) else torch.from_numpy(np.ascontiguousarray(a))
        return t.to(self.device) if self.device is not None else t

    def __call__(self, kspace, maps, target, fname):
        seed = tuple(map(ord, fname)) if self.use_seed else None
        kspace = self._to(kspace).unsqueeze(0)
        maps = self._to(maps).unsqueeze(0)
        target = self._to(target).unsqueeze(0)
        kspace, maps, target = self._augment(kspace, maps, target, seed)
        A = T.SenseModel(maps, weights=None)
        target = A(kspace, adjoint=True)                                    # pp:143
        mask = self.mask_func((1, 1) + tuple(kspace.shape[2:5]), seed).to(kspace.device)   # pp:146
        masked = _mask_scale(kspace, mask)
        image = A(utils.time_average(masked, dim=2), adjoint=True)          # pp:149-151
        scale = percentile_scale(image)                                     # pp:152-153
        masked = _mask_scale(masked, scale=scale)                           # pp:156-157
        target = _mask_scale(target, scale=scale)
        init = utils.sliding_window(masked, dim=2, window_size=5) if self.config.MODEL.PARAMETERS.SLWIN_INIT \
            else masked                                                     # pp:160-163
        init_image = A(init, adjoint=True)
        return masked[0], mask[0], maps[0], init_image[0], scale, target[0]


class DataTransform:
    """Inference preprocessing of fully- or under-sampled acquired k-space
    (reconstruct.py:114-152): mask from the data, fftmod, 95th-percentile scale,
    sliding-window initial guess.  Returns (kspace, maps, mask, init, scale)."""

    def __init__(self, config, device=None, fftmod=True, acceleration=1):
        """fftmod=False, acceleration: the H5 inference transforms (reconstruct_h5.py
        DataTransform :263-312 for acceleration 1, DataTransformSS :314-368 -- a
        VDkt k-t mask at (acceleration, acceleration) with the config's partial
        kx / ky, seed 1000, applied to fully-sampled data -- neither fftmods)."""
        self.slwin_init = config.MODEL.PARAMETERS.SLWIN_INIT
        self.device = torch.device(device) if device is not None else None
        self.fftmod = fftmod
        self.mask_func = None
        if acceleration > 1:
            from ..mri import subsample as ss
            U = config.AUG_TRAIN.UNDERSAMPLE
            self.mask_func = ss.VDktMaskFunc((acceleration, acceleration), sim_partial_kx=U.PARTIAL_KX,
                                             sim_partial_ky=U.PARTIAL_KY)

    def __call__(self, kspace, maps):
        to = lambda a: (a if torch.is_tensor(a) else torch.from_numpy(np.ascontiguousarray(a)))
        kspace = to(kspace).unsqueeze(0)
        maps = to(maps).unsqueeze(0)
        if self.device is not None:
            kspace, maps = kspace.to(self.device), maps.to(self.device)
        if self.mask_func is not None:
            from ..mri import subsample as ss
            kspace, mask = ss.subsample(kspace, self.mask_func, seed=1000, mode='3D')      # rh5:336
        else:
            mask = utils.get_mask(kspace)[:, 0:1]
        if self.fftmod:
            kspace = utils.fftmod(kspace.clone())
            maps = utils.fftmod(maps.clone())
        A = T.SenseModel(maps, weights=None)
        scale = percentile_scale(A(utils.time_average(kspace, dim=2), adjoint=True))
        kspace = _mask_scale(kspace, scale=scale)
        init = utils.sliding_window(kspace, dim=2, window_size=5) if self.slwin_init else kspace
        return kspace[0], maps[0], mask[0], A(init, adjoint=True)[0], scale
