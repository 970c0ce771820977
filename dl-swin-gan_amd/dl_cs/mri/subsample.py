"""k-t undersampling masks (ss = dl_cs/mri/subsample.py of the reference).

VDktMaskFunc is the variable-density k-t sampling of the cine training data
(ss:65-254; config_swin.yaml UNDERSAMPLE: ACCELERATIONS (10, 15), PARTIAL_KX /
PARTIAL_KY 0.25).  It is a short sequential host algorithm (one numpy
RandomState draw per perturbed ky sample, a binary search over the
acceleration), so it runs on the host and its [1, 1, T, Y, X] float mask is
uploaded once; the per-voxel work that consumes it (mask multiply, time
averages, scaling) runs in the HIP preprocessing kernels (dl_cs.data.preprocess).

The sampling is restated step by step from the reference's description so the
random stream is consumed in the same order: the masks are bit-identical to the
reference's for the same seed (tests/test_preprocess.py against
tests/golden/misc.npz).
"""
from math import ceil, floor

import numpy as np
import torch

GOLDEN_RATIO = 0.618034


class MaskFunc:
    """ss:13-33 -- acceleration drawn uniformly from [lo, hi) per mask."""

    def __init__(self, accelerations):
        self.accelerations = accelerations
        self.rng = np.random.RandomState()

    def choose_acceleration(self):
        lo, hi = self.accelerations[0], self.accelerations[1]
        return lo + (hi - lo) * self.rng.rand()


def _vd_warp(pos, accel, degree):
    """Map normalised ky positions in [-1, 1] through the variable-density warp
    (denser near the centre): pos * (a |pos| + b)^degree with a = (f - 1) / f,
    b = 1 / f, f = accel^(1/degree)."""
    f = accel ** (1.0 / degree) if degree > 0 else accel
    a_coef, b_coef = (f - 1.0) / f, 1.0 / f
    return pos * (a_coef * np.abs(pos) + b_coef) ** degree


class VDktMaskFunc(MaskFunc):
    """ss:65-254 -- variable-density k-t mask (Peng Lai's scheme), optional
    partial readout (sim_partial_kx) and alternating partial-ky (sim_partial_ky)."""

    def __init__(self, accelerations, sim_partial_kx=0.25, sim_partial_ky=0.0):
        super().__init__(accelerations)
        self.sim_partial_kx = sim_partial_kx
        self.sim_partial_ky = sim_partial_ky
        self.golden_ratio = GOLDEN_RATIO

    def __call__(self, out_shape, seed=None):
        """out_shape (1, 1, T, Y, X) -> float32 mask of that shape."""
        self.rng.seed(seed)
        nkx, nky, nt = out_shape[4], out_shape[3], out_shape[2]
        accel = self.choose_acceleration()
        if self.sim_partial_ky > 0.0:
            kt = self.vdkt_partial_ky(nky, nt, accel, partialFourierFactor=self.sim_partial_ky)
        else:
            kt = self.vdkt(nky, nt, accel)
        if self.sim_partial_kx > 0.0:                 # partial echo: the first readout fraction unsampled
            kt = np.stack(nkx * [kt], axis=0)
            kt[:int(self.sim_partial_kx * nkx)] = 0
        return torch.from_numpy(kt.transpose(2, 1, 0).reshape(out_shape).astype(np.float32))

    def goldenratio_shift(self, accel, nt):
        return np.round(np.arange(0, nt) * self.golden_ratio * accel) % accel

    # -- one frame ------------------------------------------------------------
    def _frame_positions(self, shift, ny, accel, perturb, adhere):
        """Uniform ky lattice of one frame with random jitter; each jitter also
        drags the two neighbours by `adhere` of it.  Returns float positions."""
        ys = np.arange(shift, ny, accel)
        lo, hi = perturb * accel, ny - perturb * accel
        for n in range(ys.size if perturb > 0 else 0):
            if ys[n] < lo or ys[n] >= hi:
                continue
            d = perturb * accel * (self.rng.rand() - 0.5)
            ys[n] += d
            if n > 0:
                ys[n - 1] += adhere * d
            if n < ys.size - 1:
                ys[n + 1] += adhere * d
        return np.clip(ys, 0, ny - 1)

    @staticmethod
    def _place_upper(col, ys, idx, radius, ny):
        """Snap the non-negative half (sorted by |ky|) onto free grid lines going
        outwards; a collision moves to the next free edge line and re-scales the
        remaining positions into the space left (ss:173-188)."""
        scale, origin = 1.0, 0.0
        edge = floor(ys[idx[0]] * radius + radius + 0.0001)
        for n in range(idx.size):
            y = ys[idx[n]]
            loc = min(floor((origin + (y - origin) * scale) * radius + radius + 0.0001), ny - 1)
            if col[loc] == 0:
                col[loc] = 1
                edge = loc + 1
            else:
                col[edge] = 1
                origin = y
                scale = (radius - float(edge - radius)) / (radius * (1 - abs(origin)))
                edge += 1

    @staticmethod
    def _place_lower(col, ys, idx, radius):
        """The negative half, snapped going inwards-to-outwards downwards (ss:190-212)."""
        scale, origin = 1.0, 0.0
        edge = floor(ys[idx[0]] * radius + radius + 0.0001)
        if col[edge] == 1:
            edge -= 1
            origin = ys[idx[0]]
            scale = (radius + float(edge - radius)) / (radius * (1.0 - abs(origin)))
        for n in range(idx.size):
            y = ys[idx[n]]
            loc = max(floor((origin + (y - origin) * scale) * radius + radius + 0.0001), 0)
            if col[loc] == 0:
                col[loc] = 1
                edge = loc + 1
            else:
                col[edge] = 1
                origin = y
                scale = (radius - float(edge - radius)) / (radius * (1 - abs(origin)))
                edge -= 1

    def vdkt(self, ny, nt, accel, nCal=1, vdDegree=1.5, vdFactor=None, perturbFactor=0.4, adhereFactor=0.33):
        """[ny, nt] float32 k-t mask at `accel` (ss:118-214)."""
        degree = max(vdDegree, 0.0)
        perturb = min(max(perturbFactor, 0.0), 1.0)
        adhere = min(max(adhereFactor, 0.0), 1.0)
        ncal = max(nCal, 0)
        if vdFactor is None or vdFactor > accel:
            vdFactor = accel
        centre, radius = floor(ny / 2.0), (ny - 1) / 2.0
        kt = np.zeros([ny, nt], np.float32)
        shifts = self.goldenratio_shift(accel, nt)
        for t in range(nt):
            ys = self._frame_positions(shifts[t], ny, accel, perturb, adhere)
            ys = _vd_warp((ys - radius) / radius, vdFactor, degree)
            ys = ys[np.argsort(np.abs(ys))]
            col = kt[:, t]
            self._place_upper(col, ys, np.where(ys >= 0)[0], radius, ny)
            self._place_lower(col, ys, np.where(ys < 0)[0], radius)
        kt[(centre - ceil(ncal / 2)):(centre + ncal - 1 - ceil(ncal / 2)), :] = 1     # calibration lines
        return kt

    def vdkt_partial_ky(self, nky, nphases, tgt_accel, partialFourierFactor=0.25, tol=0.1, max_iter=10):
        """Binary search on the requested rate so that, after removing the
        alternating partial-Fourier ky band, the net rate hits tgt_accel (ss:216-254)."""
        lo, hi = 1.0, tgt_accel
        act, it, kt = 1.0, 0, None
        nband = int(nky * partialFourierFactor)
        while abs(act - tgt_accel) > tol and it < max_iter:
            guess = 0.5 * (lo + hi)
            kt = self.vdkt(nky, nphases, guess)
            kt[(nky - nband):nky, 0::2] = 0
            kt[0:nband, 1::2] = 0
            act = (nky * nphases) / np.sum(kt)
            if act < tgt_accel:
                lo = guess
            else:
                hi = guess
            it += 1
        return kt


def subsample(data, mask_func, seed=None, mode='2D'):
    """ss:257-283 -- (mask * data, mask); data [N, coils, (T,) Y, X]."""
    shape = tuple(data.shape)
    if mode == '2D':
        mshape = (1, 1) + shape[2:4]
    elif mode == '3D':
        mshape = (1, 1) + shape[2:5]
    else:
        raise ValueError('Only 2D and 3D undersampling masks are supported.')
    mask = mask_func(mshape, seed).to(data.device)
    return mask * data, mask
