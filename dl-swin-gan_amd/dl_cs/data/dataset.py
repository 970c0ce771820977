"""Slice datasets (ds = dl_cs/data/dataset.py of the reference, ds:14-55).

One example per slice of a per-patient file holding ``kspace`` [sl, C, T, Y, X],
``maps`` [sl, E, C, 1, Y, X] and ``target`` [sl, E, T, Y, X] (the layout
datasets/prepare_stage2.py:232-242 writes).  Hdf5Dataset reads the reference's
.h5 files (h5py is optional: it is imported on use); NpzDataset reads the same
three arrays from uncompressed .npz files (memory-mapped); SyntheticCineDataset
makes random fully-sampled slices of that layout for smoke runs and benchmarks.
Items are (kspace, maps, target, fname) passed through ``transform``."""
import glob
import os
import random

import numpy as np
from torch.utils.data import Dataset


class Hdf5Dataset(Dataset):
    def __init__(self, root_directory, transform, sample_rate=1.0):
        try:
            import h5py  # noqa: F401
        except ImportError as e:
            raise ImportError("Hdf5Dataset needs h5py; convert the files with "
                              "NpzDataset.from_arrays or use --data npz") from e
        self.transform = transform
        files = sorted(glob.glob(os.path.join(root_directory, '*.h5')))
        if sample_rate < 1.0:
            random.shuffle(files)
            files = sorted(files[:round(len(files) * sample_rate)])
        self.examples = []
        import h5py
        for fn in files:
            with h5py.File(fn, 'r') as f:
                self.examples += [(fn, s) for s in range(f['kspace'].shape[0])]

    def __len__(self):
        return len(self.examples)

    def __getitem__(self, index):
        import h5py
        fn, s = self.examples[index]
        with h5py.File(fn, 'r') as f:
            k, m, t = f['kspace'][s], f['maps'][s], f['target'][s]
        return self.transform(k, m, t, fn)


class NpzDataset(Dataset):
    def __init__(self, root_directory, transform, sample_rate=1.0):
        self.transform = transform
        files = sorted(glob.glob(os.path.join(root_directory, '*.npz')))
        if sample_rate < 1.0:
            random.shuffle(files)
            files = sorted(files[:round(len(files) * sample_rate)])
        self.examples = []
        for fn in files:
            with np.load(fn, mmap_mode='r') as z:
                self.examples += [(fn, s) for s in range(z['kspace'].shape[0])]

    @staticmethod
    def from_arrays(path, kspace, maps, target):
        np.savez(path, kspace=kspace.astype(np.complex64), maps=maps.astype(np.complex64),
                 target=target.astype(np.complex64))

    def __len__(self):
        return len(self.examples)

    def __getitem__(self, index):
        fn, s = self.examples[index]
        with np.load(fn, mmap_mode='r') as z:
            k, m, t = np.array(z['kspace'][s]), np.array(z['maps'][s]), np.array(z['target'][s])
        return self.transform(k, m, t, fn)


class SyntheticCineDataset(Dataset):
    """n random slices: x_true ~ CN(0, 1) [E, T, Y, X], maps normalised so
    sum_{e,c} |S|^2 = 1 per pixel, fully-sampled k-space = F(S x) (the bench
    slice, bench.py::make_slice)."""

    def __init__(self, n, transform, coils=8, emaps=2, frames=20, ny=192, nx=160, seed=1000):
        self.n, self.transform = n, transform
        self.shape = (coils, emaps, frames, ny, nx)
        self.seed = seed

    def __len__(self):
        return self.n

    def __getitem__(self, index):
        C, E, T, Y, X = self.shape
        rng = np.random.default_rng(self.seed + index)
        cn = lambda *s: (rng.standard_normal(s) + 1j * rng.standard_normal(s)).astype(np.complex64)
        x = cn(E, T, Y, X)
        maps = cn(E, C, 1, Y, X)
        maps /= np.sqrt((np.abs(maps) ** 2).sum(axis=(0, 1), keepdims=True))
        coil_img = np.einsum("etyx,ecyx->ctyx", x, maps[:, :, 0])
        k = (np.fft.fft2(coil_img, norm="ortho")).astype(np.complex64)
        return self.transform(k, maps, x, f"synthetic_{index:05d}.npz")
