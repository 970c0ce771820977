"""Cine preprocessing vs the reference's own outputs
(tests/golden/prep.npz, made by importing dl_cs.data.preprocess and
dl_cs.mri.{subsample,utils} of the reference): VDkt masks bit-exact, k-t helpers
and the full CinePreprocess (seeded by file name) on the CPU path here; the GPU
path (HIP kernels) is checked in tests/test_gpu_preprocess.py."""
import numpy as np
import pytest
import torch

from golden.make_golden import PREP_CASES, VDKT_CASES, prep_config, prep_inputs
from goldutil import nrmse


def test_vdkt_masks_bit_exact(golden):
    from dl_cs.mri import subsample as ss
    g = golden("prep")
    for i, (acc, pkx, pky, shape, seed) in enumerate(VDKT_CASES):
        m = ss.VDktMaskFunc(acc, sim_partial_kx=pkx, sim_partial_ky=pky)(shape, seed=seed if seed is not None else 0)
        bits = np.unpackbits(g[f"vdkt{i}_bits"])[:m.numel()]
        assert np.array_equal(bits, (m.numpy().reshape(-1) != 0).astype(np.uint8)), i


def test_vdkt_baseline_mask_bit_exact(golden):
    from dl_cs.mri import subsample as ss
    g = golden("misc")
    m = ss.VDktMaskFunc((10, 15), 0.25, 0.25)((1, 1, 20, 192, 160), seed=1000)
    bits = np.unpackbits(g["vdkt_seed1000_bits"])[:m.numel()]
    assert np.array_equal(bits, (m.numpy().reshape(-1) != 0).astype(np.uint8))
    assert float(m.sum()) == float(g["vdkt_seed1000_sum"])


def test_kt_helpers_host(golden):
    from dl_cs.mri import utils
    g = golden("prep")
    k = torch.from_numpy(g["ta_in"])
    assert nrmse(g["ta_out"], utils.time_average(k, dim=2).numpy()) < 1e-6
    for w in (1, 3, 5, 9):
        assert nrmse(g[f"slwin{w}_out"], utils.sliding_window(k, dim=2, window_size=w).numpy()) < 1e-6, w


@pytest.mark.parametrize("i", range(len(PREP_CASES)))
def test_cine_preprocess_host(golden, i):
    from dl_cs.data.preprocess import CinePreprocess
    g = golden("prep")
    C, T, Y, X, E, crop, zpad, slwin, fname = PREP_CASES[i]
    out = CinePreprocess(prep_config(crop, zpad, slwin), use_seed=True)(*prep_inputs(i, C, T, Y, X, E), fname)
    for name, v in zip(("kspace", "mask", "maps", "init", "scale", "target"), out):
        ref = g[f"prep{i}_{name}"]
        assert tuple(v.shape) == ref.shape, name
        if name == "mask":
            assert np.array_equal(v.numpy(), ref), name
        else:
            assert nrmse(ref, v.numpy()) < 1e-6, (name, nrmse(ref, v.numpy()))
