"""GPU cine preprocessing (dlcs_crop_flip, dlcs_fft2,
dlcs_sense_adj, dlcs_cplx_mask_scale, dlcs_kt_window_average,
dlcs_kth_largest_abs) vs the reference's own CinePreprocess outputs
(tests/golden/prep.npz).  Tolerances: masks bit-exact; the rest NRMSE <= 1e-5
(fp32, a different FFT summation order); the scale (a selection, not a sum)
to 1e-6 relative."""
import numpy as np
import pytest
import torch

from golden.make_golden import PREP_CASES, prep_config, prep_inputs
from goldutil import nrmse

pytestmark = pytest.mark.gpu


def test_kt_helpers_gpu(golden):
    from dl_cs.mri import utils
    g = golden("prep")
    k = torch.from_numpy(g["ta_in"]).cuda()
    assert nrmse(g["ta_out"], utils.time_average(k, dim=2).cpu().numpy()) < 1e-6
    for w in (1, 3, 5, 9):
        assert nrmse(g[f"slwin{w}_out"], utils.sliding_window(k, dim=2, window_size=w).cpu().numpy()) < 1e-6, w


@pytest.mark.parametrize("n", [20, 1000, 61440, 300001])
def test_kth_largest_abs(n):
    from dl_cs.data.preprocess import percentile_scale
    g = torch.Generator().manual_seed(n)
    x = torch.complex(torch.randn(n, generator=g), torch.randn(n, generator=g))
    x[: n // 7] = 0                                     # ties at zero, like masked k-space
    ref = percentile_scale(x)
    got = percentile_scale(x.cuda())
    assert float(got) == float(ref)             # a selection: bit-exact


@pytest.mark.parametrize("i", range(len(PREP_CASES)))
def test_cine_preprocess_gpu(golden, i):
    from dl_cs.data.preprocess import CinePreprocess
    g = golden("prep")
    C, T, Y, X, E, crop, zpad, slwin, fname = PREP_CASES[i]
    out = CinePreprocess(prep_config(crop, zpad, slwin), use_seed=True, device="cuda")(
        *prep_inputs(i, C, T, Y, X, E), fname)
    for name, v in zip(("kspace", "mask", "maps", "init", "scale", "target"), out):
        assert v.is_cuda, name
        ref = g[f"prep{i}_{name}"]
        v = v.cpu().numpy()
        assert v.shape == ref.shape, name
        if name == "mask":
            assert np.array_equal(v, ref), name
        elif name == "scale":
            assert abs(float(v) - float(ref)) <= 1e-6 * abs(float(ref)), (float(v), float(ref))
        else:
            assert nrmse(ref, v) < 1e-5, (name, nrmse(ref, v))
