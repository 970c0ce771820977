"""The PRODUCT modules pinned directly to the reference goldens (CPU, no GPU
calls): the window clamping of dl_cs.models._window (vst:72-85), the
relative_position_index state_dict buffer of WindowAttention3D (vst:111-129,
a checkpoint-compatibility key) and dl_cs.utils.metrics (met:20-39, :121-125).
The oracle's own copies are pinned in test_oracle_*.py; these check the code
that ships."""
import numpy as np
import torch

from oracle import recipe


def test_product_get_window_size_cases(golden):
    from dl_cs.models._window import get_window_size
    for row in golden("windex")["get_window_size_cases"]:
        xs, w, s, a, b = (tuple(int(v) for v in row[i:i + 3]) for i in range(0, 15, 3))
        assert get_window_size(xs, w, s) == (a, b), (xs, w, s)
        assert get_window_size(xs, w) == a


def test_product_relative_position_index_buffer(golden):
    from dl_cs.models import video_swin_transformer_mri_downsample as vst
    wa = vst.WindowAttention3D(160, (7, 8, 8), 8, qkv_bias=True)
    buf = wa.state_dict()["relative_position_index"]
    assert buf.shape == (448, 448)
    np.testing.assert_array_equal(buf.numpy().astype(np.int64), golden("windex")["rpi_7x8x8"].astype(np.int64))
    # persistent: part of the checkpoint schema (vst:129)
    assert "relative_position_index" in dict(wa.named_buffers())


def test_product_metrics(golden):
    from dl_cs.utils import metrics
    g = golden("misc")
    ref = recipe.crandn(61, (1, 2, 4, 8, 8))
    pred = ref + 0.1 * recipe.crandn(62, (1, 2, 4, 8, 8))
    assert abs(float(metrics.l1(ref, pred)) - float(g["metric_l1"])) < 1e-6
    assert abs(float(metrics.l2(ref, pred)) - float(g["metric_l2"])) < 1e-6
    assert abs(float(metrics.psnr(ref, pred)) - float(g["metric_psnr"])) < 1e-4
    # LOSS_WEIGHT=False is the identity weighting
    assert float(metrics.l1(ref, pred, False)) == float(metrics.l1(ref, pred))
