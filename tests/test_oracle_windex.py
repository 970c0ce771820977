"""Oracle pin: integer window bookkeeping vs goldens from the reference (bit-exact)."""
import numpy as np
import pytest

from oracle import windex

GRIDS = [(7, 48, 40), (7, 48, 16), (7, 16, 16), (7, 8, 8), (7, 12, 10), (3, 16, 24), (8, 8, 8), (8, 48, 40)]
WINDOW = (7, 8, 8)


@pytest.mark.parametrize("grid", GRIDS)
def test_window_size_and_perms(golden, grid):
    g = golden("windex")
    tag = "%dx%dx%d" % grid
    ws, ss = windex.get_window_size(grid, WINDOW, (3, 4, 4))
    assert tuple(g[f"ws_{tag}"]) == ws
    assert tuple(g[f"ss_{tag}"]) == ss
    for shifted in (0, 1):
        s = ss if shifted else (0, 0, 0)
        src = windex.partition_src(1, *grid, ws, s)
        np.testing.assert_array_equal(src, g[f"part_{tag}_s{shifted}"])
        dst = windex.reverse_dst(1, *grid, ws, s)
        np.testing.assert_array_equal(dst, g[f"rev_{tag}_s{shifted}"])


@pytest.mark.parametrize("grid", GRIDS)
def test_compute_mask(golden, grid):
    g = golden("windex")
    tag = "%dx%dx%d" % grid
    ws, ss = windex.get_window_size(grid, WINDOW, (3, 4, 4))
    Dp, Hp, Wp = windex.padded_grid(*grid, ws)
    m = windex.compute_mask(Dp, Hp, Wp, ws, ss)
    assert tuple(m.shape) == tuple(g[f"maskshape_{tag}"])
    bits = np.packbits((m != 0).reshape(-1))
    np.testing.assert_array_equal(bits, g[f"mask_{tag}"])
    assert set(np.unique(m).tolist()) <= {0.0, -100.0}
    np.testing.assert_array_equal(np.unique(m), g[f"maskvals_{tag}"])


def test_relative_position_index(golden):
    g = golden("windex")
    idx = windex.relative_position_index(WINDOW)
    np.testing.assert_array_equal(idx, g["rpi_7x8x8"].astype(np.int64))
    assert idx.min() == 0 and idx.max() == (2 * 7 - 1) * (2 * 8 - 1) * (2 * 8 - 1) - 1


def test_get_window_size_cases(golden):
    for row in golden("windex")["get_window_size_cases"]:
        xs, w, s, a, b = (tuple(row[i:i + 3]) for i in range(0, 15, 3))
        assert windex.get_window_size(xs, w, s) == (a, b)


def test_baseline_grid_mask_counts():
    """30 windows at the BASELINE grid, 10 with a non-zero mask."""
    ws, ss = windex.get_window_size((7, 48, 40), WINDOW, (3, 4, 4))
    assert ss == (0, 4, 4)
    m = windex.compute_mask(7, 48, 40, ws, ss)
    assert m.shape == (30, 448, 448)
    assert int(((m != 0).reshape(30, -1).any(1)).sum()) == 10
