"""numpy restatement of the Swin window bookkeeping (TEST INFRASTRUCTURE).

All integer / bit-exact.  References are to
/root/reference/dl_cs/models/video_swin_transformer_mri_downsample.py ("vst").
"""
import numpy as np


def get_window_size(x_size, window_size, shift_size=None):
    """vst:72-85 -- clamp window (and zero shift) on every dim where x <= window."""
    ws = list(window_size)
    ss = list(shift_size) if shift_size is not None else None
    for i in range(len(x_size)):
        if x_size[i] <= window_size[i]:
            ws[i] = x_size[i]
            if ss is not None:
                ss[i] = 0
    if ss is None:
        return tuple(ws)
    return tuple(ws), tuple(ss)


def padded_grid(D, H, W, ws):
    """vst:221-226 -- pad (after LayerNorm) up to a multiple of the window."""
    return tuple(int(np.ceil(n / w)) * w for n, w in zip((D, H, W), ws))


def partition_src(B, D, H, W, ws, ss):
    """Row r of the windowed tensor [B*nW*N, C] reads token src[r] of [B*D*H*W, C].

    Combines the cyclic shift (torch.roll by -ss, vst:229) with window_partition
    (vst:41-52): window id = ((b*nD + iD)*nH + iH)*nW + iW, token id inside the
    window = (td*Wh + th)*Ww + tw.  src = -1 marks a zero pad row (vst:225).
    """
    Dp, Hp, Wp = padded_grid(D, H, W, ws)
    wd, wh, ww = ws
    nD, nH, nW = Dp // wd, Hp // wh, Wp // ww
    b, iD, iH, iW, td, th, tw = np.meshgrid(
        np.arange(B), np.arange(nD), np.arange(nH), np.arange(nW),
        np.arange(wd), np.arange(wh), np.arange(ww), indexing="ij")
    d = (iD * wd + td + ss[0]) % Dp
    h = (iH * wh + th + ss[1]) % Hp
    w = (iW * ww + tw + ss[2]) % Wp
    valid = (d < D) & (h < H) & (w < W)
    src = ((b * D + d) * H + h) * W + w
    src = np.where(valid, src, -1)
    return src.reshape(-1).astype(np.int64)


def reverse_dst(B, D, H, W, ws, ss):
    """Token t of the output [B*D*H*W, C] reads windowed row dst[t].

    window_reverse (vst:55-67) followed by torch.roll(+ss) (vst:243) and the
    crop back to (D, H, W) (vst:247-248): the inverse permutation of
    partition_src restricted to real tokens.
    """
    src = partition_src(B, D, H, W, ws, ss)
    dst = np.full(B * D * H * W, -1, dtype=np.int64)
    rows = np.nonzero(src >= 0)[0]
    dst[src[rows]] = rows
    return dst


def _region_labels(n, w, s):
    """Label of each coordinate along one dim, exactly as the three slices of
    compute_mask (vst:346-349) leave it: later slices overwrite earlier ones.
    slice(-w) -> 0, slice(-w, -s) -> 1, slice(-s, None) -> 2; with s == 0 the
    last slice is slice(0, None) (whole axis) and slice(-w, 0) is empty."""
    lab = np.zeros(n, dtype=np.int64)
    idx = np.arange(n)
    for k, sl in enumerate((slice(-w) if w else slice(0, 0), slice(-w, -s), slice(-s, None))):
        sel = np.zeros(n, dtype=bool)
        sel[idx[sl]] = True
        lab[sel] = k
    return lab


def region_labels(Dp, Hp, Wp, ws, ss):
    ld = _region_labels(Dp, ws[0], ss[0])
    lh = _region_labels(Hp, ws[1], ss[1])
    lw = _region_labels(Wp, ws[2], ss[2])
    return (ld[:, None, None] * 9 + lh[None, :, None] * 3 + lw[None, None, :])


def compute_mask(Dp, Hp, Wp, ws, ss):
    """vst:342-355 -> float32 [nW, N, N] with 0 where labels match, -100 elsewhere."""
    lab = region_labels(Dp, Hp, Wp, ws, ss)
    wd, wh, ww = ws
    lw_ = lab.reshape(Dp // wd, wd, Hp // wh, wh, Wp // ww, ww).transpose(0, 2, 4, 1, 3, 5)
    lw_ = lw_.reshape(-1, wd * wh * ww)
    diff = lw_[:, None, :] - lw_[:, :, None]
    return np.where(diff != 0, np.float32(-100.0), np.float32(0.0)).astype(np.float32)


def relative_position_index(ws):
    """vst:114-129 -- idx[i, j] = (dd+Wd-1)*(2Wh-1)*(2Ww-1) + (dh+Wh-1)*(2Ww-1) + (dw+Ww-1),
    d* = coord_i - coord_j, tokens numbered (d*Wh + h)*Ww + w."""
    wd, wh, ww = ws
    d, h, w = np.meshgrid(np.arange(wd), np.arange(wh), np.arange(ww), indexing="ij")
    c = np.stack([d.reshape(-1), h.reshape(-1), w.reshape(-1)])
    rel = c[:, :, None] - c[:, None, :]
    return ((rel[0] + wd - 1) * (2 * wh - 1) * (2 * ww - 1)
            + (rel[1] + wh - 1) * (2 * ww - 1) + (rel[2] + ww - 1)).astype(np.int64)
