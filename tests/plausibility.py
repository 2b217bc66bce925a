"""Independent plausibility metrics of a decoded halfmoonbay (parity of the
pixel stages is otherwise only GPU == oracle; the reference computes no pixels
and libheif is absent).

1. The HDR gain map (item 52) is a separately coded 4:0:0 stream of the same
   scene at half resolution.  A correct decode of both correlates strongly
   with the 2x2-mean-downsampled primary luma, over the image and per
   textured 512x512 tile; the same luma with its tiles permuted does not
   (negative control).  A wrong transform, prediction or loop filter in either
   decode destroys the correlation of the tiles it touches.
2. No CTB-aligned blocking or drift: the mean |horizontal / vertical luma
   step| across 32-sample CTB boundaries and 512-sample tile boundaries, over
   the mean step inside CTBs (excluding the 8x8 deblocking grid).
Values for the committed decode are in tests/golden/plausibility.json
(tools/make_plausibility.py).
"""
import numpy as np

from heif_amd.synthetic import permutation

THRESHOLDS = {"corr_min": 0.75, "tile_corr_min": 0.5, "control_abs_max": 0.1, "edge_ratio_max": 1.5}


def downsample2(y):
    h, w = y.shape
    return y[:h // 2 * 2, :w // 2 * 2].reshape(h // 2, 2, w // 2, 2).mean(axis=(1, 3))


def corr(a, b):
    return float(np.corrcoef(a.ravel(), b.ravel())[0, 1])


def permute_tiles(y, seed, rows=6, cols=8, t=512):
    out = np.zeros_like(y)
    p = permutation(rows * cols, seed)
    H, W = y.shape
    for k in range(rows * cols):
        r, c = divmod(k, cols)
        rr, cc = divmod(p[k], cols)
        h = min(t, H - t * r, H - t * rr)
        w = min(t, W - t * c, W - t * cc)
        out[t * r:t * r + h, t * c:t * c + w] = y[t * rr:t * rr + h, t * cc:t * cc + w]
    return out


def metrics(luma, gain):
    y = luma.astype(np.float64)
    g = gain.astype(np.float64)
    ds = downsample2(y)
    tile_corr = []
    for k in range(48):
        r, c = divmod(k, 8)
        a = ds[256 * r:256 * (r + 1), 256 * c:256 * (c + 1)]
        b = g[256 * r:256 * (r + 1), 256 * c:256 * (c + 1)]
        if a.std() > 1 and b.std() > 1:  # textured in both
            tile_corr.append(corr(a, b))
    gx = np.abs(np.diff(y, axis=1))
    gy = np.abs(np.diff(y, axis=0))
    cx = np.arange(gx.shape[1])
    ry = np.arange(gy.shape[0])
    inner_x = (cx % 32 != 31) & (cx % 8 != 7)
    inner_y = (ry % 32 != 31) & (ry % 8 != 7)
    return {
        "corr": corr(ds, g),
        "tile_corr_min": min(tile_corr),
        "textured_tiles": len(tile_corr),
        "control_corr": corr(downsample2(permute_tiles(y, 1)), g),
        "ctb_edge_ratio_x": float(gx[:, cx % 32 == 31].mean() / gx[:, inner_x].mean()),
        "ctb_edge_ratio_y": float(gy[ry % 32 == 31].mean() / gy[inner_y].mean()),
        "tile_edge_ratio_x": float(gx[:, cx % 512 == 511].mean() / gx[:, inner_x].mean()),
        "tile_edge_ratio_y": float(gy[ry % 512 == 511].mean() / gy[inner_y].mean()),
    }


def check(m):
    assert m["corr"] >= THRESHOLDS["corr_min"], m
    assert m["tile_corr_min"] >= THRESHOLDS["tile_corr_min"], m
    assert abs(m["control_corr"]) <= THRESHOLDS["control_abs_max"], m
    for k in ("ctb_edge_ratio_x", "ctb_edge_ratio_y", "tile_edge_ratio_x", "tile_edge_ratio_y"):
        assert m[k] <= THRESHOLDS["edge_ratio_max"], (k, m)
