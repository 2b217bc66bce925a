"""numpy restatement of heifgpu_ycbcr_to_rgb (test infrastructure).

H.273 YCbCr -> R'G'B' with the coefficients rounded to 16.16 fixed point
exactly as the library's color_coefs (heif_amd/csrc/kernels/kernels.hpp),
subsampled chroma (4:2:0, 4:2:2) by replication, then the irot rotation (anticlockwise, 90
degrees per unit; np.rot90 rotates anticlockwise).  The reference has no RGB
path (it parses `irot` and stops), so this restatement is the checker:
"parity unpinned" against libheif, which is not available here.
"""
import numpy as np


def coefs(matrix: int, full: bool):
    kr, kb = 0.299, 0.114
    if matrix == 1:
        kr, kb = 0.2126, 0.0722
    elif matrix == 9:
        kr, kb = 0.2627, 0.0593
    kg = 1.0 - kr - kb
    ys, cs = (1.0, 1.0) if full else (255.0 / 219.0, 255.0 / 224.0)

    def fx(v):
        return int(v * 65536.0 + 0.5)

    return dict(yoff=0 if full else 16, ys=fx(ys), cr_r=fx(2 * (1 - kr) * cs), cb_b=fx(2 * (1 - kb) * cs),
                cb_g=fx(2 * kb * (1 - kb) / kg * cs), cr_g=fx(2 * kr * (1 - kr) / kg * cs))


def ycbcr_to_rgb(y, cb, cr, matrix: int, full: bool, rotation: int, bit_depth: int = 8):
    c = coefs(matrix, full)
    sh = bit_depth - 8
    Y = (y.astype(np.int64) >> sh)
    if cb is None:
        Cb = Cr = np.zeros_like(Y)
    else:
        h, w = Y.shape
        sy, sx = int(cb.shape[0] < h), int(cb.shape[1] < w)  # 4:2:0 / 4:2:2 / 4:4:4 from the plane shape
        rows, cols = np.arange(h)[:, None] >> sy, np.arange(w)[None, :] >> sx
        Cb = (cb.astype(np.int64) >> sh)[rows, cols] - 128
        Cr = (cr.astype(np.int64) >> sh)[rows, cols] - 128
    yv = c["ys"] * (Y - c["yoff"])
    r = (yv + c["cr_r"] * Cr + 32768) >> 16
    g = (yv - c["cb_g"] * Cb - c["cr_g"] * Cr + 32768) >> 16
    b = (yv + c["cb_b"] * Cb + 32768) >> 16
    rgb = np.clip(np.stack([r, g, b], axis=-1), 0, 255).astype(np.uint8)
    return np.rot90(rgb, k=rotation & 3)
