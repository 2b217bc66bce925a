"""§8(f) rows 2 and 4 on CPU: the auxiliary HDR gain map item (4:0:0, RExt
profile, WPP) through the host parser and the oracle, and the RGB
restatement's known answers.  The GPU halves are in tests/test_gpu.py."""
import numpy as np

import rgb_ref


def test_aux_item_found_by_host_and_oracle(halfmoonbay, oracle_mod):
    import heif_amd as H

    prim = H.HeifImage.parse(halfmoonbay).info
    assert prim.item_id == 49 and prim.primary_item_id == 49
    assert prim.aux_item_id == 52  # auxl 52 -> 49
    assert oracle_mod.aux_item(halfmoonbay) == 52


def test_aux_item_parameters(halfmoonbay):
    import heif_amd as H

    inf = H.HeifImage.parse(halfmoonbay, 52).info
    # hvcC (ipco 7): 2016x1520 coded, conformance window -> 2016x1512 (ispe 8), 4:0:0, 8-bit
    assert (inf.width, inf.height) == (2016, 1512)
    assert (inf.ispe_width, inf.ispe_height) == (2016, 1512)
    assert inf.chroma_format_idc == 0 and inf.bit_depth == 8
    assert inf.item_id == 52 and inf.num_tiles == 1 and inf.grid_rows == inf.grid_cols == 1
    assert inf.rotation == 3  # ipma: irot (ipco 5) is shared with the primary
    tp = H.HeifImage.parse(halfmoonbay, 52).tile_params(0)
    assert tp["general_profile_idc"] == 4 and tp["entropy_coding_sync"] == 1
    assert tp["pic_width"] == 2016 and tp["pic_height"] == 1520


def test_aux_item_oracle_decodes(halfmoonbay, oracle_mod):
    tiles, (ho, hl) = oracle_mod.list_tiles(halfmoonbay, 52)
    assert len(tiles) == 1
    o, n = tiles[0]
    y, _, _ = oracle_mod.decode_tile(halfmoonbay[ho:ho + hl], halfmoonbay[o:o + n], 2016, 1512)
    assert y.shape == (1512, 2016) and 0 < y.mean() < 255


def test_missing_item_rejected(halfmoonbay):
    import heif_amd as H

    try:
        H.HeifImage.parse(halfmoonbay, 999)
    except H.HeifGpuError as e:
        assert e.code == -2
    else:
        raise AssertionError("item 999 parsed")


def test_rgb_restatement_known_answers():
    y = np.array([[0, 128, 255, 16]], np.uint16)
    g = np.full((1, 2), 128, np.uint16)
    # full-range neutral chroma: R = G = B = Y
    out = rgb_ref.ycbcr_to_rgb(y, g, g, 6, True, 0)
    assert out[0, :, 0].tolist() == [0, 128, 255, 16] and (out[..., 0] == out[..., 1]).all()
    # limited range: Y 16 -> 0, Y 235 -> 255
    out = rgb_ref.ycbcr_to_rgb(np.array([[16, 235]], np.uint16), np.full((1, 1), 128, np.uint16),
                               np.full((1, 1), 128, np.uint16), 1, False, 0)
    assert out[0, :, 1].tolist() == [0, 255]
    # BT.601 full range: pure red (Y 76, Cb 85, Cr 255) comes back red
    out = rgb_ref.ycbcr_to_rgb(np.array([[76, 76]], np.uint16), np.array([[85]], np.uint16),
                               np.array([[255]], np.uint16), 6, True, 0)
    r, g_, b = out[0, 0]
    assert r >= 250 and g_ <= 5 and b <= 5


def test_rgb_restatement_rotation():
    y = np.arange(6, dtype=np.uint16).reshape(2, 3) * 40
    out = rgb_ref.ycbcr_to_rgb(y, None, None, 6, True, 1)
    assert out.shape == (3, 2, 3)
    # anticlockwise: the top-right sample becomes the top-left
    assert out[0, 0, 0] == y[0, 2] and out[2, 0, 0] == y[0, 0]
    assert rgb_ref.ycbcr_to_rgb(y, None, None, 6, True, 3)[0, 0, 0] == y[1, 0]


def test_nclx_colr_overrides_vui(halfmoonbay):
    """§8(f) row 1: an nclx colr (reference: heif/reader.rs:525 todo!()) sets
    the matrix / range used for RGB; without one the SPS VUI applies."""
    import heif_amd as H

    base = H.HeifImage.parse(halfmoonbay).info
    assert (base.matrix_coeffs, base.full_range) == (6, 1)  # VUI
    i = halfmoonbay.index(b"colrprof") + 4  # colour_type of the primary's ICC colr (548-byte box)
    patched = bytearray(halfmoonbay)
    patched[i:i + 11] = b"nclx" + bytes([0, 1, 0, 1, 0, 1, 0x00])  # BT.709 primaries/transfer/matrix, limited
    inf = H.HeifImage.parse(bytes(patched)).info
    assert (inf.matrix_coeffs, inf.full_range) == (1, 0)
