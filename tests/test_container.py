"""Host demux and parameter-set robustness.

Container variants the reference's reader gets wrong or leaves todo!()
(src/heif/reader.rs): items split over several iloc extents (:47 todo!),
infe version 0/1 entries (:303 todo!), unknown ipco properties ahead of the
known ones (:460-463 drops them, shifting every later ipma index), and 16-bit
ipma indices (:496-500 masks them with 0x7F).  Each variant of a synthetic
file must parse to the same image (info, tile payloads) and decode to the same
planes as the plain layout.

Then malformed inputs that must end in a clean HEIFGPU_E_PARSE /
HEIFGPU_E_UNSUPPORTED error instead of a wild host read or a device fault:
wrapping iloc offsets, conformance windows outside the picture, block-size
ladders and QPs outside their H.265 ranges, bit depths above 12.
"""
import hashlib

import numpy as np
import pytest

import ps_writer as W

S = pytest.importorskip("heif_amd.synth_encoder")
H = pytest.importorskip("heif_amd")

P = S.SynthParams(width=128, height=96)
LAYOUTS = {
    "multi_extent": S.BoxLayout(extents=3),
    "unknown_props_first": S.BoxLayout(unknown_props=3),
    "ipma_16bit_index_over_127": S.BoxLayout(unknown_props=200, ipma_16bit=True),
    "infe_v0_v1_items": S.BoxLayout(legacy_infe_items=2),
    "iloc_8byte_fields_base_offset": S.BoxLayout(offset_size=8, length_size=8, base_offset_size=8, base_offset=7),
    "everything": S.BoxLayout(extents=2, unknown_props=150, ipma_16bit=True, legacy_infe_items=3),
}


def _files(layout):
    return S.single_heic(P, 5, layout=layout), S.grid_heic(300, 200, P, 6, layout=layout)


def _digest(img):
    h = hashlib.sha256()
    for pl in (img.y, img.cb, img.cr):
        if pl is not None:
            h.update(np.ascontiguousarray(pl).astype("<u2").tobytes())
    return h.hexdigest()


@pytest.fixture(scope="module")
def plain():
    return _files(None)


def _info_tuple(img):
    i = img.info
    return (i.width, i.height, i.grid_rows, i.grid_cols, i.num_tiles, i.coded_bytes, i.bit_depth)


@pytest.mark.parametrize("name", list(LAYOUTS))
def test_layout_variant_parses_like_plain(plain, name):
    for want, got in zip(plain, _files(LAYOUTS[name])):
        a, b = H.HeifImage.parse(want), H.HeifImage.parse(got)
        assert _info_tuple(a) == _info_tuple(b), name
        for t in range(a.info.num_tiles):
            pa, pb = a.tile_params(t), b.tile_params(t)
            assert pa == pb, (name, t)


@pytest.mark.parametrize("name", list(LAYOUTS))
def test_layout_variant_oracle_planes_equal(oracle_mod, plain, name):
    for want, got in zip(plain, _files(LAYOUTS[name])):
        assert _digest(oracle_mod.decode_heic(got, with_checks=False)) == \
            _digest(oracle_mod.decode_heic(want, with_checks=False)), name


def test_ipma_16bit_index_is_not_masked():
    """Property 201 of ipco is the hvcC: a 0x7F mask (reader.rs:496-500) would
    point the tile at property 73, an unknown box."""
    d = S.single_heic(P, 5, layout=S.BoxLayout(unknown_props=200, ipma_16bit=True))
    assert H.HeifImage.parse(d).info.width == 128


# ------------------------------------------------------------------ malformed
def _assert_error(data, unsupported=False):
    with pytest.raises(H.HeifGpuError) as e:
        H.HeifImage.parse(data)
    assert isinstance(e.value, H.UnsupportedError) == unsupported, str(e.value)
    return str(e.value)


def test_iloc_offset_wrap_rejected():
    """offset 2^64-16, length 16+: offset + length wraps to a small number, so an
    unchecked sum would pass and read below the file buffer."""
    d = S.single_heic(P, 5, layout=S.BoxLayout(offset_size=8, length_size=8, first_extent_offset=(1 << 64) - 16))
    assert "out of bounds" in _assert_error(d)


def test_iloc_base_offset_wrap_rejected():
    """base_offset + extent_offset wrapping round 2^64 is rejected while parsing iloc."""
    d = S.single_heic(P, 5, layout=S.BoxLayout(offset_size=8, length_size=8, base_offset_size=8,
                                                base_offset=(1 << 64) - 8))
    assert "overflow" in _assert_error(d)


def _with_sets(sps=None, pps=None, p=P, nal=None):
    vps, s0, p0 = S.parameter_sets(p)
    return S.single_heic(p, 5, param_sets=(vps, sps or s0, pps or p0), nal=nal)


@pytest.mark.parametrize("conf", [(0, 0, 0, 48), (0, 0, 48, 0), (32, 32, 0, 0), (0, 0, 0, (1 << 31) - 1),
                                  ((1 << 32) - 2, 0, 0, 0)])
def test_conformance_window_outside_picture_rejected(conf):
    """7.4.3.2: SubWidthC * (left + right) < width (likewise vertically); huge
    ue values must not wrap into negative offsets (k_sao_out reads the crop
    window out of the reconstruction arena)."""
    assert "conformance" in _assert_error(_with_sets(sps=W.sps(conf=conf)))


def test_conformance_window_legal_crop_accepted():
    d = _with_sets(sps=W.sps(conf=(0, 3, 0, 1)))
    assert (H.HeifImage.parse(d).info.width, H.HeifImage.parse(d).info.height) == (122, 94)


@pytest.mark.parametrize("over", [
    dict(log2_min_tb_minus2=1),                    # MinTb (8) == MinCb (8)
    dict(log2_diff_max_min_tb=4),                  # MaxTb 64
    dict(log2_diff_max_min_cb=0),                  # CTB 8
    dict(log2_min_cb_minus3=3, log2_diff_max_min_cb=1),  # CTB 128
    dict(depth_intra=4),                           # deeper than CtbLog2 - MinTbLog2 (3)
    dict(log2_diff_max_min_cb=(1 << 32) - 2),      # ue that would wrap to -2 as int
    dict(width=100),                               # not a multiple of MinCbSize
    dict(width=0),
    dict(width=20000),                             # beyond the level 6.2 limit
    dict(pcm=(8, 8, 0, 3)),                        # Log2MaxIpcmCbSizeY 6 > Min(CtbLog2SizeY, 5)
    dict(log2_min_cb_minus3=1, log2_diff_max_min_cb=1, log2_diff_max_min_tb=2,
         pcm=(8, 8, 0, 1)),                        # Log2MinIpcmCbSizeY 3 < Min(MinCbLog2SizeY 4, 5) (7.4.3.2)
    dict(pcm=(9, 8, 0, 1)),                        # PCM luma bit depth above BitDepthY
])
def test_sps_out_of_range_rejected(over):
    _assert_error(_with_sets(sps=W.sps(**over)))


def test_valid_pcm_sps_accepted():
    """PCM enabled with legal sizes parses (PCM CUs decode: tests/test_synth.py pcm_* cases)."""
    d = _with_sets(sps=W.sps(log2_min_cb_minus3=1, log2_diff_max_min_cb=1, log2_diff_max_min_tb=2, pcm=(8, 8, 1, 0)))
    assert H.HeifImage.parse(d).info.width == 128


def test_bit_depth_above_12_is_unsupported():
    _assert_error(_with_sets(sps=W.sps(bit_depth=13)), unsupported=True)
    _assert_error(_with_sets(sps=W.sps(bit_depth=16)), unsupported=True)


def test_bit_depth_12_accepted():
    """Main 12 (no extended precision): 8..12-bit streams decode (tests/test_synth.py main12 cases)."""
    assert H.HeifImage.parse(_with_sets(sps=W.sps(bit_depth=12))).info.width == 128


@pytest.mark.parametrize("over", [dict(cb_qp_offset=13), dict(cr_qp_offset=-13), dict(diff_cu_qp_delta_depth=3),
                                  dict(beta=7), dict(tc=-7), dict(init_qp_minus26=26)])
def test_pps_out_of_range_rejected(over):
    _assert_error(_with_sets(pps=W.pps(**over)))


@pytest.mark.parametrize("delta", [30, -40])
def test_slice_qp_out_of_range_rejected(delta):
    """SliceQpY = 26 + init_qp_minus26 + slice_qp_delta outside [-QpBdOffsetY, 51]."""
    p = S.SynthParams(width=128, height=96, slice_qp_delta=delta)
    assert "SliceQpY" in _assert_error(S.single_heic(p, 5))


def test_valid_handwritten_sets_decode_on_oracle(oracle_mod):
    """The writer itself is sound: its default SPS/PPS equal the generator's
    semantics, so the generated picture decodes under them."""
    d = _with_sets(sps=W.sps(), pps=W.pps())
    img = oracle_mod.decode_heic(d)
    assert all(c["term_ok"] for c in img.checks)
    assert H.HeifImage.parse(d).info.width == 128


@pytest.mark.gpu
def test_gpu_layout_variants_bit_exact(oracle_mod, plain):
    """The variant containers through the whole GPU path, one batch, against
    the oracle's decode of the plain layout."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    datas = [f for name in ("everything", "multi_extent", "ipma_16bit_index_over_127") for f in _files(LAYOUTS[name])]
    want = [oracle_mod.decode_heic(f, with_checks=False) for f in plain] * 3
    ctx = H.DecodeContext(0)
    imgs = [H.HeifImage.parse(d) for d in datas]
    b = ctx.prepare(imgs)
    outs = ctx.alloc_outputs(imgs)
    b.decode_async(outs)
    assert not any(b.status())
    for k, (o, w) in enumerate(zip(outs, want)):
        for g, r in ((o.y, w.y), (o.cb, w.cb), (o.cr, w.cr)):
            assert np.array_equal(g.cpu().numpy().astype(np.uint16), r), k
    b.free()
    ctx.close()
