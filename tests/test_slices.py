"""Pictures of several slice segments (the reference reads only the first
segment of a picture: slice.rs:61-64 asserts first_slice_segment_in_pic_flag;
its slice-header grammar, slice.rs:44-204, is the anchor for the fields).

Oracle: spec-literal slices (oracle/hevc_decode.c decode_picture: segments in
tile scan from slice_segment_address, 9.3.1 context initialisation /
dependent-segment synchronisation, slice-bounded availability 6.4.1 and SAO
merge 7.3.8.3, qPY_PREV restart 8.6.1, per-slice deblocking parameters and
slice_loop_filter_across_slices_enabled_flag in 8.7.2 / 8.7.3).  Pinning: a
picture whose slices are bands of CTB rows with no loop filter across them
must equal its slices decoded as stand-alone pictures (tests/hevc_tiles.py
rewrites each segment's header), and the single-slice decode is pinned by the
reference's fixtures (test_oracle.py).  The generator and the oracle agreeing
on every substream end (the per-substream checks) pins context selection
for the other layouts (mid-row slices, dependent segments, slices with tiles).

GPU: each slice of such a picture is decoded as its own picture
(heif_amd/csrc/host/batch.cpp), its dependent segments back to back in it
(SP_ROW_SEGMENTS: one substream-table entry per CTB row, flagged where a
segment ends or, without WPP, where the engine runs on); when every slice is
filtered across its upper boundary (one set of deblocking values) the slices
are children of an assembly picture filtered whole (desc.hpp PD_ASSEMBLY).
A dependent segment starting inside a CTB row is decoded in place (count in
PicDesc.flags bits 16-30: the substream of its row switches to its data after
end_of_slice_segment_flag; with WPP each row's lane starts from a per-row
count of the earlier ones); independent slices starting inside a row,
filtering across some slice boundaries only and segments starting inside an
HEVC tile are HEIFGPU_E_UNSUPPORTED; slices of whole tiles decode as one
sub-picture per tile.
"""
import os
import subprocess

import numpy as np
import pytest

from hevc_tiles import _nal_units, assemble, split_slices
from conftest import make_emu

S = pytest.importorskip("heif_amd.synth_encoder")

# every layout the oracle decodes (128x96 / CTB 32 = 4 x 3 CTBs unless set)
PARSE_CASES = [
    ("rows_nowpp", dict(slice_ctus=4)),
    ("rows_wpp", dict(slice_ctus=4, wpp=1)),
    ("midrow_nowpp", dict(slice_ctus=5)),
    ("midrow_wpp", dict(slice_ctus=5, wpp=1)),
    ("dependent_nowpp", dict(slice_ctus=5, slice_dependent=1)),
    ("dependent_alt_wpp", dict(slice_ctus=3, wpp=1, slice_dependent=2)),
    ("across_mixed_dbk", dict(slice_ctus=3, wpp=1, slice_dependent=1, slice_lf_across=2, slice_dbk_vary=1)),
    ("tiles_and_slices", dict(slice_ctus=3, tile_cols=2, tile_rows=2)),
    ("tiles_slices_across", dict(slice_ctus=7, tile_cols=2, tile_rows=2, slice_dependent=2, slice_lf_across=2,
                                 tile_lf_across=1)),
    ("one_ctu_slices_10b", dict(slice_ctus=1, bit_depth=10, slice_dbk_vary=1)),
]

# bands of CTB rows, independent, nothing filtered across (the GPU's layouts)
ROW_CASES = [
    ("rows1_nowpp", dict(slice_ctus=4)),
    ("rows2_wpp_dbk", dict(slice_ctus=8, wpp=1, slice_dbk_vary=1)),
    ("crop_10b_wpp", dict(width=200, height=120, conf_right=6, conf_bottom=2, bit_depth=10, slice_ctus=7, wpp=1,
                          slice_dbk_vary=1)),
    ("ctb16_rows2", dict(log2_ctb=4, log2_max_tb=4, max_th_depth_intra=2, slice_ctus=16)),
    ("ctb64_partial_tools", dict(width=200, height=200, log2_ctb=6, bit_depth=10, slice_ctus=4, wpp=1,
                                 tq_bypass=1, transform_skip=1, scaling_list=1, diff_cu_qp_delta_depth=2,
                                 max_th_depth_intra=3)),
    ("mono_rows", dict(chroma_format=0, slice_ctus=4, wpp=1)),
    ("c422_rows_wpp", dict(chroma_format=2, slice_ctus=4, wpp=1)),
    ("c444_rows_10b", dict(chroma_format=3, bit_depth=10, slice_ctus=8)),
]

# dependent slice segments starting at CTB rows (GPU: a slice's segments back
# to back in one picture, one substream-table entry per row)
DEP_CASES = [
    ("dep_all_nowpp", dict(slice_ctus=4, slice_dependent=1)),
    ("dep_all_wpp", dict(slice_ctus=4, slice_dependent=1, wpp=1)),
    ("dep_alt_wpp", dict(slice_ctus=4, slice_dependent=2, wpp=1)),
    ("dep_alt_nowpp_ctb16_pcm", dict(log2_ctb=4, log2_max_tb=4, max_th_depth_intra=2, slice_ctus=8, slice_dependent=2,
                                     pcm=1, pcm_pct=20, pcm_log2_max=4)),
    ("dep_crop_10b_dbk", dict(width=200, height=120, conf_right=6, conf_bottom=2, bit_depth=10, slice_ctus=14,
                              slice_dependent=1, wpp=1, slice_dbk_vary=1)),
    ("dep_alt_across", dict(width=128, height=192, slice_ctus=4, slice_dependent=2, wpp=1, slice_lf_across=1)),
    # dependent segments starting inside CTB rows, no WPP (the slice's one
    # substream switches to the next segment's data after end_of_slice_segment_flag;
    # the lanes engine only: parse_mode_for makes such a batch a lanes parse
    # whatever mode is asked, so the solo / spread cases below run lanes too)
    ("dep_mid_nowpp", dict(slice_ctus=5, slice_dependent=1)),
    ("dep_mid_1ctu_10b", dict(slice_ctus=1, slice_dependent=1, bit_depth=10)),
    ("dep_mid_ctb16_pcm", dict(log2_ctb=4, log2_max_tb=4, max_th_depth_intra=2, slice_ctus=7, slice_dependent=1,
                               pcm=1, pcm_pct=20, pcm_log2_max=4)),
    ("dep_mid_c444_across", dict(chroma_format=3, width=160, height=96, slice_ctus=3, slice_dependent=1,
                                 slice_lf_across=1)),
    # with WPP: a segment starting inside a row continues that row's substream,
    # its entry points start the rows below; each row's lane starts counting the
    # mid-row segments from those of earlier rows (the tall one: 18 CTB rows, so
    # lanes take a second row of the picture)
    ("dep_mid_wpp", dict(slice_ctus=3, slice_dependent=1, wpp=1)),
    ("dep_mid_wpp_10b_dbk", dict(width=200, height=120, conf_right=6, conf_bottom=2, bit_depth=10, slice_ctus=5,
                                 slice_dependent=1, wpp=1, slice_dbk_vary=1)),
    ("dep_mid_wpp_ctb16_tall", dict(width=64, height=288, log2_ctb=4, log2_max_tb=4, max_th_depth_intra=2,
                                    slice_ctus=7, slice_dependent=1, wpp=1)),
    ("dep_mid_wpp_c422", dict(chroma_format=2, slice_ctus=6, slice_dependent=1, wpp=1)),
]


# slices of whole HEVC tiles (7.4.7.1's other option than tiles of whole slices):
# each tile a sub-picture with its own slice's header values (QP, SAO flags,
# deblocking), independent and dependent segments, with and without WPP;
# nothing filtered across tiles (256x192, CTB 32: 8x6 CTBs)
TILE_SLICE_CASES = [
    ("tile_per_slice_dbk", dict(width=256, height=192, tile_cols=2, tile_rows=2, slice_ctus=12, slice_dbk_vary=1)),
    ("two_tiles_per_slice_dep_wpp", dict(width=256, height=192, tile_cols=2, tile_rows=2, slice_ctus=24,
                                         slice_dependent=2, wpp=1)),
    ("cols4_dependent_10b", dict(width=256, height=192, tile_cols=4, tile_rows=1, slice_ctus=12, slice_dependent=1,
                                 bit_depth=10)),
]


def params(over):
    return S.SynthParams(**{**dict(width=128, height=96, wpp=0), **over})


def checks_ok(img):
    return all(c["term_ok"] and c["raw_start"] == c["raw_entry"] for c in img.checks)


@pytest.mark.parametrize("name,over", PARSE_CASES, ids=[c[0] for c in PARSE_CASES])
def test_oracle_decodes_slice_layouts(oracle_mod, name, over):
    """Every segment's substreams end exactly at their entry points, with
    end_of_slice_segment_flag on the segment's last CTU."""
    p = params(over)
    for seed in range(3):
        item = S.picture_item(p, seed)
        assert len(_nal_units(item)) > 1
        img = oracle_mod.decode_heic(S.single_heic(p, seed=seed))
        assert checks_ok(img), (name, seed)
        assert img.y.shape == (p.height - p.conf_bottom, p.width - p.conf_right)


def _split_decode(oracle_mod, p, item):
    def dec(sp):
        img = oracle_mod.decode_heic(S.single_heic(sp.params, nal=sp.nal))
        assert checks_ok(img)
        return img.y, img.cb, img.cr

    return assemble(p, split_slices(p, item), dec)


@pytest.mark.parametrize("name,over", ROW_CASES, ids=[c[0] for c in ROW_CASES])
def test_oracle_slices_equal_standalone_slices(oracle_mod, name, over):
    p = params(over)
    for seed in range(3):
        img = oracle_mod.decode_heic(S.single_heic(p, seed=seed))
        want = _split_decode(oracle_mod, p, S.picture_item(p, seed))
        for got, ref, c in zip((img.y, img.cb, img.cr), want, "YUV"):
            if ref is None:
                assert got is None
                continue
            assert got.shape == ref.shape, (name, seed, c)
            assert int((got != ref).sum()) == 0, (name, seed, c)


@pytest.mark.parametrize("across", [1, 2])
def test_oracle_slices_loop_filter_across(oracle_mod, across):
    """slice_loop_filter_across_slices_enabled_flag = 1 on every slice (1) or
    on the even-numbered ones (2): the decode differs from the stand-alone
    slices only within the loop filters' reach of a slice boundary whose lower
    slice has the flag, and does differ there."""
    base = dict(width=128, height=192, slice_ctus=4, wpp=1)  # 6 one-row slices
    p0, p1 = params(base), params({**base, "slice_lf_across": across})
    differs = 0
    for seed in range(3):
        img = oracle_mod.decode_heic(S.single_heic(p1, seed=seed))
        assert checks_ok(img)
        want = _split_decode(oracle_mod, p0, S.picture_item(p0, seed))
        for got, ref, sub in zip((img.y, img.cb, img.cr), want, (1, 2, 2)):
            near = np.zeros(ref.shape, bool)
            reach = 4 if sub == 1 else 2
            for k in range(1, 6):
                if across == 2 and k % 2:
                    continue  # odd-numbered slices keep their upper boundary unfiltered
                e = k * 32 // sub
                near[e - reach:e + reach, :] = True
            diff = got != ref
            assert not (diff & ~near).any(), seed
            differs += int(diff.sum())
    assert differs > 0


def test_synth_writes_segments():
    """slice_ctus splits the picture into segments of that many CTUs; a
    single-NAL request for a multi-segment picture is refused."""
    p = params(dict(slice_ctus=5))
    assert len(_nal_units(S.picture_item(p, 0))) == 3
    assert len(_nal_units(S.picture_item(params(dict()), 0))) == 1
    with pytest.raises(ValueError):
        S.picture(p, 0)


@pytest.mark.parametrize("over,why", [
    (dict(slice_ctus=5), "a slice segment starting inside a CTB row"),
    (dict(slice_ctus=5, slice_dependent=2, wpp=1), "a slice segment starting inside a CTB row"),
    (dict(slice_ctus=5, slice_dependent=2), "a slice segment starting inside a CTB row"),
    (dict(slice_ctus=4, slice_lf_across=2), "slices filtered across some slice boundaries only"),
    (dict(slice_ctus=4, slice_lf_across=1, slice_dbk_vary=1), "with different deblocking values"),
    (dict(slice_ctus=8, tile_cols=2, tile_rows=1), "several slice segments together with HEVC tiles"),
])
def test_host_rejects_unsupported_slice_layouts(over, why):
    import heif_amd as H

    with pytest.raises(H.UnsupportedError, match=why):
        H.HeifImage.parse(S.single_heic(params(over), seed=1))


@pytest.mark.parametrize("name,over", TILE_SLICE_CASES, ids=[c[0] for c in TILE_SLICE_CASES])
def test_oracle_and_host_take_slices_of_whole_tiles(oracle_mod, name, over):
    """Slices of whole tiles: every substream of every segment ends at its
    entry point in the oracle, and the host accepts the layout."""
    import heif_amd as H

    d = S.single_heic(params(over), seed=3)
    img = oracle_mod.decode_heic(d)
    assert img.checks and all(c["term_ok"] for c in img.checks), name
    H.HeifImage.parse(d)


def test_host_rejects_segments_out_of_order():
    import heif_amd as H
    import struct

    p = params(dict(slice_ctus=4))
    nals = _nal_units(S.picture_item(p, 3))
    swapped = b"".join(struct.pack(">I", len(n)) + n for n in (nals[1], nals[0], nals[2]))
    data = S.single_heic(p, seed=3, nal=None)
    good = S.picture_item(p, 3)
    assert good in data
    with pytest.raises(H.HeifGpuError) as e:
        H.HeifImage.parse(data.replace(good, swapped))
    assert not isinstance(e.value, H.UnsupportedError)


# ------------------------------------------------------------ kernel emulation
CSRC = os.path.join(os.path.dirname(__file__), "..", "heif_amd", "csrc")


@pytest.fixture(scope="module")
def emu_check():
    make_emu("emu-fast")
    return os.path.join(CSRC, "build", "emu_fast", "emu_check")


@pytest.mark.parametrize("parse", ["lanes", "solo", "spread"])
@pytest.mark.parametrize("name,across", [("rows2_wpp_dbk", 0), ("crop_10b_wpp", 0), ("ctb16_rows2", 0),
                                         ("ctb16_rows2", 1), ("mono_rows", 1), ("dep_all_nowpp", 0),
                                         ("dep_alt_wpp", 0), ("dep_alt_nowpp_ctb16_pcm", 0),
                                         ("dep_alt_across", 1), ("c422_rows_wpp", 1), ("c444_rows_10b", 0),
                                         ("dep_mid_nowpp", 0), ("dep_mid_1ctu_10b", 1), ("dep_mid_ctb16_pcm", 0),
                                         ("dep_mid_c444_across", 1), ("dep_mid_wpp", 0), ("dep_mid_wpp", 1),
                                         ("dep_mid_wpp_10b_dbk", 0), ("dep_mid_wpp_ctb16_tall", 0),
                                         ("dep_mid_wpp_c422", 1)])
def test_emulated_kernels_slices(emu_check, tmp_path, name, across, parse):
    """The kernels' source compiled for the host decodes a picture of row
    slices (one picture per slice, its dependent segments back to back;
    filtered across: children of an assembly) bit-exactly against the oracle."""
    p = params({**dict(ROW_CASES + DEP_CASES)[name], "slice_lf_across": across})
    path = tmp_path / "s.heic"
    path.write_bytes(S.single_heic(p, seed=5))
    r = subprocess.run([emu_check, str(path), "5"], capture_output=True, text=True, timeout=600,
                       env={**os.environ, "HEIFGPU_PARSE": parse})
    assert r.returncode == 0 and "EMU PARITY OK" in r.stdout + r.stderr, (r.stdout + r.stderr)[-2000:]


@pytest.mark.parametrize("parse", ["lanes", "solo", "spread"])
@pytest.mark.parametrize("name", [c[0] for c in TILE_SLICE_CASES])
def test_emulated_kernels_slices_of_tiles(emu_check, tmp_path, name, parse):
    """Slices of whole tiles through the kernels compiled for the host, bit-exact vs the oracle."""
    path = tmp_path / "t.heic"
    path.write_bytes(S.single_heic(params(dict(TILE_SLICE_CASES)[name]), seed=5))
    r = subprocess.run([emu_check, str(path), "5"], capture_output=True, text=True, timeout=600,
                       env={**os.environ, "HEIFGPU_PARSE": parse})
    assert r.returncode == 0 and "EMU PARITY OK" in r.stdout + r.stderr, (r.stdout + r.stderr)[-2000:]


# ------------------------------------------------------------------ GPU parity
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def H():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import heif_amd

    return heif_amd


def _planes(o):
    return [None if t is None else t.cpu().numpy().astype(np.uint16) for t in (o.y, o.cb, o.cr)]


def _assert_equal(got, img, tag):
    for g, r, c in zip(got, (img.y, img.cb, img.cr), "YUV"):
        if r is None:
            assert g is None, tag
            continue
        assert g.shape == r.shape, (tag, c)
        assert int((g != r).sum()) == 0, (tag, c)


@pytest.mark.gpu
@pytest.mark.parametrize("parse", ["lanes", "solo", "spread"])
def test_gpu_row_slices_bit_exact(H, oracle_mod, parse):
    """Every row-slice case, with and without filtering across slices, two
    seeds each, one batch per format, checked against the spec-literal
    oracle; plus a grid of sliced pictures batched with a tiled one."""
    ctx = H.DecodeContext(0)
    for depth, chroma in ((8, 1), (10, 1), (8, 0), (8, 2), (10, 3)):
        datas = []
        for name, over in ROW_CASES + DEP_CASES:
            for across in (0, 1):
                p = params({**over, "slice_lf_across": across})
                if across and p.slice_dbk_vary:
                    continue  # different deblocking values per slice: unsupported when filtered across
                if (p.bit_depth, p.chroma_format) == (depth, chroma):
                    datas += [S.single_heic(p, seed=s) for s in (1, 2)]
        if depth == 8 and chroma == 1:
            datas.append(S.grid_heic(700, 500, params(dict(width=256, height=256, slice_ctus=16, wpp=1)), seed=4))
            datas.append(S.single_heic(params(dict(width=256, height=128, tile_cols=2, tile_rows=2)), seed=4))
        imgs = [H.HeifImage.parse(d) for d in datas]
        b = ctx.prepare(imgs, parse=parse)
        outs = ctx.alloc_outputs(imgs)
        b.decode_async(outs)
        assert not any(b.status()), (depth, chroma)
        for k, (d, o) in enumerate(zip(datas, outs)):
            _assert_equal(_planes(o), oracle_mod.decode_heic(d, with_checks=False), (depth, chroma, k))
        b.free()
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("parse", ["lanes", "spread"])
def test_gpu_slices_of_tiles_bit_exact(H, oracle_mod, parse):
    """Slices of whole tiles on the GPU, two seeds per case, against the oracle."""
    ctx = H.DecodeContext(0)
    for depth in (8, 10):
        datas = [S.single_heic(params(over), seed=s) for _, over in TILE_SLICE_CASES
                 for s in (1, 2) if params(over).bit_depth == depth]
        imgs = [H.HeifImage.parse(d) for d in datas]
        b = ctx.prepare(imgs, parse=parse)
        outs = ctx.alloc_outputs(imgs)
        b.decode_async(outs)
        assert not any(b.status()), depth
        for k, (d, o) in enumerate(zip(datas, outs)):
            _assert_equal(_planes(o), oracle_mod.decode_heic(d, with_checks=False), (depth, k))
        b.free()
    ctx.close()
