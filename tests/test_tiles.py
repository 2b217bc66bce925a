"""HEVC tiles inside a picture (tiles_enabled_flag = 1; the reference parses
the PPS tile syntax at parameter_set_reader.rs:380-408 and reads entry points
for tiles at slice.rs:155-171, but its slice-data loop assumes no tiles,
slice.rs:207).

Oracle: spec-literal tiles (oracle/hevc_decode.c: tile scan 6.5.1, per-tile
CABAC initialisation 9.3.1, tile-bounded availability 6.4.1 / SAO merge
7.3.8.3, qPY_PREV restart 8.6.1, loop filters across tiles 8.7).  Pinning:
with loop_filter_across_tiles_enabled_flag = 0 a tiled picture must equal its
tiles decoded as stand-alone pictures (tests/hevc_tiles.py cuts them out of
the bitstream), and the untiled decode is pinned by the reference's fixtures
(test_oracle.py).  With the flag = 1 the two may differ only within the loop
filters' reach of a tile boundary.

GPU: the host decodes a tiled picture as one picture per tile
(heif_amd/csrc/host/batch.cpp); with loop_filter_across_tiles = 1 the tiles
are children of an assembly picture that k_assemble puts together before the
loop filters run on it whole (desc.hpp PD_ASSEMBLY).  Tiles together with WPP:
each tile is a WPP picture whose substreams are the tile's CTB rows.
"""
import os
import subprocess

import numpy as np
import pytest

from hevc_tiles import assemble, split_tiles
from conftest import make_emu

S = pytest.importorskip("heif_amd.synth_encoder")

# (name, overrides): uniform / explicit spacing, one row or column of tiles,
# partial CTBs and a conformance crop in the edge tiles, CTB 16 / 64, 10-bit,
# 4:0:0, every optional tool
CASES = [
    ("u2x2", dict(tile_cols=2, tile_rows=2)),
    ("cols3_explicit", dict(tile_cols=3, tile_rows=1, tile_uniform=0, tile_col_w=(1, 2))),
    ("rows3", dict(tile_cols=1, tile_rows=3)),
    ("crop_4x3_explicit_10b", dict(width=200, height=120, conf_right=6, conf_bottom=2, bit_depth=10, tile_cols=4,
                                   tile_rows=3, tile_uniform=0, tile_col_w=(2, 1, 1), tile_row_h=(1, 1))),
    ("ctb16_4x3", dict(tile_cols=4, tile_rows=3, log2_ctb=4, log2_max_tb=4, max_th_depth_intra=2)),
    ("ctb64_partial_tools", dict(width=200, height=136, log2_ctb=6, bit_depth=10, tile_cols=2, tile_rows=2,
                                 tq_bypass=1, transform_skip=1, scaling_list=1, diff_cu_qp_delta_depth=2,
                                 max_th_depth_intra=3)),
    ("mono_1ctb_tiles", dict(chroma_format=0, tile_cols=4, tile_rows=3)),
    ("dense_lowqp_10b", dict(width=256, height=128, bit_depth=10, tile_cols=4, tile_rows=2, init_qp=22,
                             slice_qp_delta=-30, density=80, beta_offset_div2=3, tc_offset_div2=-2)),
    ("c422_3x2", dict(chroma_format=2, tile_cols=3, tile_rows=2)),
    ("c444_2x2_10b", dict(chroma_format=3, bit_depth=10, tile_cols=2, tile_rows=2, scaling_list=1)),
    # tiles together with WPP: every CTB row of a tile a substream, synced with
    # the tile's row above (one-CTB-wide tiles never sync), qPY_PREV restarting
    # at each row of a tile (slice.rs:155-171 reads the entry points for both)
    ("wpp_3x2", dict(width=256, height=192, tile_cols=3, tile_rows=2, wpp=1)),
    ("wpp_explicit_1ctb_col_10b", dict(width=200, height=160, bit_depth=10, tile_cols=3, tile_rows=2, tile_uniform=0,
                                       tile_col_w=(1, 3), tile_row_h=(2,), wpp=1, conf_right=6)),
    ("wpp_c444_ctb16", dict(chroma_format=3, log2_ctb=4, log2_max_tb=4, max_th_depth_intra=2, tile_cols=2,
                            tile_rows=2, wpp=1)),
]


def params(over, across=0):
    return S.SynthParams(**{**dict(width=128, height=96, wpp=0, tile_lf_across=across), **over})


def checks_ok(img):
    return all(c["term_ok"] and c["raw_start"] == c["raw_entry"] for c in img.checks)


def _split_decode(oracle_mod, p, nal):
    def dec(sp):
        img = oracle_mod.decode_heic(S.single_heic(sp.params, nal=sp.nal), debug_flags=4)
        assert checks_ok(img)
        return img.y, img.cb, img.cr

    return assemble(p, split_tiles(p, nal), dec)


@pytest.mark.parametrize("name,over", CASES, ids=[c[0] for c in CASES])
def test_oracle_tiles_equal_standalone_tiles(oracle_mod, name, over):
    """loop_filter_across_tiles = 0: the spec-literal tiled decode equals the
    tiles decoded as separate pictures, sample for sample, and every tile's
    substream ends exactly at its entry point."""
    p = params(over)
    for seed in range(3):
        nal = S.picture(p, seed)
        img = oracle_mod.decode_heic(S.single_heic(p, nal=nal))
        ctb = 1 << p.log2_ctb
        nsub = p.tile_cols * (-(-p.height // ctb)) if p.wpp else p.tile_cols * p.tile_rows
        assert checks_ok(img) and len(img.checks) == nsub, (name, seed)
        want = _split_decode(oracle_mod, p, nal)
        for got, ref, c in zip((img.y, img.cb, img.cr), want, "YUV"):
            if ref is None:
                assert got is None
                continue
            assert got.shape == ref.shape, (name, seed, c)
            assert int((got != ref).sum()) == 0, (name, seed, c)


@pytest.mark.parametrize("name,over", CASES[:5], ids=[c[0] for c in CASES[:5]])
def test_oracle_tiles_loop_filter_across(oracle_mod, name, over):
    """loop_filter_across_tiles = 1: same coded data, so the decode differs
    from the stand-alone tiles only where deblocking (3 samples, 1 for chroma)
    and SAO (one more) reach across a tile boundary; it does differ there."""
    p0 = params(over)
    p1 = params(over, across=1)
    ctb = 1 << p0.log2_ctb
    from hevc_tiles import tile_bounds

    cols = tile_bounds(p0.tile_cols, -(-p0.width // ctb), p0.tile_uniform, p0.tile_col_w)[1:-1]
    rows = tile_bounds(p0.tile_rows, -(-p0.height // ctb), p0.tile_uniform, p0.tile_row_h)[1:-1]
    differs = 0
    for seed in range(3):
        nal = S.picture(p1, seed)
        img = oracle_mod.decode_heic(S.single_heic(p1, nal=nal))
        assert checks_ok(img)
        want = _split_decode(oracle_mod, p0, S.picture(p0, seed))
        for got, ref, sub in zip((img.y, img.cb, img.cr), want, (1, 2, 2)):
            if ref is None:
                continue
            near = np.zeros(ref.shape, bool)
            reach = 4 if sub == 1 else 2
            for c in cols:
                e = c * ctb // sub
                near[:, max(e - reach, 0):e + reach] = True
            for r in rows:
                e = r * ctb // sub
                near[max(e - reach, 0):e + reach, :] = True
            diff = got != ref
            assert not (diff & ~near).any(), (name, seed)
            differs += int(diff.sum())
    if not (p0.deblock_disabled and not p0.sao):
        assert differs > 0, name


def test_synth_tiled_stream_layout():
    """The generator writes tiles_enabled_flag, the tile layout, one entry
    point per tile (per CTB row of each tile with WPP), and refuses explicit
    sizes that leave no CTB for the last column."""
    p = params(dict(tile_cols=3, tile_rows=2))
    subs = split_tiles(p, S.picture(p, 0))
    assert len(subs) == 6
    assert [(s.x0, s.y0) for s in subs] == [(0, 0), (32, 0), (64, 0), (0, 32), (32, 32), (64, 32)]
    assert [(s.params.width, s.params.height) for s in subs][:3] == [(32, 32), (32, 32), (64, 32)]
    pw = params(dict(width=128, height=160, tile_cols=2, tile_rows=2, wpp=1))  # 5 CTB rows: tiles of 2 and 3
    subs = split_tiles(pw, S.picture(pw, 0))
    assert [(s.x0, s.y0, s.params.height, s.params.wpp) for s in subs] == [
        (0, 0, 64, 1), (64, 0, 64, 1), (0, 64, 96, 1), (64, 64, 96, 1)]
    with pytest.raises(ValueError):
        S.picture(params(dict(tile_cols=2, tile_rows=1, tile_uniform=0, tile_col_w=(4,))), 0)


def test_host_accepts_tiles_and_tiles_with_wpp(oracle_mod):
    """Host parse: tiles with and without loop filtering across them, and
    tiles together with WPP, are accepted; a tiles + WPP PPS over slice data
    with one entry point per tile (not per tile row) is a malformed stream."""
    import heif_amd as H
    import ps_writer as W

    p = params(dict(tile_cols=2, tile_rows=2))
    inf = H.HeifImage.parse(S.single_heic(p, seed=1)).info
    assert (inf.width, inf.height) == (128, 96)
    H.HeifImage.parse(S.single_heic(params(dict(tile_cols=2, tile_rows=2), across=1), seed=1))
    H.HeifImage.parse(S.single_heic(params(dict(tile_cols=2, tile_rows=2, wpp=1)), seed=1))
    vps, sps, _ = S.parameter_sets(p)
    pps = W.pps(wpp=1, tiles=dict(cols=2, rows=2))
    both = S.single_heic(p, param_sets=(vps, sps, pps), nal=S.picture(p, 1))
    with pytest.raises(H.HeifGpuError) as e:
        H.HeifImage.parse(both)
    assert not isinstance(e.value, H.UnsupportedError)
    # explicit column widths that overrun the picture (4 CTB columns)
    bad = W.pps(wpp=0, tiles=dict(cols=2, rows=1, uniform=0, col_w=(5,), row_h=()))
    with pytest.raises(H.HeifGpuError) as e:
        H.HeifImage.parse(S.single_heic(p, param_sets=(vps, sps, bad), nal=S.picture(p, 1)))
    assert not isinstance(e.value, H.UnsupportedError)


def test_host_rejects_missing_tile_entry_points():
    """A tiled picture must carry one entry point per tile (7.4.7.1)."""
    import heif_amd as H

    p = params(dict(tile_cols=2, tile_rows=2))
    p3 = params(dict(tile_cols=3, tile_rows=2))
    # PPS says 3x2 tiles, the slice header holds 2x2 = 3 entry points
    data = S.single_heic(p3, param_sets=S.parameter_sets(p3), nal=S.picture(p, 2))
    with pytest.raises(H.HeifGpuError) as e:
        H.HeifImage.parse(data)
    assert not isinstance(e.value, H.UnsupportedError)


# ------------------------------------------------------------ kernel emulation
CSRC = os.path.join(os.path.dirname(__file__), "..", "heif_amd", "csrc")


@pytest.fixture(scope="module")
def emu_check():
    make_emu("emu-fast")
    return os.path.join(CSRC, "build", "emu_fast", "emu_check")


@pytest.mark.parametrize("parse", ["lanes", "solo", "spread"])
@pytest.mark.parametrize("name,across", [("crop_4x3_explicit_10b", 0), ("ctb64_partial_tools", 0),
                                         ("mono_1ctb_tiles", 0), ("crop_4x3_explicit_10b", 1), ("u2x2", 1),
                                         ("c422_3x2", 1), ("c444_2x2_10b", 0)])
def test_emulated_kernels_tiled(emu_check, tmp_path, name, across, parse):
    """The kernels' source compiled for the host decodes tiled pictures (one
    picture per tile; with loop filtering across tiles, children of an
    assembly) bit-exactly against the spec-literal oracle."""
    p = params(dict(CASES)[name], across=across)
    path = tmp_path / "t.heic"
    path.write_bytes(S.single_heic(p, seed=7))
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
def test_gpu_tiled_pictures_bit_exact(H, oracle_mod, parse):
    """Every tile case, with and without loop filtering across tiles, two
    seeds each, in one batch per parse mode and format (8-bit 4:2:0, 10-bit
    4:2:0, 8-bit 4:0:0, 8-bit 4:2:2, 10-bit 4:4:4), checked against the
    spec-literal oracle."""
    ctx = H.DecodeContext(0)
    for depth, chroma in ((8, 1), (10, 1), (8, 0), (8, 2), (10, 3)):
        datas = []
        for name, over in CASES:
            for across in (0, 1):  # loop_filter_across_tiles_enabled_flag (1: an assembly picture)
                p = params(over, across=across)
                if (p.bit_depth, p.chroma_format) == (depth, chroma):
                    datas += [S.single_heic(p, seed=s) for s in (1, 2)]
        imgs = [H.HeifImage.parse(d) for d in datas]
        b = ctx.prepare(imgs, parse=parse)
        outs = ctx.alloc_outputs(imgs)
        b.decode_async(outs)
        assert not any(b.status()), depth
        for k, (d, o) in enumerate(zip(datas, outs)):
            _assert_equal(_planes(o), oracle_mod.decode_heic(d, with_checks=False), (depth, k))
        b.free()
    ctx.close()


@pytest.mark.gpu
def test_gpu_tiled_grid_mixed_with_untiled(H, oracle_mod, halfmoonbay):
    """A HEIF grid whose grid tiles are themselves HEVC-tiled pictures (a 3x2
    tile layout in each 512x256 picture, filtered across tiles: six
    assemblies), batched with halfmoonbay (WPP) and an untiled picture: each
    picture keeps its own substream layout; every image checked, over two
    pipelined decodes."""
    p = params(dict(width=512, height=256, tile_cols=3, tile_rows=2, tile_uniform=0, tile_col_w=(4, 6),
                    tile_row_h=(3,)), across=1)
    grid = S.grid_heic(1000, 500, p, seed=9)
    plain = S.single_heic(params(dict(width=512, height=256)), seed=9)
    datas = [grid, halfmoonbay, plain]
    ctx = H.DecodeContext(0)
    imgs = [H.HeifImage.parse(d) for d in datas]
    b = ctx.prepare(imgs)
    outs = ctx.alloc_outputs(imgs)
    for _ in range(2):
        b.decode_async(outs)
    assert b.status() == [0, 0, 0]
    for k, (d, o) in enumerate(zip(datas, outs)):
        _assert_equal(_planes(o), oracle_mod.decode_heic(d, with_checks=False), k)
    b.free()
    ctx.close()
