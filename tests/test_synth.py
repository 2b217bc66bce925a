"""Synthetic HEVC-intra inputs (Main-10 / 8K grid,
BASELINE config 5, plus the coding tools halfmoonbay does not use).

The generator (heif_amd/csrc/synth/hevc_synth.c) draws every syntax element
at random, so a stream it writes is decodable only if encoder and decoder
agree on every context selection and binarization: the oracle's per-substream
self-check (end_of_subset_one_bit at the entry point, alignment bits) fails
almost surely otherwise.  Reconstruction of these streams is "parity
unpinned" against the reference (it computes no pixels and ships no 10-bit
sample); the GPU must equal the oracle bit-exactly.
"""
import hashlib
import json

import numpy as np
import pytest

from conftest import GOLDEN, make_emu

S = pytest.importorskip("heif_amd.synth_encoder")

# (name, overrides): every optional tool, bit depths 8/9/10, 4:0:0, CTB 16/32/64,
# partial CTBs and a conformance crop
CASES = [
    ("main8", dict()),
    ("main10", dict(bit_depth=10)),
    ("mono10", dict(bit_depth=10, chroma_format=0)),
    ("mono8", dict(chroma_format=0)),
    # Main 12 / RExt 12-bit: QpBdOffset 24, tc and beta scaled by 16, SAO offsets
    # capped at 31 without scaling (log2_sao_offset_scale is a rejected RExt tool)
    ("main12", dict(bit_depth=12)),
    ("mono12_bypass", dict(bit_depth=12, chroma_format=0, tq_bypass=1)),
    ("c444_12b_pcm", dict(chroma_format=3, bit_depth=12, pcm=1, pcm_pct=30, pcm_bd_y=12, pcm_bd_c=11)),
    ("b11_lowqp_dense", dict(bit_depth=11, init_qp=22, slice_qp_delta=-40, density=80, transform_skip=1)),
    ("b9_ctb16", dict(bit_depth=9, log2_ctb=4, log2_max_tb=4, max_th_depth_intra=2, diff_cu_qp_delta_depth=0)),
    ("ctb64_tskip_bypass", dict(bit_depth=10, log2_ctb=6, max_th_depth_intra=3, diff_cu_qp_delta_depth=2,
                                transform_skip=1, tq_bypass=1)),
    ("scaling_nosdh_qpoff", dict(bit_depth=10, scaling_list=1, sign_hiding=0, strong_intra=0, cb_qp_offset=-3,
                                 cr_qp_offset=5, init_qp=40, slice_qp_delta=-30)),
    ("lowqp_dense_dbk_offsets", dict(bit_depth=10, init_qp=22, slice_qp_delta=-33, beta_offset_div2=3,
                                     tc_offset_div2=-2, density=80)),
    ("no_loopfilter_cb16", dict(deblock_disabled=1, sao=0, cu_qp_delta=0, log2_min_cb=4)),
    ("crop_200x120", dict(width=200, height=120, conf_right=6, conf_bottom=2, bit_depth=10)),
    ("one_cb", dict(width=8, height=8)),
    ("ctb64_partial", dict(width=72, height=40, log2_ctb=6, bit_depth=10, tq_bypass=1, transform_skip=1,
                           scaling_list=1)),
    # entropy_coding_sync_enabled_flag = 0: the slice is one CABAC substream
    # (BASELINE config 2; the reference's main read_data path, slice.rs:206-231)
    ("nowpp_512", dict(width=512, height=512, wpp=0)),
    ("nowpp_ctb16_10b", dict(bit_depth=10, log2_ctb=4, log2_max_tb=4, max_th_depth_intra=2, wpp=0)),
    # more than 64 CTB rows: WPP rows wrap round a picture's 64 lanes
    ("rows68_ctb16", dict(width=64, height=1088, log2_ctb=4, log2_max_tb=4, max_th_depth_intra=2)),
    ("rows135_main10", dict(width=96, height=4320, bit_depth=10)),
    ("rows68_nowpp", dict(width=64, height=1088, log2_ctb=4, log2_max_tb=4, wpp=0)),
    # 132 CTBs wide x 70 rows: the row above a wrapped lane's next row is still
    # being parsed when its contexts are stored (the staging block)
    ("ring_wide_2112x1120", dict(width=2112, height=1120, log2_ctb=4, log2_max_tb=4, density=10)),
    # PCM coding units (pcm_sample(): raw samples between two engine runs;
    # parameter_set_reader.rs:107-125 parses the SPS fields): PCM bit depths
    # below the coding bit depth, 8x8..32x32 CUs, loop filters off for them,
    # 4:0:0, transquant bypass, every eligible CU PCM
    ("pcm_8b", dict(pcm=1, pcm_pct=30)),
    ("pcm_lowbd_nofilter_nowpp", dict(pcm=1, pcm_bd_y=5, pcm_bd_c=7, pcm_lf_disabled=1, pcm_pct=30, wpp=0)),
    ("pcm_10b_16_32", dict(bit_depth=10, pcm=1, pcm_bd_y=9, pcm_bd_c=10, pcm_log2_min=4, pcm_log2_max=5, pcm_pct=40)),
    ("pcm_mono_bypass", dict(chroma_format=0, pcm=1, pcm_pct=30, tq_bypass=1)),
    ("pcm_all_ctb16", dict(pcm=1, pcm_pct=100, pcm_lf_disabled=1, log2_ctb=4, log2_max_tb=4, pcm_log2_max=4)),
    # 4:2:2 (two chroma TBs per component, stacked; Table 8-3 mode mapping) and
    # 4:4:4 (chroma TBs the luma size, four chroma modes in an NxN CU, reference
    # sample filtering, 32x32 chroma scaling factors); the reference's
    # parameter_set_reader.rs reads chroma_format_idc 0..3
    ("c422_8b", dict(chroma_format=2)),
    ("c444_8b", dict(chroma_format=3)),
    ("c422_10b_ctb64_tools", dict(chroma_format=2, bit_depth=10, log2_ctb=6, max_th_depth_intra=3, transform_skip=1,
                                  tq_bypass=1, scaling_list=1, cb_qp_offset=-2, cr_qp_offset=3)),
    ("c444_10b_ctb16_scaling", dict(chroma_format=3, bit_depth=10, log2_ctb=4, log2_max_tb=4, max_th_depth_intra=2,
                                    scaling_list=1, transform_skip=1)),
    ("c444_ctb64_scaling32", dict(chroma_format=3, log2_ctb=6, max_th_depth_intra=3, scaling_list=1)),
    ("c422_lowqp_dense_nowpp", dict(chroma_format=2, bit_depth=10, init_qp=22, slice_qp_delta=-33, density=80,
                                    wpp=0)),
    ("c444_lowqp_dense", dict(chroma_format=3, bit_depth=10, init_qp=22, slice_qp_delta=-33, density=80)),
    ("c422_crop_200x120", dict(chroma_format=2, width=200, height=120, conf_right=6, conf_bottom=3)),
    ("c444_crop_200x120", dict(chroma_format=3, width=200, height=120, conf_right=5, conf_bottom=3, bit_depth=9)),
    ("c422_pcm_nowpp", dict(chroma_format=2, pcm=1, pcm_pct=30, pcm_bd_c=6, wpp=0)),
    ("c444_pcm_nofilter", dict(chroma_format=3, pcm=1, pcm_pct=30, pcm_lf_disabled=1, pcm_log2_max=5)),
]


def params(over):
    return S.SynthParams(**{**dict(width=128, height=96), **over})


def checks_ok(img):
    return all(c["term_ok"] and c["raw_start"] == c["raw_entry"] for c in img.checks)


@pytest.mark.parametrize("name,over", CASES, ids=[c[0] for c in CASES])
def test_oracle_decodes_synthetic_streams(oracle_mod, name, over):
    p = params(over)
    for seed in range(4):
        data = S.single_heic(p, seed=seed)
        img = oracle_mod.decode_heic(data)
        assert checks_ok(img), (name, seed)
        assert img.bit_depth == p.bit_depth
        assert img.y.shape == (p.height - p.conf_bottom, p.width - p.conf_right)
        assert (img.cb is None) == (p.chroma_format == 0)
        assert int(img.y.max()) < (1 << p.bit_depth)


def test_gpu_cases_cover_every_chroma_pair(oracle_mod):
    """The 4:2:0 cases test_gpu_synthetic_bit_exact decodes (seeds 0 and 1)
    hold 4x4 and 8x8 chroma TBs of every IntraPredModeC, with and without
    coefficients: k_intra's GPU-only Cb+Cr pair path (predict_pair, which the
    host emulation does not build) is pinned bit-exact on all 140 kinds."""
    tot = np.zeros((2, 35, 2), np.int64)
    for name, over in CASES:
        p = params(over)
        if p.chroma_format != 1:
            continue
        for seed in range(2):
            oracle_mod.chroma_tb_hist(True)
            oracle_mod.decode_heic(S.single_heic(p, seed=seed), with_checks=False, debug_flags=8)
            tot += oracle_mod.chroma_tb_hist(True)
    assert (tot > 0).all(), np.argwhere(tot == 0)[:10]


def test_generator_is_deterministic():
    p = params(dict(bit_depth=10))
    assert S.picture(p, 3) == S.picture(p, 3)
    assert S.picture(p, 3) != S.picture(p, 4)


def test_generator_rejects_bad_parameters():
    with pytest.raises(ValueError):
        S.picture(params(dict(width=100)), 0)      # not a multiple of MinCbSize
    with pytest.raises(ValueError):
        S.picture(params(dict(bit_depth=13)), 0)
    with pytest.raises(ValueError):
        S.picture(params(dict(log2_max_tb=6, log2_ctb=6)), 0)


def test_host_parses_config5_grid(oracle_mod):
    """BASELINE config 5 geometry: 7680x4320 10-bit -> 15 x 9 tiles of 512x512."""
    import heif_amd as H

    p = S.SynthParams(bit_depth=10, density=5)
    pics = [S.picture(p, 0)] * 135           # geometry only: one picture repeated
    data = S.grid_heic(7680, 4320, p, pictures=pics)
    meta = oracle_mod.read_meta(data)
    assert (meta["grid_rows"], meta["grid_cols"], meta["num_tiles"]) == (9, 15, 135)
    assert (meta["out_width"], meta["out_height"], meta["luma_bits"]) == (7680, 4320, 10)
    inf = H.HeifImage.parse(data).info
    assert (inf.width, inf.height, inf.bit_depth, inf.bytes_per_sample) == (7680, 4320, 10, 2)


def _golden_hash(img):
    h = hashlib.sha256()
    for pl in (img.y, img.cb, img.cr):
        if pl is not None:
            h.update(pl.astype("<u2").tobytes())
    return h.hexdigest()


def test_oracle_synthetic_golden_hashes(oracle_mod):
    """Regression pin of the oracle's reconstruction of two synthetic streams
    (tests/golden/synth_planes.json, written by tools/make_golden.py)."""
    g = json.loads((GOLDEN / "synth_planes.json").read_text())
    for name, ent in g.items():
        p = S.SynthParams(**ent["params"])
        data = S.grid_heic(ent["out_w"], ent["out_h"], p, seed=ent["seed"])
        assert hashlib.sha256(data).hexdigest() == ent["heic_sha256"], name
        assert _golden_hash(oracle_mod.decode_heic(data, with_checks=False)) == ent["planes_sha256"], name


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
        bad = int((g != r).sum())
        assert bad == 0, f"{tag} {c}: {bad} samples differ"


@pytest.fixture(scope="module")
def gctx(H):
    c = H.DecodeContext(0)
    yield c
    c.close()


def _decode(H, ctx, datas, parse, ppw=0):
    imgs = [H.HeifImage.parse(d) for d in datas]
    b = ctx.prepare(imgs, parse=parse, pics_per_wave=ppw)
    outs = ctx.alloc_outputs(imgs)
    b.decode_async(outs)
    st = b.status()
    b.free()
    return outs, st


@pytest.mark.gpu
@pytest.mark.parametrize("parse", ["solo", "spread", "lanes"])
@pytest.mark.parametrize("name,over", CASES, ids=[c[0] for c in CASES])
def test_gpu_synthetic_bit_exact(H, gctx, oracle_mod, name, over, parse):
    """Every tool / geometry case in every parse mode: k_parse_solo<false>
    (one substream per wave, a picture's rows in one workgroup; rows beyond 16
    wrap round the waves), k_parse_solo<true> (spread: every row its own
    workgroup, WPP through coherent global memory) and k_parse_lanes (one
    substream per lane; rows beyond 64 wrap round the lanes)."""
    p = params(over)
    for seed in range(2):
        data = S.single_heic(p, seed=seed)
        outs, st = _decode(H, gctx, [data], parse)
        assert st == [0], (name, seed)
        _assert_equal(_planes(outs[0]), oracle_mod.decode_heic(data, with_checks=False), (name, seed))


@pytest.mark.gpu
@pytest.mark.parametrize("cf,bd", [(2, 8), (3, 10)])
def test_gpu_chroma_format_grid_rgb_gather(H, oracle_mod, cf, bd):
    """A 4:2:2 / 4:4:4 grid (cropped last row and column): bit-exact planes of
    the Cb / Cr shapes chroma_dims gives, RGB exact against tests/rgb_ref.py,
    and the tile split over two batches gathered (heifgpu_gather_tiles) back
    into the same planes."""
    import numpy as np
    import torch

    import rgb_ref

    data = S.grid_heic(300, 200, params(dict(chroma_format=cf, bit_depth=bd)), seed=5)
    ref = oracle_mod.decode_heic(data, with_checks=False)
    ctx = H.DecodeContext(0)
    img = H.HeifImage.parse(data)
    assert img.info.chroma_format_idc == cf
    out = ctx.alloc_outputs([img])[0]
    assert tuple(out.cb.shape) == H.chroma_dims(img.info) == ref.cb.shape
    b = ctx.prepare([img])
    b.decode_async([out])
    assert b.status() == [0]
    _assert_equal(_planes(out), ref, ("grid", cf))
    rgb = ctx.to_rgb(out).cpu().numpy()
    want = rgb_ref.ycbcr_to_rgb(out.y.cpu().numpy(), out.cb.cpu().numpy(), out.cr.cpu().numpy(),
                                img.info.matrix_coeffs, bool(img.info.full_range), img.info.rotation, bd)
    assert np.array_equal(rgb, want)
    dst = ctx.alloc_outputs([img])[0]
    for t in (dst.y, dst.cb, dst.cr):
        t.fill_(0)
    for g in range(2):
        part = ctx.alloc_outputs([img])[0]
        bb = ctx.prepare([img], tile_stride=2, tile_offset=g)
        bb.decode_async([part])
        assert bb.status() == [0]
        bb.free()
        ctx.gather_tiles(dst, part, 2, g)
    torch.cuda.synchronize()
    _assert_equal(_planes(dst), ref, ("gather", cf))


@pytest.mark.gpu
def test_gpu_mixed_geometry_batch(H, oracle_mod):
    """One batch of 10-bit 4:2:0 grids whose tiles differ in size, CTB size and
    coding tools (one SeqParams per distinct SPS/PPS); a batch that mixes bit
    depth or chroma format is rejected with HEIFGPU_E_UNSUPPORTED."""
    datas = [S.grid_heic(1000, 700, params(dict(width=256, height=256, bit_depth=10)), seed=1),
             S.grid_heic(900, 500, params(dict(bit_depth=10, log2_ctb=6, transform_skip=1, tq_bypass=1)), seed=2),
             S.grid_heic(300, 200, params(dict(width=64, height=64, bit_depth=10, log2_ctb=4, log2_max_tb=4,
                                               scaling_list=1)), seed=3)]
    ctx = H.DecodeContext(0)
    imgs = [H.HeifImage.parse(d) for d in datas]
    b = ctx.prepare(imgs)
    outs = ctx.alloc_outputs(imgs)
    b.decode_async(outs)
    assert b.status() == [0, 0, 0]
    for k, (d, o) in enumerate(zip(datas, outs)):
        _assert_equal(_planes(o), oracle_mod.decode_heic(d, with_checks=False), k)
    b.free()
    mixed = [H.HeifImage.parse(datas[0]), H.HeifImage.parse(S.single_heic(params(dict()), seed=4))]
    with pytest.raises(H.UnsupportedError):
        ctx.prepare(mixed)
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("parse", ["solo", "spread", "lanes"])
def test_gpu_mixed_wpp_ring_batch(H, oracle_mod, halfmoonbay, parse):
    """One batch mixing a 48-tile WPP grid (halfmoonbay), a non-WPP 512x512
    single-substream picture (config 2) and a 68-row CTB-16 picture whose WPP
    rows wrap round its 64 lanes (16 waves in solo mode): lanes per picture is
    the batch maximum, and each picture keeps its own substream layout."""
    datas = [halfmoonbay, S.single_heic(params(dict(width=512, height=512, wpp=0)), seed=11),
             S.single_heic(params(dict(width=64, height=1088, log2_ctb=4, log2_max_tb=4)), seed=12)]
    ctx = H.DecodeContext(0)
    imgs = [H.HeifImage.parse(d) for d in datas]
    b = ctx.prepare(imgs, parse=parse)
    outs = ctx.alloc_outputs(imgs)
    for _ in range(2):  # two pipelined decodes (alternate parse sets)
        b.decode_async(outs)
    assert b.status() == [0, 0, 0]
    for k, (d, o) in enumerate(zip(datas, outs)):
        _assert_equal(_planes(o), oracle_mod.decode_heic(d, with_checks=False), k)
    b.free()
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("parse,ppw", [("lanes", 64), ("lanes", 0), ("solo", 0), ("spread", 0)])
def test_gpu_nowpp_batch_64_per_wave(H, gctx, oracle_mod, parse, ppw):
    """128 non-WPP pictures (one substream each).  ("lanes", 64): every
    k_parse_lanes wave packs 64 pictures, one per lane (2 waves); ("lanes", 0):
    the adaptive packing, which for 128 pictures is one picture per wave; solo:
    one single-wave workgroup per picture.  Every picture checked."""
    p = params(dict(width=64, height=64, wpp=0))
    datas = [S.single_heic(p, seed=100 + k) for k in range(128)]
    outs, st = _decode(H, gctx, datas, parse, ppw)
    assert not any(st)
    for k in range(128):
        _assert_equal(_planes(outs[k]), oracle_mod.decode_heic(datas[k], with_checks=False), k)


@pytest.mark.gpu
def test_gpu_config5_8k_main10_grid(H, oracle_mod):
    """BASELINE config 5 at full size: 7680x4320 Main-10 grid, 135 tiles."""
    c5 = S.CONFIG5
    data = S.grid_heic(c5["out_w"], c5["out_h"], c5["params"], seed=5)
    out = H.HeicDecoder.decode(data)
    torch.cuda.synchronize()
    assert out.y.dtype == torch.int16 and out.y.shape == (4320, 7680)
    _assert_equal(_planes(out), oracle_mod.decode_heic(data, with_checks=False), "config5")


# ------------------------------------------- kernels compiled for the host
@pytest.mark.parametrize("parser", ["solo", "spread", "lanes", "ppw1"])
def test_emulated_kernels_on_synthetic_streams(tmp_path, parser):
    """The GPU kernels' source built for the host (HG_HOST_EMU, see
    test_emulation.py) decodes every synthetic case bit-exactly vs the oracle."""
    import os
    import pathlib
    import subprocess

    csrc = pathlib.Path(__file__).resolve().parents[1] / "heif_amd" / "csrc"
    make_emu("emu-fast")
    exe = csrc / "build" / "emu_fast" / "emu_check"
    env = dict(os.environ, HEIFGPU_PARSE=parser if parser in ("solo", "spread") else "lanes",
               **({"HEIFGPU_LANES_PPW": "1"} if parser == "ppw1" else {}))
    for name, over in CASES:
        path = tmp_path / f"{name}.heic"
        path.write_bytes(S.single_heic(params(over), seed=1))
        r = subprocess.run([str(exe), str(path), "5"], capture_output=True, text=True, env=env, timeout=300)
        assert r.returncode == 0 and "EMU PARITY OK" in r.stdout + r.stderr, (name, (r.stdout + r.stderr)[-400:])


# ------------------------------------------- corrupt synthetic streams
def _corrupt_synth(mode):
    """A 10-bit CTB-64 grid (transform skip, bypass, scaling lists) with slice
    data damaged in three tiles (random bytes) or one tile half zeroed."""
    import random

    from oracle import oracle

    p = params(dict(width=256, height=256, bit_depth=10, log2_ctb=6, transform_skip=1, tq_bypass=1, scaling_list=1))
    data = bytearray(S.grid_heic(700, 500, p, seed=9))
    tiles, _ = oracle.list_tiles(bytes(data))
    rng = random.Random(2)
    if mode == "random":
        for k in (0, 2, 5):
            o, n = tiles[k]
            for _ in range(40):
                data[o + 30 + rng.randrange(n - 30)] = rng.randrange(256)
    else:
        o, n = tiles[4]
        data[o + n // 2:o + n] = bytes(n - n // 2)
    return bytes(data)


@pytest.mark.parametrize("mode", ["random", "zeroed"])
def test_emulated_kernels_survive_corrupt_synthetic(tmp_path, mode):
    import pathlib
    import subprocess

    csrc = pathlib.Path(__file__).resolve().parents[1] / "heif_amd" / "csrc"
    make_emu("emu-fast")
    path = tmp_path / f"{mode}.heic"
    path.write_bytes(_corrupt_synth(mode))
    r = subprocess.run([str(csrc / "build" / "emu_fast" / "emu_check"), str(path), "5"], capture_output=True,
                       text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode in (0, 1), out[-2000:]
    line = next(l for l in out.splitlines() if l.startswith("parse: status"))
    assert int(line.split()[2].rstrip(","), 16) != 0


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["random", "zeroed"])
def test_gpu_corrupt_synthetic_sets_status(H, oracle_mod, mode):
    """Damaged 10-bit CTB-64 streams end in status bits, never a device fault;
    the clean image in the same batch stays bit-exact."""
    clean = S.grid_heic(700, 500, params(dict(width=256, height=256, bit_depth=10, log2_ctb=6)), seed=10)
    ctx = H.DecodeContext(0)
    imgs = [H.HeifImage.parse(_corrupt_synth(mode)), H.HeifImage.parse(clean)]
    b = ctx.prepare(imgs)
    outs = ctx.alloc_outputs(imgs)
    b.decode_async(outs)
    st = b.status()
    assert st[0] != 0 and st[1] == 0
    _assert_equal(_planes(outs[1]), oracle_mod.decode_heic(clean, with_checks=False), "clean")
    b.free()
    ctx.close()
