"""GPU parity through the C ABI (run with -m gpu on an MI355X).

Bar: bit-exact planes against the CPU oracle on the same input.  At the
bench's batch sizes the check is size-independent: a permuted image is the
oracle's 48 independently decoded tiles re-placed by the permutation, so
every image of a large batch is checked without re-running the oracle per
image.
"""
import ctypes
import hashlib
import json

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def H():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import heif_amd

    return heif_amd


@pytest.fixture(scope="module")
def ctx(H):
    c = H.DecodeContext(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def oracle_tiles(oracle_mod, halfmoonbay):
    tiles, (ho, hl) = oracle_mod.list_tiles(halfmoonbay)
    hvcc = halfmoonbay[ho:ho + hl]
    return [oracle_mod.decode_tile(hvcc, halfmoonbay[o:o + n], 512, 512) for o, n in tiles]


def assemble(tiles, perm, rows=6, cols=8, w=4032, h=3024):
    y = np.zeros((h, w), np.uint16)
    cb = np.zeros((h // 2, w // 2), np.uint16)
    cr = np.zeros_like(cb)
    for k in range(rows * cols):
        r, c = divmod(k, cols)
        ty, tcb, tcr = tiles[perm[k]]
        hh, ww = min(512, h - 512 * r), min(512, w - 512 * c)
        y[512 * r:512 * r + hh, 512 * c:512 * c + ww] = ty[:hh, :ww]
        cb[256 * r:256 * r + hh // 2, 256 * c:256 * c + ww // 2] = tcb[:hh // 2, :ww // 2]
        cr[256 * r:256 * r + hh // 2, 256 * c:256 * c + ww // 2] = tcr[:hh // 2, :ww // 2]
    return y, cb, cr


def planes_np(o):
    return [t.cpu().numpy().astype(np.uint16) for t in (o.y, o.cb, o.cr)]


def test_halfmoonbay_bit_exact(H, oracle_halfmoonbay, halfmoonbay):
    """Config 3 through the reference-mirror API (one image: spread parse)."""
    out = H.HeicDecoder.decode(halfmoonbay)
    y, cb, cr = planes_np(out)
    assert np.array_equal(y, oracle_halfmoonbay.y)
    assert np.array_equal(cb, oracle_halfmoonbay.cb)
    assert np.array_equal(cr, oracle_halfmoonbay.cr)
    g = json.loads((GOLDEN / "halfmoonbay_planes.json").read_text())
    assert hashlib.sha256(out.y.cpu().numpy().tobytes()).hexdigest() == g["planes"]["y"]


@pytest.mark.parametrize("parse,ppw,geom", [
    ("solo", 0, {"mode": "solo", "workgroups": 48, "pics_per_wave": 1, "waves_per_workgroup": 16}),
    ("spread", 0, {"mode": "spread", "workgroups": 768, "pics_per_wave": 1, "waves_per_workgroup": 1}),
    ("lanes", 0, {"mode": "lanes", "workgroups": 48, "pics_per_wave": 1, "waves_per_workgroup": 1}),
    ("lanes", 4, {"mode": "lanes", "workgroups": 12, "pics_per_wave": 4, "waves_per_workgroup": 1}),
])
def test_halfmoonbay_parse_modes(H, ctx, oracle_halfmoonbay, halfmoonbay, parse, ppw, geom):
    """Config 3 in every parse geometry: solo (a workgroup of 16 waves per
    tile, one WPP row per wave), spread (one single-wave workgroup per WPP
    row: 768), lanes with one tile per wave, lanes packed four tiles per
    wave.  (r05's rows geometry is gone in ABI 6: test_rows_mode_removed.)"""
    img = H.HeifImage.parse(halfmoonbay)
    b = ctx.prepare([img], parse=parse, pics_per_wave=ppw)
    assert b.parse_geometry() == geom
    out = ctx.alloc_outputs([img])
    b.decode_async(out)
    assert b.status() == [0]
    b.free()
    for got, want in zip(planes_np(out[0]), (oracle_halfmoonbay.y, oracle_halfmoonbay.cb, oracle_halfmoonbay.cr)):
        assert np.array_equal(got, want)


@pytest.mark.parametrize("stream", ["0", "patience0", "default"])
def test_halfmoonbay_streaming_modes(H, oracle_halfmoonbay, halfmoonbay, monkeypatch, stream):
    """Spread parse with k_intra_stream (the default for one image), without it
    (k_transform + k_intra after the parse), and with a first launch that gives
    every picture up at once (HEIFGPU_STREAM_PATIENCE_US=0: what a profiler that
    serialises dispatches does to it), so the second launch after the parse
    reconstructs all of them.  Bit-exact with status 0 in every case.  (The
    knobs are read when a context is created: each case makes its own.)"""
    if stream == "0":
        monkeypatch.setenv("HEIFGPU_STREAM", "0")
    elif stream == "patience0":
        monkeypatch.setenv("HEIFGPU_STREAM_PATIENCE_US", "0")
    c = H.DecodeContext(0)
    try:
        img = H.HeifImage.parse(halfmoonbay)
        b = c.prepare([img], parse="spread")
        out = c.alloc_outputs([img])
        for _ in range(2):  # the second decode reuses the set's progress / done words
            b.decode_async(out)
        assert b.status() == [0]
        b.free()
    finally:
        c.close()
    for got, want in zip(planes_np(out[0]), (oracle_halfmoonbay.y, oracle_halfmoonbay.cb, oracle_halfmoonbay.cr)):
        assert np.array_equal(got, want)


@pytest.mark.parametrize("parse", ["lanes", "spread"])
def test_prep_stream_option(H, oracle_halfmoonbay, halfmoonbay, monkeypatch, parse):
    """HEIFGPU_PREP_STREAM=1 (read when a context is created): k_rbsp of each
    decode on its own stream, into the decode's parse set; three pipelined
    decodes (every set once) stay bit-exact with status 0."""
    monkeypatch.setenv("HEIFGPU_PREP_STREAM", "1")
    c = H.DecodeContext(0)
    try:
        img = H.HeifImage.parse(halfmoonbay)
        b = c.prepare([img], parse=parse)
        out = c.alloc_outputs([img])
        for _ in range(3):
            b.decode_async(out)
        assert b.status() == [0]
        b.free()
        for got, want in zip(planes_np(out[0]), (oracle_halfmoonbay.y, oracle_halfmoonbay.cb, oracle_halfmoonbay.cr)):
            assert np.array_equal(got, want)
    finally:
        c.close()


def check_permuted(outs, seeds, oracle_tiles):
    """Every image of a permuted batch, tile window by tile window against the
    oracle's 48 tile decodes placed by the image's permutation (the per-tile
    loop the batch replaces: /root/reference/src/heic/decoder.rs:114-119)."""
    from heif_amd.synthetic import permutation

    for s, o in zip(seeds, outs):
        perm = permutation(48, s)
        planes = [t.cpu().numpy() for t in (o.y, o.cb, o.cr)]
        for k in range(48):
            r, c = divmod(k, 8)
            for ci, pl in enumerate(planes):
                sh = 1 if ci else 0
                ts = 512 >> sh
                win = pl[ts * r:ts * (r + 1), ts * c:ts * (c + 1)]
                ref = oracle_tiles[perm[k]][ci][:win.shape[0], :win.shape[1]]
                assert np.array_equal(win, ref), (s, k, ci)


@pytest.mark.parametrize("parse,geom", [
    ("auto", {"mode": "lanes", "workgroups": 2048, "pics_per_wave": 3, "waves_per_workgroup": 1}),
    ("solo", {"mode": "solo", "workgroups": 6144, "pics_per_wave": 1, "waves_per_workgroup": 16}),
    ("spread", {"mode": "spread", "workgroups": 98304, "pics_per_wave": 1, "waves_per_workgroup": 1}),
    ("lanes4", {"mode": "lanes", "workgroups": 1536, "pics_per_wave": 4, "waves_per_workgroup": 1}),
])
def test_bench_shard_every_image(H, ctx, oracle_tiles, halfmoonbay, parse, geom):
    """The headline configuration itself (bench.py, config 4 shard): 128
    permuted 4032x3024 images = 6144 pictures.  The automatic choice packs three
    16-row pictures per k_parse_lanes wave (2048 waves, two per SIMD); solo runs 6144
    16-wave workgroups, spread 98,304 one-wave workgroups.  Every image is
    checked, decoded three times back to back (all three parse-output sets of
    the pipeline, each into its own planes)."""
    from heif_amd.synthetic import permuted_heic

    seeds = list(range(128))
    imgs = H.HeifImage.parse_many([permuted_heic(halfmoonbay, s) for s in seeds], threads=8)
    mode = {"lanes4": "lanes"}.get(parse, parse)
    b = ctx.prepare(imgs, parse=mode, pics_per_wave=4 if parse == "lanes4" else 0)
    assert b.parse_geometry() == geom
    outs = [ctx.alloc_outputs(imgs) for _ in range(3)]
    for o in outs:
        b.decode_async(o)
    assert not any(b.status())
    b.free()
    for o in outs:
        check_permuted(o, seeds, oracle_tiles)


def _damaged_halfmoonbay(oracle_mod, data, tile=5):
    """halfmoonbay with the last eighth of one grid tile's slice data
    overwritten with 0xff: the host accepts it, the kernels flag it."""
    items, _ = oracle_mod.list_tiles(data)
    o, n = items[tile]
    d = bytearray(data)
    d[o + n - n // 8:o + n] = b"\xff" * (n // 8)
    return bytes(d)


@pytest.mark.parametrize("sets", [0, 2, 1])
@pytest.mark.parametrize("parse", ["lanes", "spread"])
def test_status_sticky_over_pipelined_decodes(H, ctx, oracle_mod, oracle_tiles, halfmoonbay, parse, sets):
    """heifgpu_batch_status reports the OR over every decode since the last
    query (/root/reference/src/heic/decoder.rs:109-112: errors reach the
    caller): a batch with one damaged image decoded three times back to back
    (every parse-output set) shows the damage after each decode and after the
    three together, the clean images stay bit-exact, a query with no decode
    since the last one reads zero, and a reload without the damaged image
    reports clean."""
    bad = _damaged_halfmoonbay(oracle_mod, halfmoonbay)
    files = [halfmoonbay, bad, halfmoonbay]
    imgs = H.HeifImage.parse_many(files, threads=4)
    b = ctx.prepare(imgs, parse=parse, pipeline_sets=sets)
    outs = [ctx.alloc_outputs(imgs) for _ in range(3)]
    for o in outs:
        b.decode_async(o)
    st = b.status()
    assert st[0] == 0 and st[2] == 0 and st[1] != 0, st
    assert b.status() == [0, 0, 0]  # cleared by the query, nothing decoded since
    for o in outs:  # one query per decode: each sees the damage
        b.decode_async(o)
        st = b.status()
        assert st[0] == 0 and st[2] == 0 and st[1] != 0, st
    ident = list(range(48))
    for o in outs:
        for i in (0, 2):
            y, cb, cr = assemble(oracle_tiles, ident)
            assert np.array_equal(o[i].y.cpu().numpy(), y)
            assert np.array_equal(o[i].cb.cpu().numpy(), cb) and np.array_equal(o[i].cr.cpu().numpy(), cr)
    # a reload starts a new record: the damaged load's last decode (in flight
    # when the reload is issued) is not reported against the clean images, but
    # it reaches the caller through heifgpu_batch_status_previous
    clean = H.HeifImage.parse_many([halfmoonbay] * 3, threads=4)
    b.decode_async(outs[0])
    ctx.prepare(clean, reuse=b, wait=False)
    b.decode_async(outs[1])
    b.decode_async(outs[2])
    assert b.status() == [0, 0, 0]
    prev = b.status_previous()
    assert len(prev) == 3 and prev[0] == 0 and prev[2] == 0 and prev[1] != 0, prev
    assert b.status_previous() == [0, 0, 0]  # read and cleared
    b.free()


def test_status_previous_after_failed_reload(H, ctx, oracle_mod, halfmoonbay, monkeypatch):
    """A reload that fails after it has begun to overwrite its descriptor
    generation (injected: HEIFGPU_FAULT_INJECT=prepare) leaves the batch
    unusable until a reload succeeds; that reload must not overwrite the last
    good load's generation, so heifgpu_batch_status_previous still reports the
    last good load's decode errors, sized for it."""
    bad = _damaged_halfmoonbay(oracle_mod, halfmoonbay)
    a_imgs = H.HeifImage.parse_many([halfmoonbay, bad, halfmoonbay], threads=4)
    b = ctx.prepare(a_imgs)
    outs = ctx.alloc_outputs(a_imgs)
    b.decode_async(outs)  # load A, damaged image 1, status not read
    clean = H.HeifImage.parse_many([halfmoonbay] * 2, threads=4)
    monkeypatch.setenv("HEIFGPU_FAULT_INJECT", "prepare")
    with pytest.raises(H.HeifGpuError, match="injected"):
        ctx.prepare(clean, reuse=b, wait=False)
    monkeypatch.delenv("HEIFGPU_FAULT_INJECT")
    with pytest.raises(H.HeifGpuError, match="not loaded"):
        b.decode_async(outs)
    with pytest.raises(H.HeifGpuError, match="not loaded"):
        b.status_previous()
    ctx.prepare(clean, reuse=b)  # load B
    outs_b = ctx.alloc_outputs(clean)
    b.decode_async(outs_b)
    assert b.status() == [0, 0]
    prev = b.status_previous()  # A, three images, its damage kept
    assert len(prev) == 3 and prev[0] == 0 and prev[2] == 0 and prev[1] != 0, prev
    # a failure after a good reload: the next good reload's previous load is B
    monkeypatch.setenv("HEIFGPU_FAULT_INJECT", "prepare")
    with pytest.raises(H.HeifGpuError, match="injected"):
        ctx.prepare(a_imgs, reuse=b)
    monkeypatch.delenv("HEIFGPU_FAULT_INJECT")
    ctx.prepare(a_imgs, reuse=b)
    b.decode_async(outs)
    st = b.status()
    assert st[0] == 0 and st[2] == 0 and st[1] != 0, st
    assert b.status_previous() == [0, 0]
    b.free()


def test_permuted_batch_row_parallel(H, ctx, oracle_tiles, halfmoonbay):
    from heif_amd.synthetic import permutation, permuted_heic

    seeds = [1, 2, 3]
    imgs = [H.HeifImage.parse(permuted_heic(halfmoonbay, s)) for s in seeds]
    outs = ctx.alloc_outputs(imgs)
    b = ctx.prepare(imgs)
    b.decode_async(outs)
    assert b.status() == [0, 0, 0]
    for s, o in zip(seeds, outs):
        want = assemble(oracle_tiles, permutation(48, s))
        for got, w in zip(planes_np(o), want):
            assert np.array_equal(got, w), s
    b.free()


def test_large_batch_many_waves(H, ctx, oracle_tiles, halfmoonbay):
    """22 images = 1056 pictures.  AUTO takes the spread parse (up to 1536
    pictures, rows dequeued in row-major order: 16,896 single-wave jobs, far
    more than the chip holds at once).  Forced to lanes, the adaptive packing
    takes the fewest pictures per wave that fit one wave per SIMD, 2 here
    (528 waves on the 1024 SIMDs), size-sorted snake order across waves.
    Every image checked in both."""
    from heif_amd.synthetic import permuted_heic

    seeds = list(range(100, 122))
    imgs = [H.HeifImage.parse(permuted_heic(halfmoonbay, s)) for s in seeds]
    outs = ctx.alloc_outputs(imgs)
    for parse, geom in (("auto", {"mode": "spread", "workgroups": 16896, "pics_per_wave": 1, "waves_per_workgroup": 1}),
                        ("lanes", {"mode": "lanes", "workgroups": 528, "pics_per_wave": 2, "waves_per_workgroup": 1})):
        b = ctx.prepare(imgs, parse=parse)
        assert b.parse_geometry() == geom
        for o in outs:
            for t in (o.y, o.cb, o.cr):
                t.fill_(0)
        b.decode_async(outs)
        assert not any(b.status())
        check_permuted(outs, seeds, oracle_tiles)
        b.free()


def test_repeat_decode_is_deterministic(H, ctx, halfmoonbay):
    imgs = [H.HeifImage.parse(halfmoonbay)]
    outs = ctx.alloc_outputs(imgs)
    b = ctx.prepare(imgs)
    b.decode_async(outs)
    first = [t.clone() for t in (outs[0].y, outs[0].cb, outs[0].cr)]
    for _ in range(3):
        for t in (outs[0].y, outs[0].cb, outs[0].cr):
            t.fill_(0)
        b.decode_async(outs)
        assert b.status() == [0]
        for a, t in zip(first, (outs[0].y, outs[0].cb, outs[0].cr)):
            assert torch.equal(a, t)
    b.free()


def test_pitched_outputs(H, ctx, oracle_halfmoonbay, halfmoonbay):
    """Caller-owned planes with a row pitch larger than the width."""
    from heif_amd import _lib

    img = H.HeifImage.parse(halfmoonbay)
    y = torch.zeros((3024, 4096), dtype=torch.uint8, device="cuda")
    cb = torch.zeros((1512, 2048), dtype=torch.uint8, device="cuda")
    cr = torch.zeros((1512, 2048), dtype=torch.uint8, device="cuda")
    planes = (_lib.Planes * 1)()
    for c, t in enumerate((y, cb, cr)):
        planes[0].plane[c] = t.data_ptr()
        planes[0].pitch[c] = t.stride(0)
    st = (ctypes.c_uint32 * 1)()
    arr = (ctypes.c_void_p * 1)(img._h.value)
    s = torch.cuda.current_stream().cuda_stream
    assert _lib.lib.heifgpu_decode_batch(ctx._h, arr, 1, planes, ctypes.c_void_p(s), st) == 0
    assert st[0] == 0
    assert np.array_equal(y[:, :4032].cpu().numpy(), oracle_halfmoonbay.y)
    assert np.array_equal(cr[:, :2016].cpu().numpy(), oracle_halfmoonbay.cr)
    assert int(y[:, 4032:].abs().sum()) == 0  # nothing written past the width


@pytest.mark.parametrize("mode", ["random", "zeroed"])
def test_corrupt_stream_sets_status_not_fault(H, ctx, halfmoonbay, mode):
    from test_emulation import _corrupt

    imgs = [H.HeifImage.parse(_corrupt(halfmoonbay, mode)), H.HeifImage.parse(halfmoonbay)]
    outs = ctx.alloc_outputs(imgs)
    b = ctx.prepare(imgs)
    b.decode_async(outs)
    st = b.status()
    assert st[0] != 0 and st[1] == 0
    b.free()


def test_empty_batch_rejected(H, ctx):
    with pytest.raises(H.HeifGpuError):
        ctx.prepare([])


def test_native_library_is_loaded(H):
    import pathlib

    maps = pathlib.Path("/proc/self/maps").read_text()
    assert "libheifgpu" in maps


def test_pipelined_decodes_back_to_back(H, ctx, oracle_tiles, halfmoonbay):
    """Several decodes of one batch issued without synchronisation: the parse of
    call n+1 overlaps the reconstruction of call n (alternate parse sets), and
    every call's planes must still be exact."""
    from heif_amd.synthetic import permutation, permuted_heic

    seeds = [7, 8]
    imgs = [H.HeifImage.parse(permuted_heic(halfmoonbay, s)) for s in seeds]
    b = ctx.prepare(imgs)
    outs = [ctx.alloc_outputs(imgs) for _ in range(4)]
    for o in outs:
        b.decode_async(o)
    assert b.status() == [0, 0]
    for o in outs:
        for s, oi in zip(seeds, o):
            want = assemble(oracle_tiles, permutation(48, s))
            for got, w in zip(planes_np(oi), want):
                assert np.array_equal(got, w), s
    b.free()


def test_aux_gain_map_bit_exact(H, oracle_mod, halfmoonbay):
    """§8(f) row 4: the HDR gain map item (4:0:0 monochrome, RExt profile 4,
    2016x1520 coded, 48 WPP rows in one picture) through the same kernels."""
    aux = H.HeifImage.parse(halfmoonbay).info.aux_item_id
    out = H.HeicDecoder.decode(halfmoonbay, item_id=aux)
    assert out.cb is None and out.cr is None
    tiles, (ho, hl) = oracle_mod.list_tiles(halfmoonbay, aux)
    o, n = tiles[0]
    y, _, _ = oracle_mod.decode_tile(halfmoonbay[ho:ho + hl], halfmoonbay[o:o + n], 2016, 1512)
    assert np.array_equal(out.y.cpu().numpy().astype(np.uint16), y)


def test_rgb_rotated_matches_restatement(H, halfmoonbay):
    """§8(f) row 2: YCbCr -> RGB8 + irot on the GPU, exact against the numpy
    restatement of the same fixed-point arithmetic (tests/rgb_ref.py)."""
    import rgb_ref

    out = H.HeicDecoder.decode(halfmoonbay)
    inf = out.info
    rgb = H.HeicDecoder.context().to_rgb(out).cpu().numpy()
    assert rgb.shape == (4032, 3024, 3)  # irot 3: 4032x3024 stored, shown portrait
    want = rgb_ref.ycbcr_to_rgb(out.y.cpu().numpy(), out.cb.cpu().numpy(), out.cr.cpu().numpy(),
                                inf.matrix_coeffs, bool(inf.full_range), inf.rotation)
    assert np.array_equal(rgb, want)
    # the monochrome gain map: R = G = B
    aux = H.HeicDecoder.decode_rgb(halfmoonbay, item_id=inf.aux_item_id).cpu().numpy()
    assert aux.shape == (2016, 1512, 3) and (aux[..., 0] == aux[..., 2]).all()


@pytest.mark.parametrize("G", [2, 3, 8])
def test_tile_split_gather_bit_exact(H, ctx, oracle_halfmoonbay, halfmoonbay, G):
    """Row e2: one image split by grid tile over G "ranks" (here G batches on
    one device; on a node, one per GPU), each decoding tiles k % G == g into
    its own full-size planes, then gathered (heifgpu_gather_tiles) into one
    image: bit-exact with the oracle, and each rank wrote only its tiles."""
    img = H.HeifImage.parse(halfmoonbay)
    dst = ctx.alloc_outputs([img])[0]
    for t in (dst.y, dst.cb, dst.cr):
        t.fill_(0)
    for g in range(G):
        part = ctx.alloc_outputs([img])[0]
        for t in (part.y, part.cb, part.cr):
            t.fill_(0xA5)
        b = ctx.prepare([img], tile_stride=G, tile_offset=g)
        b.decode_async([part])
        assert b.status() == [0]
        b.free()
        y = part.y.cpu().numpy()
        for k in range(48):
            r, c = divmod(k, 8)
            win = y[512 * r:512 * (r + 1), 512 * c:512 * (c + 1)]
            ref = oracle_halfmoonbay.y[512 * r:512 * (r + 1), 512 * c:512 * (c + 1)]
            if k % G == g:
                assert np.array_equal(win, ref), (g, k)
            else:
                assert (win == 0xA5).all(), (g, k)
        ctx.gather_tiles(dst, part, G, g)
    torch.cuda.synchronize()
    y, cb, cr = planes_np(dst)
    assert np.array_equal(y, oracle_halfmoonbay.y)
    assert np.array_equal(cb, oracle_halfmoonbay.cb)
    assert np.array_equal(cr, oracle_halfmoonbay.cr)


def test_tile_subset_without_pictures(H, ctx, oracle_mod, halfmoonbay):
    """A subset that selects no picture (a 1x1 item, offset 1 of 2) decodes nothing and reports clean."""
    aux = H.HeifImage.parse(halfmoonbay, H.HeifImage.parse(halfmoonbay).info.aux_item_id)
    out = ctx.alloc_outputs([aux])[0]
    out.y.fill_(7)
    b = ctx.prepare([aux], tile_stride=2, tile_offset=1)
    b.decode_async([out])
    assert b.status() == [0]
    assert int((out.y != 7).sum()) == 0
    b.free()


def test_reloaded_batches_alternate(H, ctx, oracle_tiles, halfmoonbay):
    """f1: two batches reloaded in turn (heifgpu_batch_prepare_ex with a batch
    to reuse, uploads not waited for) while the other decodes; every load's
    planes exact, including a reload with more images (arena growth)."""
    from heif_amd.synthetic import permutation, permuted_heic

    loads = [[11], [12, 13], [14], [15, 16, 17], [18]]
    batches = [None, None]
    results = []
    for i, seeds in enumerate(loads):
        imgs = H.HeifImage.parse_many([permuted_heic(halfmoonbay, s) for s in seeds], threads=4)
        outs = ctx.alloc_outputs(imgs)
        batches[i % 2] = ctx.prepare(imgs, reuse=batches[i % 2], wait=False)
        batches[i % 2].decode_async(outs)
        results.append((seeds, outs))
    torch.cuda.synchronize()
    for seeds, outs in results:
        for s, o in zip(seeds, outs):
            want = assemble(oracle_tiles, permutation(48, s))
            for got, w in zip(planes_np(o), want):
                assert np.array_equal(got, w), s
    for b in batches:
        assert not any(b.status())
        b.free()


def test_rows_mode_removed(H, ctx, halfmoonbay):
    """HEIFGPU_PARSE_ROWS (ABI 5's row waves) is gone in ABI 6:
    prepare answers HEIFGPU_E_UNSUPPORTED and the batch is not created."""
    import ctypes

    from heif_amd import _lib

    img = H.HeifImage.parse(halfmoonbay)
    arr = (ctypes.c_void_p * 1)(img._h.value)
    opts = _lib.BatchOpts(1, 0, _lib.PARSE_ROWS, 0, 0)
    b = ctypes.c_void_p()
    rc = _lib.lib.heifgpu_batch_prepare_ex(ctx._h, arr, 1, ctypes.byref(opts), ctypes.byref(b))
    assert rc == _lib.HEIFGPU_E_UNSUPPORTED and not b.value
    assert "ABI 6" in _lib.last_error()
