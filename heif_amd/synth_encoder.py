"""Synthetic HEVC-intra HEIC generator (Main-10 / 8K
grid, BASELINE config 5).  No 10-bit sample ships with the reference (its
tests/ hold only halfmoonbay.heic), so 10-bit and other-geometry inputs are
made here: ``libhevcsynth.so`` (heif_amd/csrc/synth/hevc_synth.c) draws every
H.265 I-slice syntax element from a seeded RNG and CABAC-encodes it, and this
module wraps the pictures in a HEIF grid container laid out like
halfmoonbay's (ftyp, meta{hdlr, pitm, iinf/infe v2, iref dimg, iprp{ipco
hvcC/ispe, ipma}, idat grid, iloc v1}, mdat; reference grammar:
src/heif/grammar.rs, reader.rs:33-57).

Data generator only: it is not on the decode path and the decoder never
loads it.
"""
from __future__ import annotations

import ctypes
import dataclasses
import pathlib
import struct
from typing import List, Optional, Tuple

_LIB_PATH = pathlib.Path(__file__).resolve().parent / "libhevcsynth.so"
_lib = None


class _Params(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "width", "height", "conf_right", "conf_bottom", "chroma_format", "bit_depth",
        "log2_ctb", "log2_min_cb", "log2_min_tb", "log2_max_tb", "max_th_depth_intra",
        "sign_hiding", "cu_qp_delta", "diff_cu_qp_delta_depth",
        "transform_skip", "tq_bypass", "scaling_list", "strong_intra",
        "init_qp", "slice_qp_delta", "cb_qp_offset", "cr_qp_offset",
        "sao", "deblock_disabled", "beta_offset_div2", "tc_offset_div2", "density", "wpp",
        "tile_cols", "tile_rows", "tile_uniform", "tile_lf_across")] + [
        ("tile_col_w", ctypes.c_int32 * 8), ("tile_row_h", ctypes.c_int32 * 8)] + [
        (n, ctypes.c_int32) for n in ("slice_ctus", "slice_dependent", "slice_lf_across", "slice_dbk_vary",
                                      "pcm", "pcm_bd_y", "pcm_bd_c", "pcm_log2_min", "pcm_log2_max",
                                      "pcm_lf_disabled", "pcm_pct")]


@dataclasses.dataclass
class SynthParams:
    """Coded-picture parameters (one HEIF tile).  Defaults: a 512x512 8-bit
    4:2:0 tile with CTB 32 / CB 8..32 / TB 4..32 like halfmoonbay's, plus the
    optional tools its stream does not use."""
    width: int = 512
    height: int = 512
    conf_right: int = 0
    conf_bottom: int = 0
    chroma_format: int = 1
    bit_depth: int = 8
    log2_ctb: int = 5
    log2_min_cb: int = 3
    log2_min_tb: int = 2
    log2_max_tb: int = 5
    max_th_depth_intra: int = 1
    sign_hiding: int = 1
    cu_qp_delta: int = 1
    diff_cu_qp_delta_depth: int = 1
    transform_skip: int = 0
    tq_bypass: int = 0
    scaling_list: int = 0
    strong_intra: int = 1
    init_qp: int = 26
    slice_qp_delta: int = 0
    cb_qp_offset: int = 0
    cr_qp_offset: int = 0
    sao: int = 1
    deblock_disabled: int = 0
    beta_offset_div2: int = 0
    tc_offset_div2: int = 0
    density: int = 35
    wpp: int = 1  # entropy_coding_sync_enabled_flag (0: one CABAC substream per picture, BASELINE config 2)
    # HEVC tiles inside the picture (tiles_enabled_flag when tile_cols * tile_rows > 1; needs wpp=0)
    tile_cols: int = 1
    tile_rows: int = 1
    tile_uniform: int = 1
    tile_lf_across: int = 0          # loop_filter_across_tiles_enabled_flag
    tile_col_w: Tuple[int, ...] = ()  # explicit widths / heights in CTBs (all but the last), tile_uniform=0
    tile_row_h: Tuple[int, ...] = ()

    # slice segments (see hevc_synth.h): CTUs per segment (0 = one), dependent
    # segments (1 all after the first, 2 odd-numbered), loop filter across
    # slices (0 none, 1 all, 2 even-numbered slices), per-slice deblocking override
    slice_ctus: int = 0
    slice_dependent: int = 0
    slice_lf_across: int = 0
    slice_dbk_vary: int = 0
    # PCM coding units (see hevc_synth.h): enable, sample bit depths, CU sizes, loop filter off, probability
    pcm: int = 0
    pcm_bd_y: int = 8
    pcm_bd_c: int = 8
    pcm_log2_min: int = 3
    pcm_log2_max: int = 5
    pcm_lf_disabled: int = 0
    pcm_pct: int = 10

    def _c(self) -> _Params:
        c = _Params()
        for n, t in _Params._fields_:
            if t is ctypes.c_int32:
                setattr(c, n, getattr(self, n))
        for name in ("tile_col_w", "tile_row_h"):
            v = list(getattr(self, name))
            if len(v) > 8:
                raise ValueError(f"{name}: at most 8 entries")
            getattr(c, name)[:len(v)] = v
        return c


def _load():
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            raise RuntimeError(f"{_LIB_PATH} missing: run `make -C heif_amd/csrc synth`")
        lib = ctypes.CDLL(str(_LIB_PATH))
        for f in ("synth_vps", "synth_sps", "synth_pps"):
            getattr(lib, f).restype = ctypes.c_long
            getattr(lib, f).argtypes = [ctypes.POINTER(_Params), ctypes.c_void_p, ctypes.c_size_t]
        for f in ("synth_picture", "synth_picture_item"):
            getattr(lib, f).restype = ctypes.c_long
            getattr(lib, f).argtypes = [ctypes.POINTER(_Params), ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t]
        lib.synth_check_params.restype = ctypes.c_int
        lib.synth_check_params.argtypes = [ctypes.POINTER(_Params)]
        _lib = lib
    return _lib


def _call(fn, p: SynthParams, *args, cap: int) -> bytes:
    buf = ctypes.create_string_buffer(cap)
    cp = p._c()
    n = fn(ctypes.byref(cp), *args, buf, cap)
    if n < 0:
        raise ValueError(f"{fn.__name__} failed ({n}) for {p}")
    return buf.raw[:n]


def parameter_sets(p: SynthParams) -> Tuple[bytes, bytes, bytes]:
    lib = _load()
    return (_call(lib.synth_vps, p, cap=256), _call(lib.synth_sps, p, cap=512), _call(lib.synth_pps, p, cap=256))


def picture(p: SynthParams, seed: int) -> bytes:
    """One IDR NAL unit (2-byte header included); single-segment pictures."""
    lib = _load()
    # worst case: dense 32x32 blocks with long level tails
    cap = max(1 << 16, p.width * p.height * 8)
    return _call(lib.synth_picture, p, ctypes.c_uint64(seed), cap=cap)


def picture_item(p: SynthParams, seed: int) -> bytes:
    """The picture's slice segments as 4-byte-length-prefixed IDR NAL units
    (a HEIF coded image item's payload)."""
    lib = _load()
    cap = max(1 << 16, p.width * p.height * 8)
    return _call(lib.synth_picture_item, p, ctypes.c_uint64(seed), cap=cap)


# ---------------------------------------------------------------- HEIF boxes
def _box(typ: bytes, payload: bytes) -> bytes:
    return struct.pack(">I4s", 8 + len(payload), typ) + payload


def _fbox(typ: bytes, version: int, flags: int, payload: bytes) -> bytes:
    return _box(typ, struct.pack(">I", (version << 24) | flags) + payload)


def _unescape(b: bytes) -> bytes:
    out, z = bytearray(), 0
    for x in b:
        if z >= 2 and x == 3:
            z = 0
            continue
        out.append(x)
        z = z + 1 if x == 0 else 0
    return bytes(out)


def hvcc(p: SynthParams, vps: bytes, sps: bytes, pps: bytes) -> bytes:
    """HEVCDecoderConfigurationRecord (ISO/IEC 14496-15 8.3.3.1); the
    profile/level bytes are copied from the SPS's profile_tier_level."""
    # SPS: 2-byte NAL header, 1 byte (vps id / max sub layers / nesting), then
    # 12 bytes of general profile/tier/level (read from the RBSP: its zero
    # compatibility/constraint bytes can carry emulation prevention).
    ptl = _unescape(sps[2:])[1:13]
    rec = bytes([1]) + ptl[:1] + ptl[1:5] + ptl[5:11] + ptl[11:12]
    par = 3 if p.wpp else 2 if p.tile_cols * p.tile_rows > 1 else 0  # parallelismType: 3 wavefront, 2 tiles
    rec += struct.pack(">H", 0xF000) + bytes([0xFC | par])  # min_spatial_segmentation, parallelism
    rec += bytes([0xFC | p.chroma_format, 0xF8 | (p.bit_depth - 8), 0xF8 | (p.bit_depth - 8)])
    rec += struct.pack(">H", 0) + bytes([0x0F])                     # avgFrameRate, 1 layer, nested, 4-byte lengths
    arrays = b""
    for typ, nal in ((32, vps), (33, sps), (34, pps)):
        arrays += bytes([0x80 | typ]) + struct.pack(">HH", 1, len(nal)) + nal
    return _box(b"hvcC", rec + bytes([3]) + arrays)


def _ispe(w: int, h: int) -> bytes:
    return _fbox(b"ispe", 0, 0, struct.pack(">II", w, h))


@dataclasses.dataclass
class BoxLayout:
    """Container variants the reference's reader gets wrong or leaves todo!()
    (src/heif/reader.rs): items split into several iloc extents (:47), infe
    version 0/1 entries (:303), unknown ipco properties ahead of the known
    ones (:460-463 drops them, shifting ipma indices), 16-bit ipma indices
    (flags & 1, :496-500), and the iloc field widths / base offset (for the
    overflow cases of the host's bounds checks)."""
    extents: int = 1            # iloc extents per mdat item (data split evenly)
    legacy_infe_items: int = 0  # extra metadata items declared with infe version 0 / 1 (alternating)
    unknown_props: int = 0      # unknown property boxes inserted at the front of ipco
    ipma_16bit: bool = False    # ipma flags & 1: 15-bit property indices
    offset_size: int = 4        # iloc offset_size / length_size / base_offset_size (bytes)
    length_size: int = 4
    base_offset_size: int = 0
    base_offset: int = 0        # added to every mdat extent offset (iloc base_offset)
    first_extent_offset: Optional[int] = None  # raw value written for the first mdat extent's offset (corruption)


def _be(v: int, n: int) -> bytes:
    return (v & ((1 << (8 * n)) - 1)).to_bytes(n, "big") if n else b""


def _assemble(items: List[Tuple[int, bytes, bytes]], primary: int, props: List[bytes],
              assoc: List[Tuple[int, List[int]]], iref: bytes, idat: bytes,
              layout: Optional[BoxLayout] = None) -> bytes:
    """items: (item_id, item_type, data); data of 'grid' items lives in idat
    (construction_method 1), everything else in mdat."""
    L = layout or BoxLayout()
    ftyp = _box(b"ftyp", b"heic" + struct.pack(">I", 0) + b"mif1heic")
    hdlr = _fbox(b"hdlr", 0, 0, struct.pack(">I", 0) + b"pict" + bytes(12) + b"\0")
    pitm = _fbox(b"pitm", 0, 0, struct.pack(">H", primary))
    infes = b"".join(_fbox(b"infe", 2, 0, struct.pack(">HH", iid, 0) + typ + b"\0") for iid, typ, _ in items)
    # ISO/IEC 14496-12 8.11.6 infe v0 / v1: item_ID, protection index, item_name,
    # content_type, content_encoding (+ v1: extension_type); no item_type.  HEIF
    # image items need v2+, so these are metadata items the reader must skip.
    base_id = max(iid for iid, _, _ in items) + 1
    legacy = [(base_id + k, b"legacy-%d" % k) for k in range(L.legacy_infe_items)]
    for k, (iid, name) in enumerate(legacy):
        v = k & 1
        infes += _fbox(b"infe", v, 0, struct.pack(">HH", iid, 0) + name + b"\0application/octet-stream\0\0" +
                       (b"fdel" if v else b""))
        items = items + [(iid, b"meta", b"\x00" * (16 + k))]
    iinf = _fbox(b"iinf", 0, 0, struct.pack(">H", len(items)) + infes)
    unknown = [_box(b"zzz%d" % (k % 10), bytes(4 + k)) for k in range(L.unknown_props)]
    ipco = _box(b"ipco", b"".join(unknown + props))
    shift = L.unknown_props
    ipma_p = struct.pack(">I", len(assoc))
    for iid, idxs in assoc:
        ipma_p += struct.pack(">HB", iid, len(idxs))
        if L.ipma_16bit:
            ipma_p += b"".join(struct.pack(">H", 0x8000 | (i + shift)) for i in idxs)
        else:
            ipma_p += bytes(0x80 | (i + shift) for i in idxs)
    iprp = _box(b"iprp", ipco + _fbox(b"ipma", 0, 1 if L.ipma_16bit else 0, ipma_p))
    idat_box = _box(b"idat", idat) if idat else b""

    def build(mdat_start: int) -> Tuple[bytes, bytes]:
        os_, ls_, bs_ = L.offset_size, L.length_size, L.base_offset_size
        ent = struct.pack(">BBH", (os_ << 4) | ls_, bs_ << 4, len(items))
        off = mdat_start
        body = b""
        for iid, typ, data in items:
            if typ == b"grid":
                ent += struct.pack(">HHH", iid, 1, 0) + _be(0, bs_) + struct.pack(">H", 1) + _be(0, os_) + \
                    _be(len(data), ls_)
            else:
                n = max(1, min(L.extents, len(data)))
                cuts = [len(data) * k // n for k in range(n + 1)]
                ent += struct.pack(">HHH", iid, 0, 0) + _be(L.base_offset, bs_) + struct.pack(">H", n)
                for k in range(n):
                    eo = off + cuts[k] - L.base_offset
                    if L.first_extent_offset is not None and off == mdat_start and k == 0:
                        eo = L.first_extent_offset
                    ent += _be(eo, os_) + _be(cuts[k + 1] - cuts[k], ls_)
                off += len(data)
                body += data
        iloc = _fbox(b"iloc", 1, 0, ent)
        meta = _fbox(b"meta", 0, 0, hdlr + pitm + iinf + iref + iprp + idat_box + iloc)
        return meta, body

    meta, _ = build(0)
    mdat_start = len(ftyp) + len(meta) + 8
    meta, body = build(mdat_start)
    return ftyp + meta + _box(b"mdat", body)


def _len_prefixed(nal: bytes) -> bytes:
    return struct.pack(">I", len(nal)) + nal


def grid_heic(out_w: int, out_h: int, p: SynthParams, seed: int = 0, pictures: Optional[List[bytes]] = None,
              layout: Optional[BoxLayout] = None) -> bytes:
    """A grid HEIC of ceil(out_w/W) x ceil(out_h/H) synthetic tiles of p's
    size, tile k drawn with seed (seed << 16) + k."""
    cols = -(-out_w // (p.width - p.conf_right))
    rows = -(-out_h // (p.height - p.conf_bottom))
    n = rows * cols
    if pictures is None:
        items_data = [picture_item(p, (seed << 16) + k) for k in range(n)]
    else:
        items_data = [_len_prefixed(pic) for pic in pictures]
    vps, sps, pps = parameter_sets(p)
    props = [hvcc(p, vps, sps, pps), _ispe(p.width - p.conf_right, p.height - p.conf_bottom), _ispe(out_w, out_h)]
    grid_id = 1
    items = [(grid_id, b"grid", struct.pack(">BBBBHH", 0, 0, rows - 1, cols - 1, out_w, out_h))]
    for k in range(n):
        items.append((k + 2, b"hvc1", items_data[k]))
    assoc = [(grid_id, [3])] + [(k + 2, [1, 2]) for k in range(n)]
    iref = _fbox(b"iref", 0, 0, _box(b"dimg", struct.pack(">HH", grid_id, n) +
                                     b"".join(struct.pack(">H", k + 2) for k in range(n))))
    return _assemble(items, grid_id, props, assoc, iref, items[0][2], layout)


def single_heic(p: SynthParams, seed: int = 0, layout: Optional[BoxLayout] = None,
                param_sets: Optional[Tuple[bytes, bytes, bytes]] = None, nal: Optional[bytes] = None) -> bytes:
    """A single-item (non-grid) HEIC holding one synthetic picture.
    param_sets / nal replace the generated VPS/SPS/PPS / picture NAL unit
    (robustness tests hand-craft out-of-range parameter sets)."""
    vps, sps, pps = param_sets or parameter_sets(p)
    props = [hvcc(p, vps, sps, pps), _ispe(p.width - p.conf_right, p.height - p.conf_bottom)]
    items = [(1, b"hvc1", _len_prefixed(nal) if nal is not None else picture_item(p, seed))]
    return _assemble(items, 1, props, [(1, [1, 2])], b"", b"", layout)


# BASELINE config 5: 8K 10-bit Main-10 grid, 15 x 9 tiles of 512x512
CONFIG5 = dict(out_w=7680, out_h=4320, params=SynthParams(bit_depth=10))
# Control workload of config-4 geometry whose 48 grid tiles are all distinct
# bitstreams (the bench's halfmoonbay permutations repeat 48 tiles): 8-bit
# 4:2:0 512x512 WPP tiles, sig_coeff_flag density cycling over 0..100 % so the
# payloads run from ~8 to ~45 KB (halfmoonbay's tiles: 1.4 to 76 KB)
CONFIG4U = dict(out_w=4032, out_h=3024, params=SynthParams(bit_depth=8))


def config4u_tile(j: int) -> bytes:
    """Distinct tile j of the CONFIG4U workload (seed and density from j)."""
    p = dataclasses.replace(CONFIG4U["params"], density=(j * 37 + 11) % 101)
    return picture(p, (1 << 24) + j)


def config4u_image(seed: int, threads: int = 1) -> bytes:
    """Image `seed` of the CONFIG4U workload: tiles 48*seed .. 48*seed+47."""
    import concurrent.futures as cf

    js = range(48 * seed, 48 * seed + 48)
    if threads > 1:  # (ctypes releases the GIL inside the generator)
        with cf.ThreadPoolExecutor(threads) as ex:
            pics = list(ex.map(config4u_tile, js))
    else:
        pics = [config4u_tile(j) for j in js]
    return grid_heic(CONFIG4U["out_w"], CONFIG4U["out_h"], CONFIG4U["params"], pictures=pics)
