"""ctypes binding of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  The product (heif_amd/) never imports this.
See oracle/oracle.h for what the oracle restates and how it is pinned.
"""
from __future__ import annotations

import ctypes
import os
import pathlib
from dataclasses import dataclass

import numpy as np

_HERE = pathlib.Path(__file__).resolve().parent
# ORACLE_LIBRARY: another build of the same oracle (bench.py's cpu_baseline
# builds `make -C oracle native`, -march=native for the host it runs on)
LIB_PATH = pathlib.Path(os.environ.get("ORACLE_LIBRARY", _HERE / "build" / "liboracle.so"))


class _Meta(ctypes.Structure):
    _fields_ = [
        (n, ctypes.c_uint32)
        for n in (
            "primary_item_id", "ispe_width", "ispe_height", "width", "height", "rotation", "luma_bits",
            "chroma_bits", "num_thumbnails", "is_grid", "grid_rows", "grid_cols", "out_width",
            "out_height", "num_tiles", "tile_width", "tile_height", "chroma_format_idc",
        )
    ]


class _Image(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("chroma_format_idc", ctypes.c_uint32),
        ("bit_depth", ctypes.c_uint32), ("plane", ctypes.POINTER(ctypes.c_uint16) * 3),
        ("pw", ctypes.c_uint32 * 3), ("ph", ctypes.c_uint32 * 3),
    ]


class _Check(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("tile", "substream", "raw_start", "raw_entry", "term_ok", "bins")]


def _load():
    if not LIB_PATH.exists():
        raise ImportError(f"{LIB_PATH} missing: run `make -C oracle`")
    lib = ctypes.CDLL(str(LIB_PATH))
    P, SZ, I = ctypes.POINTER, ctypes.c_size_t, ctypes.c_int
    u8p = P(ctypes.c_uint8)
    lib.oracle_read_meta.argtypes = [u8p, SZ, P(_Meta)]
    lib.oracle_decode_heic.argtypes = [u8p, SZ, P(_Image), P(_Check), I, P(I)]
    lib.oracle_image_free.argtypes = [P(_Image)]
    lib.oracle_set_debug_flags.argtypes = [I]
    lib.oracle_chroma_tb_hist.argtypes = [P(ctypes.c_uint32), I]
    lib.oracle_last_error.restype = ctypes.c_char_p
    lib.oracle_remove_emulation_prevention.argtypes = [u8p, SZ, u8p]
    lib.oracle_remove_emulation_prevention.restype = SZ
    lib.oracle_read_ue.argtypes = [u8p, SZ, P(ctypes.c_uint32)]
    lib.oracle_read_se.argtypes = [u8p, SZ, P(ctypes.c_int32)]
    lib.oracle_decode_tr_bins.argtypes = [u8p, I, I, I, P(I)]
    lib.oracle_decode_chroma_mode_bins.argtypes = [u8p, I, P(I)]
    lib.oracle_decode_coeff_abs_level_remaining_bins.argtypes = [u8p, I, I, P(I)]
    lib.oracle_decode_tile.argtypes = [u8p, SZ, u8p, SZ, P(ctypes.c_uint16), I, P(ctypes.c_uint16), I,
                                       P(ctypes.c_uint16), I]
    lib.oracle_list_tiles.argtypes = [u8p, SZ, P(ctypes.c_uint32), P(ctypes.c_uint32), I,
                                      P(ctypes.c_uint32), P(ctypes.c_uint32)]
    lib.oracle_list_item_tiles.argtypes = [u8p, SZ, ctypes.c_uint32, P(ctypes.c_uint32), P(ctypes.c_uint32), I,
                                           P(ctypes.c_uint32), P(ctypes.c_uint32)]
    lib.oracle_aux_item.argtypes = [u8p, SZ]
    lib.oracle_aux_item.restype = ctypes.c_uint32
    return lib


lib = _load()


class OracleError(RuntimeError):
    pass


def _buf(data: bytes):
    return (ctypes.c_uint8 * max(len(data), 1)).from_buffer_copy(data or b"\0")


def last_error() -> str:
    return lib.oracle_last_error().decode()


def read_meta(data: bytes) -> dict:
    m = _Meta()
    if lib.oracle_read_meta(_buf(data), len(data), ctypes.byref(m)):
        raise OracleError(last_error())
    return {n: getattr(m, n) for n, _ in m._fields_}


@dataclass
class OracleImage:
    y: np.ndarray
    cb: np.ndarray | None
    cr: np.ndarray | None
    bit_depth: int
    checks: list


def decode_heic(data: bytes, with_checks: bool = True, debug_flags: int = 0) -> OracleImage:
    """debug_flags: oracle_set_debug_flags bits for this call (4: the picture
    may end like a non-last tile, see tests/hevc_tiles.py)."""
    img = _Image()
    maxc = 1 << 16
    checks = (_Check * maxc)() if with_checks else None
    nchk = ctypes.c_int(0)
    lib.oracle_set_debug_flags(debug_flags)
    try:
        rc = lib.oracle_decode_heic(_buf(data), len(data), ctypes.byref(img), checks, maxc if with_checks else 0,
                                    ctypes.byref(nchk))
    finally:
        lib.oracle_set_debug_flags(0)
    if rc:
        raise OracleError(last_error())
    try:
        planes = []
        for c in range(3):
            if not img.plane[c]:
                planes.append(None)
                continue
            n = img.pw[c] * img.ph[c]
            a = np.ctypeslib.as_array(img.plane[c], shape=(n,)).reshape(img.ph[c], img.pw[c]).copy()
            planes.append(a)
        ck = [{n: getattr(checks[i], n) for n, _ in _Check._fields_} for i in range(nchk.value)] if with_checks else []
        return OracleImage(planes[0], planes[1], planes[2], img.bit_depth, ck)
    finally:
        lib.oracle_image_free(ctypes.byref(img))


def aux_item(data: bytes) -> int:
    """Item ID of the primary image's first auxiliary image ('auxl'), 0 if none."""
    return int(lib.oracle_aux_item(_buf(data), len(data)))


def list_tiles(data: bytes, item_id: int = 0):
    """Coded pictures of an image item (0 = primary): [(offset, length)], (hvcC offset, length)."""
    off = (ctypes.c_uint32 * 4096)()
    ln = (ctypes.c_uint32 * 4096)()
    ho, hl = ctypes.c_uint32(), ctypes.c_uint32()
    n = lib.oracle_list_item_tiles(_buf(data), len(data), item_id, off, ln, 4096, ctypes.byref(ho), ctypes.byref(hl))
    if n < 0:
        raise OracleError(last_error())
    return [(off[i], ln[i]) for i in range(n)], (ho.value, hl.value)


def decode_tile(hvcc: bytes, item: bytes, width: int, height: int):
    """Decode one grid tile (one coded picture) → (Y, Cb, Cr) uint16 arrays."""
    y = np.zeros((height, width), np.uint16)
    cb = np.zeros(((height + 1) // 2, (width + 1) // 2), np.uint16)
    cr = np.zeros_like(cb)
    P = ctypes.POINTER(ctypes.c_uint16)
    rc = lib.oracle_decode_tile(_buf(hvcc), len(hvcc), _buf(item), len(item), y.ctypes.data_as(P), width,
                                cb.ctypes.data_as(P), cb.shape[1], cr.ctypes.data_as(P), cr.shape[1])
    if rc:
        raise OracleError(last_error())
    return y, cb, cr


def chroma_tb_hist(reset: bool = True) -> np.ndarray:
    """Counts of 4:2:0 chroma TBs decoded with debug flag 8, [log2 - 2][mode][cbf]."""
    out = (ctypes.c_uint32 * (2 * 35 * 2))()
    lib.oracle_chroma_tb_hist(out, 1 if reset else 0)
    return np.frombuffer(bytes(out), np.uint32).reshape(2, 35, 2).copy()
