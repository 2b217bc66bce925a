"""Split a tiled synthetic HEVC picture into one independent picture per tile
(test infrastructure only).

With loop_filter_across_tiles_enabled_flag = 0 nothing crosses a tile
boundary in an intra picture: CABAC contexts and the arithmetic decoder
restart at each tile (9.3.1), prediction availability stops at it (6.4.1),
qPY_PREV restarts at SliceQpY (8.6.1), SAO merge candidates (7.3.8.3),
deblocking (8.7.2) and SAO (8.7.3) do not reach across it.  A tile is then
the same picture as a stand-alone picture of the tile's size whose slice data
is the tile's substream.  This module builds those stand-alone pictures
directly from the bitstream (slice-header rewrite in Python, independent of
the host's C++ split in heif_amd/csrc/host/batch.cpp) so the oracle's
spec-literal tile decode can be checked against its untiled decode, which the
reference's own fixtures pin.
"""
from __future__ import annotations

import dataclasses
from typing import List, Tuple

from ps_writer import BitWriter, _ep


def _unescape(b: bytes) -> bytes:
    out, z = bytearray(), 0
    for x in b:
        if z >= 2 and x == 3:
            z = 0
            continue
        out.append(x)
        z = z + 1 if x == 0 else 0
    return bytes(out)


class _Reader:
    def __init__(self, b: bytes):
        self.b, self.pos = b, 0

    def u(self, n: int) -> int:
        v = 0
        for _ in range(n):
            v = (v << 1) | ((self.b[self.pos >> 3] >> (7 - (self.pos & 7))) & 1)
            self.pos += 1
        return v

    def ue(self) -> int:
        z = 0
        while self.u(1) == 0:
            z += 1
        return (1 << z) - 1 + self.u(z)

    def se(self) -> int:
        k = self.ue()
        return (k + 1) // 2 if k & 1 else -(k // 2)


def tile_bounds(n: int, total: int, uniform: int, explicit) -> List[int]:
    """6.5.1 (6-3 / 6-4): column or row boundaries in CTBs."""
    bd = [0]
    for i in range(n):
        sz = ((i + 1) * total) // n - (i * total) // n if uniform else (
            explicit[i] if i + 1 < n else total - bd[-1])
        bd.append(bd[-1] + sz)
    return bd


@dataclasses.dataclass
class SubPicture:
    x0: int                 # luma position in the (uncropped) tiled picture
    y0: int
    params: object          # SynthParams of the stand-alone picture
    nal: bytes              # its IDR NAL unit


def split_tiles(p, nal: bytes) -> List[SubPicture]:
    """p: the SynthParams the tiled picture was written with (with or without
    WPP; the slice header has no deblocking override and no loop-filter-across-
    slices flag, as hevc_synth.c writes it).  With WPP a tile's CTB rows are
    its substreams, and a tile alone is a WPP picture of the tile's size (9.3.1:
    a row syncs with the above-right CTB only inside its tile)."""
    rbsp = _unescape(nal[2:])
    r = _Reader(rbsp)
    assert r.u(1) == 1            # first_slice_segment_in_pic_flag
    r.u(1)                        # no_output_of_prior_pics_flag
    assert r.ue() == 0            # slice_pic_parameter_set_id
    assert r.ue() == 2            # I slice
    sao = []
    if p.sao:
        sao.append(r.u(1))
        if p.chroma_format:
            sao.append(r.u(1))
    qp_delta = r.se()
    n_entry = r.ue()
    offs = []
    if n_entry:
        ln = r.ue() + 1
        offs = [r.u(ln) + 1 for _ in range(n_entry)]
    assert r.u(1) == 1
    while r.pos & 7:
        assert r.u(1) == 0
    hdr_raw = len(_ep(rbsp[:r.pos >> 3]))  # the header ends in a nonzero byte: no EP state carries over
    starts = [2 + hdr_raw]
    for o in offs:
        starts.append(starts[-1] + o)
    starts.append(len(nal))
    ctb = 1 << p.log2_ctb
    wctb, hctb = -(-p.width // ctb), -(-p.height // ctb)
    cols = tile_bounds(p.tile_cols, wctb, p.tile_uniform, p.tile_col_w)
    rows = tile_bounds(p.tile_rows, hctb, p.tile_uniform, p.tile_row_h)
    # substreams in tile scan: one per tile, or with WPP one per CTB row of each tile
    nsub = [rows[k // p.tile_cols + 1] - rows[k // p.tile_cols] if p.wpp else 1
            for k in range(p.tile_cols * p.tile_rows)]
    assert len(starts) - 1 == sum(nsub)
    subs = []
    s0 = 0
    for k in range(p.tile_cols * p.tile_rows):
        tc, tr = k % p.tile_cols, k // p.tile_cols
        s1 = s0 + nsub[k]
        x0, y0 = cols[tc] * ctb, rows[tr] * ctb
        w = min(cols[tc + 1] * ctb, p.width) - x0
        h = min(rows[tr + 1] * ctb, p.height) - y0
        sp = dataclasses.replace(p, width=w, height=h, tile_cols=1, tile_rows=1, tile_uniform=1,
                                 tile_col_w=(), tile_row_h=(),
                                 conf_right=p.conf_right if tc == p.tile_cols - 1 else 0,
                                 conf_bottom=p.conf_bottom if tr == p.tile_rows - 1 else 0)
        hw = BitWriter()
        hw.u(1, 1)
        hw.u(0, 1)
        hw.ue(0)
        hw.ue(2)
        for f in sao:
            hw.u(f, 1)
        hw.se(qp_delta)
        if p.wpp:  # the tile's rows keep their sizes as the stand-alone picture's entry points
            lens = [starts[j + 1] - starts[j] for j in range(s0, s1 - 1)]
            hw.ue(len(lens))
            if lens:
                ln = max(1, (max(lens) - 1).bit_length())
                hw.ue(ln - 1)
                for n in lens:
                    hw.u(n - 1, ln)
        hw.trailing()
        sub_nal = nal[:2] + _ep(hw.bytes()) + nal[starts[s0]:starts[s1]]
        subs.append(SubPicture(x0, y0, sp, sub_nal))
        s0 = s1
    return subs


def assemble(p, subs: List[SubPicture], decode) -> Tuple:
    """decode(SubPicture) -> (y, cb, cr) of its cropped output; returns the
    tiled picture's cropped planes put together from them."""
    import numpy as np

    W, H = p.width - p.conf_right, p.height - p.conf_bottom
    y = np.zeros((H, W), np.uint16)
    sx, sy = int(p.chroma_format in (1, 2)), int(p.chroma_format == 1)  # log2 SubWidthC, SubHeightC
    c = [np.zeros(((H + sy) >> sy, (W + sx) >> sx), np.uint16) for _ in range(2)] if p.chroma_format else [None, None]
    for s in subs:
        py, pcb, pcr = decode(s)
        y[s.y0:s.y0 + py.shape[0], s.x0:s.x0 + py.shape[1]] = py
        if p.chroma_format:
            for dst, src in zip(c, (pcb, pcr)):
                dst[(s.y0 >> sy):(s.y0 >> sy) + src.shape[0], (s.x0 >> sx):(s.x0 >> sx) + src.shape[1]] = src
    return y, c[0], c[1]


def _nal_units(item: bytes) -> List[bytes]:
    out, pos = [], 0
    while pos < len(item):
        n = int.from_bytes(item[pos:pos + 4], "big")
        out.append(item[pos + 4:pos + 4 + n])
        pos += 4 + n
    return out


def split_slices(p, item: bytes) -> List[SubPicture]:
    """The slices of a picture written with p.slice_ctus a multiple of its
    width in CTBs (every slice a band of CTB rows, all independent, no tiles)
    as stand-alone pictures: each slice segment's header is rewritten without
    its address (first_slice_segment_in_pic_flag = 1), every other field and
    the slice data kept."""
    ctb = 1 << p.log2_ctb
    wctb, hctb = -(-p.width // ctb), -(-p.height // ctb)
    assert p.slice_ctus % wctb == 0 and not p.slice_dependent and p.tile_cols * p.tile_rows == 1
    nctb = wctb * hctb
    abits = (nctb - 1).bit_length()
    subs = []
    for k, nal in enumerate(_nal_units(item)):
        rbsp = _unescape(nal[2:])
        r = _Reader(rbsp)
        assert r.u(1) == (k == 0)
        r.u(1)
        assert r.ue() == 0
        addr = r.u(abits) if k else 0
        w = BitWriter()
        w.u(1, 1)
        w.u(0, 1)
        w.ue(0)
        # the rest of the header up to slice data: slice_type, SAO flags, QP delta,
        # deblocking override, filter-across flag, entry points (hevc_synth.c's order)
        slice_type = r.ue()
        w.ue(slice_type)
        sao = 0
        if p.sao:
            sao = r.u(1)
            w.u(sao, 1)
            if p.chroma_format:
                c = r.u(1)
                sao |= c
                w.u(c, 1)
        w.se(r.se())
        dis = p.deblock_disabled
        if p.slice_dbk_vary:
            ov = r.u(1)
            w.u(ov, 1)
            if ov:
                dis = r.u(1)
                w.u(dis, 1)
                if not dis:
                    w.se(r.se())
                    w.se(r.se())
        if p.slice_lf_across and (sao or not dis):
            w.u(r.u(1), 1)
        if p.wpp:
            n = r.ue()
            w.ue(n)
            if n:
                ln = r.ue()
                w.ue(ln)
                for _ in range(n):
                    w.u(r.u(ln + 1), ln + 1)
        assert r.u(1) == 1
        while r.pos & 7:
            assert r.u(1) == 0
        w.trailing()
        hdr_raw = len(_ep(rbsp[:r.pos >> 3]))
        y0 = addr // wctb * ctb
        h = min(y0 + p.slice_ctus // wctb * ctb, p.height) - y0
        last = y0 + h >= p.height
        sp = dataclasses.replace(p, height=h, slice_ctus=0, conf_bottom=p.conf_bottom if last else 0)
        subs.append(SubPicture(0, y0, sp, nal[:2] + _ep(w.bytes()) + nal[2 + hdr_raw:]))
    return subs
