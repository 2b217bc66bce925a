"""Synthetic HEIC batches.

Image *i* is a valid grid HEIC whose tile positions hold a permutation of a
source image's tile NAL units: the container is copied and only the order of
the grid item's ``dimg`` references (the ``iref`` box) is rewritten, so every
tile stays an independent IDR picture with the same SPS/PPS.  The permutation
is a Fisher–Yates shuffle driven by mt19937_64(seed = i); the draw for step k
is ``rng() % (k + 1)`` (documented here because std::shuffle's draw is
implementation-defined).
"""
from __future__ import annotations

import struct
from typing import List, Tuple


class MT19937_64:
    """Standard 64-bit Mersenne Twister (std::mt19937_64)."""

    N, M = 312, 156
    MATRIX_A = 0xB5026F5AA96619E9
    UM, LM = 0xFFFFFFFF80000000, 0x7FFFFFFF
    MASK = (1 << 64) - 1

    def __init__(self, seed: int):
        self.mt = [0] * self.N
        self.mt[0] = seed & self.MASK
        for i in range(1, self.N):
            self.mt[i] = (6364136223846793005 * (self.mt[i - 1] ^ (self.mt[i - 1] >> 62)) + i) & self.MASK
        self.mti = self.N

    def __call__(self) -> int:
        if self.mti >= self.N:
            mt = self.mt
            for i in range(self.N):
                x = (mt[i] & self.UM) | (mt[(i + 1) % self.N] & self.LM)
                xa = x >> 1
                if x & 1:
                    xa ^= self.MATRIX_A
                mt[i] = mt[(i + self.M) % self.N] ^ xa
            self.mti = 0
        x = self.mt[self.mti]
        self.mti += 1
        x ^= (x >> 29) & 0x5555555555555555
        x ^= (x << 17) & 0x71D67FFFEDA60000
        x ^= (x << 37) & 0xFFF7EEE000000000
        x ^= x >> 43
        return x & self.MASK


def permutation(n: int, seed: int) -> List[int]:
    rng = MT19937_64(seed)
    p = list(range(n))
    for k in range(n - 1, 0, -1):
        j = rng() % (k + 1)
        p[k], p[j] = p[j], p[k]
    return p


def _boxes(data: bytes, start: int, end: int):
    pos = start
    while pos + 8 <= end:
        size, typ = struct.unpack(">I4s", data[pos:pos + 8])
        hdr = 8
        if size == 1:
            size = struct.unpack(">Q", data[pos + 8:pos + 16])[0]
            hdr = 16
        elif size == 0:
            size = end - pos
        yield typ, pos, pos + hdr, pos + size
        pos += size


def find_dimg(data: bytes) -> Tuple[int, int, int]:
    """Returns (offset of the first to_item_ID, id byte width, count) of the
    primary grid's dimg reference."""
    primary = None
    for typ, _, p, e in _boxes(data, 0, len(data)):
        if typ != b"meta":
            continue
        for t2, _, p2, e2 in _boxes(data, p + 4, e):
            if t2 == b"pitm":
                primary = struct.unpack(">H", data[p2 + 4:p2 + 6])[0] if data[p2] == 0 else \
                    struct.unpack(">I", data[p2 + 4:p2 + 8])[0]
        for t2, _, p2, e2 in _boxes(data, p + 4, e):
            if t2 != b"iref":
                continue
            w = 2 if data[p2] == 0 else 4
            for t3, _, p3, e3 in _boxes(data, p2 + 4, e2):
                frm = int.from_bytes(data[p3:p3 + w], "big")
                cnt = struct.unpack(">H", data[p3 + w:p3 + w + 2])[0]
                if t3 == b"dimg" and frm == primary:
                    return p3 + w + 2, w, cnt
    raise ValueError("no dimg reference for the primary item")


def permuted_heic(src: bytes, seed: int) -> bytes:
    off, w, cnt = find_dimg(src)
    ids = [src[off + k * w: off + (k + 1) * w] for k in range(cnt)]
    perm = permutation(cnt, seed)
    out = bytearray(src)
    for k in range(cnt):
        out[off + k * w: off + (k + 1) * w] = ids[perm[k]]
    return bytes(out)
