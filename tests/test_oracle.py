"""The CPU oracle pinned as far as anything here can pin it.

- every one of the 768 WPP substreams of halfmoonbay ends exactly at its
  entry point with end_of_subset_one_bit / end_of_slice_segment_flag = 1
  (any syntax, context-selection or engine error desynchronises CABAC and
  fails this almost surely);
- the decoded planes equal the committed hashes (tools/make_golden.py):
  a regression guard, not independent pixel evidence (pixels are parity
  unpinned: the reference cannot reconstruct pixels and libheif is absent).
"""
import hashlib
import json

import numpy as np

from conftest import GOLDEN


def _digest(a):
    return hashlib.sha256(np.ascontiguousarray(a.astype(np.uint8)).tobytes()).hexdigest()


def test_all_substreams_terminate_at_entry_points(oracle_halfmoonbay):
    ck = oracle_halfmoonbay.checks
    assert len(ck) == 48 * 16
    bad = [c for c in ck if not c["term_ok"]]
    assert not bad, bad[:3]
    # every substream starts exactly where the slice header says it does
    assert all(c["raw_start"] == c["raw_entry"] for c in ck)


def test_planes_match_golden_hashes(oracle_halfmoonbay):
    g = json.loads((GOLDEN / "halfmoonbay_planes.json").read_text())
    img = oracle_halfmoonbay
    assert list(img.y.shape) == g["shape"]["y"] == [3024, 4032]
    assert list(img.cb.shape) == g["shape"]["cb"] == [1512, 2016]
    assert _digest(img.y) == g["planes"]["y"]
    assert _digest(img.cb) == g["planes"]["cb"]
    assert _digest(img.cr) == g["planes"]["cr"]
    assert sum(c["bins"] for c in img.checks) == g["bins"]


def test_single_tile_matches_grid_placement(oracle_mod, halfmoonbay, oracle_halfmoonbay):
    tiles, (ho, hl) = oracle_mod.list_tiles(halfmoonbay)
    assert len(tiles) == 48
    hvcc = halfmoonbay[ho:ho + hl]
    for k in (0, 13, 47):
        o, n = tiles[k]
        y, cb, cr = oracle_mod.decode_tile(hvcc, halfmoonbay[o:o + n], 512, 512)
        r, c = divmod(k, 8)
        h = min(512, 3024 - 512 * r)
        w = min(512, 4032 - 512 * c)
        assert np.array_equal(oracle_halfmoonbay.y[512 * r:512 * r + h, 512 * c:512 * c + w], y[:h, :w])
        assert np.array_equal(oracle_halfmoonbay.cb[256 * r:256 * r + h // 2, 256 * c:256 * c + w // 2],
                              cb[:h // 2, :w // 2])


def test_sample_range(oracle_halfmoonbay):
    for p in (oracle_halfmoonbay.y, oracle_halfmoonbay.cb, oracle_halfmoonbay.cr):
        assert p.max() <= 255
