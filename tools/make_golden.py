"""Regenerates tests/golden/halfmoonbay_planes.json from the CPU oracle.

The hashes pin the oracle's own output (regression guard for the oracle and
the GPU parity fixture); they are NOT independent evidence of pixel
correctness — no reference pixel decoder exists here (SURVEY.md §8(c):
pixels are "parity unpinned").

usage: python tools/make_golden.py
"""
import hashlib
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a.astype(np.uint8)).tobytes()).hexdigest()


def main():
    data = (ROOT / "tests/golden/halfmoonbay.heic").read_bytes()
    img = oracle.decode_heic(data)
    tiles, (ho, hl) = oracle.list_tiles(data)
    t0 = oracle.decode_tile(data[ho:ho + hl], data[tiles[0][0]:tiles[0][0] + tiles[0][1]], 512, 512)
    out = {
        "file": "halfmoonbay.heic",
        "generator": "tools/make_golden.py (CPU oracle, oracle/hevc_decode.c)",
        "planes": {"y": digest(img.y), "cb": digest(img.cb), "cr": digest(img.cr)},
        "shape": {"y": list(img.y.shape), "cb": list(img.cb.shape), "cr": list(img.cr.shape)},
        "tile0": {"y": digest(t0[0]), "cb": digest(t0[1]), "cr": digest(t0[2])},
        "substreams": len(img.checks),
        "substreams_terminated_ok": sum(1 for c in img.checks if c["term_ok"]),
        "bins": sum(c["bins"] for c in img.checks),
        "luma_mean": float(img.y.mean()),
    }
    path = ROOT / "tests/golden/halfmoonbay_planes.json"
    path.write_text(json.dumps(out, indent=2) + "\n")
    print(json.dumps(out, indent=2))


if __name__ == "__main__":
    main()
