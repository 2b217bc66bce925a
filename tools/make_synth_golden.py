"""Regenerates tests/golden/synth_planes.json: SHA-256 of two synthetic HEICs
(heif_amd/synth_encoder.py) and of the CPU oracle's planes for them
(little-endian uint16, Y then Cb then Cr).  Regression pin only: the
reference computes no pixels, so these hashes are "parity unpinned"."""
import hashlib
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from heif_amd import synth_encoder as S  # noqa: E402
from oracle import oracle  # noqa: E402

CASES = {
    "main10_grid_2x3": dict(out_w=1500, out_h=1000, seed=11,
                            params=dict(width=512, height=512, bit_depth=10, transform_skip=1, scaling_list=1)),
    "main8_grid_ctb16_mono": dict(out_w=400, out_h=300, seed=12,
                                  params=dict(width=256, height=160, chroma_format=0, log2_ctb=4, log2_max_tb=4,
                                              tq_bypass=1, diff_cu_qp_delta_depth=0)),
}


def main():
    out = {}
    for name, c in CASES.items():
        p = S.SynthParams(**c["params"])
        data = S.grid_heic(c["out_w"], c["out_h"], p, seed=c["seed"])
        img = oracle.decode_heic(data)
        assert all(k["term_ok"] for k in img.checks), name
        h = hashlib.sha256()
        for pl in (img.y, img.cb, img.cr):
            if pl is not None:
                h.update(pl.astype("<u2").tobytes())
        out[name] = dict(c, heic_sha256=hashlib.sha256(data).hexdigest(), planes_sha256=h.hexdigest())
    path = ROOT / "tests/golden/synth_planes.json"
    path.write_text(json.dumps(out, indent=2) + "\n")
    print(json.dumps(out, indent=2))


if __name__ == "__main__":
    main()
