"""Feasibility probe for a mixed parse (tuning only): two decode contexts, one
batch parsed by the spread engine (scalar unit), one by the lanes engine
(vector unit), decoded alone and side by side.  Prints wall ms per decode.

usage: python tools/mixed_parse.py [n_spread n_lanes lanes_ppw] ...
"""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import heif_amd as H  # noqa: E402
from heif_amd.synthetic import permuted_heic  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) * 1e3)
    return best


def main():
    src = (ROOT / "tests/golden/halfmoonbay.heic").read_bytes()
    combos = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]] or [(16, 16, 1), (24, 8, 1), (32, 16, 1)]
    need = max(a + b for a, b, _ in combos)
    imgs = [H.HeifImage.parse(permuted_heic(src, s)) for s in range(need)]
    ca, cb = H.DecodeContext(0), H.DecodeContext(0)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for ns, nl, ppw in combos:
        A, B = imgs[:ns], imgs[ns:ns + nl]
        oa, ob = ca.alloc_outputs(A), cb.alloc_outputs(B)
        ba = ca.prepare(A, parse="spread")
        bb = cb.prepare(B, parse="lanes", pics_per_wave=ppw)
        ta = timed(lambda: ba.decode_async(oa, sa.cuda_stream))
        tb = timed(lambda: bb.decode_async(ob, sb.cuda_stream))

        def both():
            ba.decode_async(oa, sa.cuda_stream)
            bb.decode_async(ob, sb.cuda_stream)
        tab = timed(both)
        print(f"spread {ns:3d} img alone {ta:7.2f} ms | lanes {nl:3d} img (ppw {ppw}, {bb.parse_geometry()['workgroups']} waves)"
              f" alone {tb:7.2f} ms | side by side {tab:7.2f} ms -> {(ns + nl) * 12192768 / tab / 1e3:8.1f} Mpix/s"
              f" (max of alone {max(ta, tb):7.2f})", flush=True)
        assert not any(ba.status()) and not any(bb.status())
        ba.free()
        bb.free()


if __name__ == "__main__":
    main()
