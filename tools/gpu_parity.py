"""Quick GPU bring-up check: decode halfmoonbay on the GPU and diff against the oracle.

usage: python tools/gpu_parity.py [file.heic]
"""
import pathlib
import sys
import time

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import heif_amd as H  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else str(ROOT / "tests/golden/halfmoonbay.heic")
    data = open(path, "rb").read()
    t0 = time.time()
    ref = oracle.decode_heic(data)
    print(f"oracle {time.time() - t0:.2f}s")
    ctx = H.DecodeContext(0)
    img = H.HeifImage.parse(data)
    outs = ctx.alloc_outputs([img])
    batch = ctx.prepare([img])
    ctx.set_timing(True)
    batch.decode_async(outs)
    st = batch.status()
    print("status", st, "stage ms", ["%.3f" % x for x in ctx.stage_times()])
    ok = True
    for name, g, r in (("Y", outs[0].y, ref.y), ("Cb", outs[0].cb, ref.cb), ("Cr", outs[0].cr, ref.cr)):
        g = g.cpu().numpy().astype(np.int32)
        r = r.astype(np.int32)
        d = np.abs(g - r)
        bad = np.argwhere(d > 0)
        print(name, g.shape, "mismatches", len(bad), "max", d.max())
        if len(bad):
            ok = False
            y, x = bad[0]
            scale = 1 if name == "Y" else 2
            print("  first mismatch at", (y, x), "tile", (y * scale // 512, x * scale // 512), "gpu", g[y, x], "ref", r[y, x])
    # throughput on a repeated decode
    for k in range(3):
        batch.decode_async(outs)
        st2 = batch.status()
        if any(st2):
            print("repeat decode", k, "status", st2)
            ok = False
    torch.cuda.synchronize()
    t0 = time.time()
    n = 10
    for _ in range(n):
        batch.decode_async(outs)
    torch.cuda.synchronize()
    dt = (time.time() - t0) / n
    print(f"gpu decode {dt * 1e3:.2f} ms/image = {12192768 / dt / 1e6:.1f} Mpix/s; stages",
          ["%.3f" % x for x in ctx.stage_times()])
    print("PARITY", "OK" if ok else "FAIL")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
