"""Diagnostic: decode the same batch repeatedly (and after dirtying device
memory with another batch) and report mismatches against the oracle."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import heif_amd as H  # noqa: E402
from heif_amd.synthetic import permuted_heic  # noqa: E402
from oracle import oracle  # noqa: E402

data = (ROOT / "tests/golden/halfmoonbay.heic").read_bytes()
ref = oracle.decode_heic(data, with_checks=False)
ctx = H.DecodeContext(0)


def report(tag, o):
    for name, g, r in (("Y", o.y, ref.y), ("Cb", o.cb, ref.cb), ("Cr", o.cr, ref.cr)):
        g = g.cpu().numpy().astype(np.int32)
        bad = np.argwhere(g != r)
        if len(bad):
            y, x = bad[0]
            s = 1 if name == "Y" else 2
            tiles = sorted({(int(a) * s // 512, int(b) * s // 512) for a, b in bad[:: max(1, len(bad) // 2000)]})
            print(f"  {tag} {name}: {len(bad)} mismatches, first {(int(y), int(x))}, tiles {tiles[:12]}")
        else:
            print(f"  {tag} {name}: ok")


# dirty the allocator with a different batch first
if len(sys.argv) > 1 and sys.argv[1] == "dirty":
    imgs = [H.HeifImage.parse(permuted_heic(data, s)) for s in range(4)]
    outs = ctx.alloc_outputs(imgs)
    b = ctx.prepare(imgs)
    b.decode_async(outs)
    print("dirty batch status", b.status())
    b.free()
    del outs

img = H.HeifImage.parse(data)
outs = ctx.alloc_outputs([img])
b = ctx.prepare([img])
for k in range(4):
    for t in (outs[0].y, outs[0].cb, outs[0].cr):
        t.fill_(0)
    b.decode_async(outs)
    print("decode", k, "status", b.status())
    report(f"d{k}", outs[0])
