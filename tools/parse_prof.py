"""k_parse cycle breakdown (tuning only).

usage: HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so python tools/parse_prof.py [n_images]

Decodes a batch of permuted halfmoonbay images with the counter-instrumented
library (`make -C heif_amd/csrc prof`) and prints the per-wave averages of
the k_parse counters (s_memtime cycles) and cycles per bin.
"""
import ctypes
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import heif_amd as H  # noqa: E402
from heif_amd import _lib  # noqa: E402
from heif_amd.synthetic import permuted_heic  # noqa: E402

NAMES = ["wave", "spin", "bins", "bypass", "refill", "cqt", "resid", "sao"]
# k_parse_lanes (HEIFGPU_PARSE=lanes): per-wave s_memtime cycles
LANES = ["l_wave", "l_passes", "l_ctu", "l_tree", "l_tb", "l_sb", "l_ctu_end", "l_refill"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    src = (ROOT / "tests/golden/halfmoonbay.heic").read_bytes()
    imgs = [H.HeifImage.parse(permuted_heic(src, s)) for s in range(n)]
    ctx = H.DecodeContext(0)
    outs = ctx.alloc_outputs(imgs)
    batch = ctx.prepare(imgs)
    ctx.set_timing(True)
    lib = _lib.lib
    buf = (ctypes.c_uint64 * 16)()
    batch.decode_async(outs)
    torch.cuda.synchronize()
    k = lib.heifgpu_debug_counters(buf, 16)
    if k <= 0:
        raise SystemExit("library has no counters: build with `make -C heif_amd/csrc prof` and set HEIFGPU_LIBRARY")
    batch.decode_async(outs)
    torch.cuda.synchronize()
    st = ctx.stage_times()
    lib.heifgpu_debug_counters(buf, 16)
    c = dict(zip(NAMES + LANES, buf[:k]))
    if c.get("l_passes"):
        print("k_parse_lanes totals:", {n: c[n] for n in LANES}, f"parse {ctx.stage_times()[0]:.3f} ms")
        return
    info = imgs[0].info
    rows = n * info.num_tiles * ((info.tile_height + 63) // 64)
    print(f"images {n}, waves(rows) {rows}, parse {st[0]:.3f} ms, status {batch.status()}")
    for name in NAMES:
        print(f"  {name:7s} total {c[name]:16d}  per wave {c[name] / rows:14.1f}")
    bins = c["bins"] + c["bypass"]
    busy = c["wave"] - c["spin"]
    print(f"  cycles/bin (busy) {busy / max(bins, 1):.1f}; cqt cycles/bin {c['cqt'] / max(bins, 1):.1f}; "
          f"spin share {c['spin'] / max(c['wave'], 1):.3f}")


if __name__ == "__main__":
    main()
