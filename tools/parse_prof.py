"""k_parse_lanes cycle breakdown (tuning only).

usage: HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so python tools/parse_prof.py [n_images] [out.json] [auto|lanes|solo]

Decodes a batch of permuted halfmoonbay images with the counter-instrumented
library (`make -C heif_amd/csrc prof`) and prints per-wave averages of the
k_parse_lanes counters (s_memtime cycles per unit kind, passes, lanes that
ran a unit), i.e. the mean active lanes per unit execution and per pass.
Solo mode (k_parse_solo, one substream per wave): "passes" and "units" both
count units run; the cycles no unit kind accounts for are the WPP waits and
the driver (window refill, dispatch).
"""
import ctypes
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import heif_amd as H  # noqa: E402
from heif_amd import _lib  # noqa: E402
from heif_amd.synthetic import permuted_heic  # noqa: E402

# slots of heifgpu_debug_counters (parse_lanes.hip g_prof_lanes), summed over waves
LANES = ["cycles", "passes", "ctu", "tree", "tb", "sb", "ctu_end", "units"]
BINS_PER_IMAGE = 15358022  # context + bypass + terminate bins of one halfmoonbay image (oracle count)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    mode = sys.argv[3] if len(sys.argv) > 3 else "auto"
    src = (ROOT / "tests/golden/halfmoonbay.heic").read_bytes()
    imgs = [H.HeifImage.parse(permuted_heic(src, s)) for s in range(n)]
    ctx = H.DecodeContext(0)
    outs = ctx.alloc_outputs(imgs)
    batch = ctx.prepare(imgs, parse=mode)
    geom = batch.parse_geometry()
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
    parse_ms = ctx.stage_times()[0]
    lib.heifgpu_debug_counters(buf, 16)
    waves = geom["workgroups"] * geom["waves_per_workgroup"]
    if "profsb" in str(_lib.LIB_PATH) and geom["mode"] == "lanes":
        # `make prof-sb`, lanes kernel: the unit kinds (slots 0-7) and the sub-block
        # unit's phases as the wave's time (slots 8-12, one lane per unit run)
        names = LANES + ["sb_head", "sb_sig", "sb_g1", "sb_rest", "sig_bins"]
        c = dict(zip(names, buf[:13]))
        sb = max(c["sb"], 1)
        res = {"images": n, "geometry": geom, "waves": waves, "parse_ms": round(parse_ms, 3),
               "per_wave": {k2: round(c[k2] / waves, 1) for k2 in names},
               "unit_cycle_share": {k2: round(c[k2] / max(c["cycles"], 1), 3) for k2 in ("ctu", "tree", "tb", "sb", "ctu_end")},
               "sb_phase_share": {k2: round(c[k2] / sb, 3) for k2 in ("sb_head", "sb_sig", "sb_g1", "sb_rest")},
               "sb_cycles_per_sig_bin_lane": round(c["sb_sig"] / max(c["sig_bins"], 1), 2),
               "note": "s_memtime cycles of the counter build; sb phases: header (coded_sub_block_flag, context "
                       "gather), sig_coeff_flag loop, greater1/2, signs + remainders + record store; the wave's "
                       "time (one lane accumulates per unit run); sig_bins summed over lanes"}
        print(json.dumps(res))
        if len(sys.argv) > 2:
            pathlib.Path(sys.argv[2]).write_text(json.dumps(res, indent=1) + "\n")
        return
    if "profsb" in str(_lib.LIB_PATH):  # `make prof-sb`: solo / spread sub-block phases
        names = ["cycles", "wait", "sb_head", "sb_sig", "sb_g1", "sb_rest", "sig_bins", "coefs", "driver"]
        c = dict(zip(names, buf[:9]))
        res = {"images": n, "geometry": geom, "waves": waves, "parse_ms": round(parse_ms, 3),
               "per_wave": {k2: round(c[k2] / waves, 1) for k2 in names},
               "share_of_cycles": {k2: round(c[k2] / max(c["cycles"], 1), 3) for k2 in names[1:6] + ["driver"]},
               "cycles_per_sig_bin": round(c["sb_sig"] / max(c["sig_bins"], 1), 1),
               "cycles_per_coef_g1": round(c["sb_g1"] / max(c["coefs"], 1), 1),
               "cycles_per_coef_rest": round(c["sb_rest"] / max(c["coefs"], 1), 1),
               "bins_per_wave": round(n * BINS_PER_IMAGE / waves, 1),
               "note": "s_memtime cycles; wait = iterations whose CTU could not start (WPP poll + sleep); driver = loop top to unit start of the units run; the rest is the units other than the sub-block"}
        print(json.dumps(res))
        if len(sys.argv) > 2:
            pathlib.Path(sys.argv[2]).write_text(json.dumps(res, indent=1) + "\n")
        return
    c = dict(zip(LANES, buf[:k]))
    res = {
        "images": n,
        "geometry": geom,
        "waves": waves,
        "parse_ms": round(parse_ms, 3),
        "per_wave": {name: round(c[name] / waves, 1) for name in LANES},
        "cycles_per_pass": round(c["cycles"] / max(c["passes"], 1), 1),
        "lanes_per_pass": round(c["units"] / max(c["passes"], 1), 2),
        "unit_cycle_share": {name: round(c[name] / max(c["cycles"], 1), 3)
                             for name in ("ctu", "tree", "tb", "sb", "ctu_end")},
        "bins_per_wave": round(n * BINS_PER_IMAGE / waves, 1),
        "unaccounted_share": round(1 - sum(c[k] for k in ("ctu", "tree", "tb", "sb", "ctu_end")) / max(c["cycles"], 1), 3),
        "note": "s_memtime shader cycles of the instrumented build (r06: the product's translation units and flags at -O3, parse +4 % over the product build at 128 images)",
    }
    print(json.dumps(res))
    if len(sys.argv) > 2:
        pathlib.Path(sys.argv[2]).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
