"""Per-wave times of k_parse_lanes (tuning only).

usage: HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so python tools/wave_times.py [n_images] [out.json] [ppw]

The counter build (`make -C heif_amd/csrc prof`) records, per lanes wave,
s_memrealtime (100 MHz, one clock for the chip) at its start, its duration,
where it ran (SIMD / CU / SE / XCD), its passes and its first three pictures.
This prints how the waves' end times spread (the kernel ends with its last
wave), the passes and times of every wave composition (source tiles of the
permuted halfmoonbay batch) and which waves shared a SIMD.
"""
import collections
import ctypes
import json
import os
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import heif_amd as H  # noqa: E402
from heif_amd import _lib  # noqa: E402
from heif_amd.synthetic import permutation, permuted_heic  # noqa: E402


# parse_lanes.hip kWaveRec / kWaveRecCap: the records of each wave's own breakdown
WAVE_REC, WAVE_REC_CAP = 4096, 4096
KINDS = ["ctu", "cqt", "cu", "tt", "tb", "sb", "ctu_end"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    ppw = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    src = (ROOT / "tests/golden/halfmoonbay.heic").read_bytes()
    imgs = [H.HeifImage.parse(permuted_heic(src, s)) for s in range(n)]
    ntiles = imgs[0].info.num_tiles
    ctx = H.DecodeContext(0)
    outs = ctx.alloc_outputs(imgs)
    batch = ctx.prepare(imgs, parse="lanes", pics_per_wave=ppw)
    geom = batch.parse_geometry()
    waves = geom["workgroups"]
    lib = _lib.lib
    sb = "profsb" in str(_lib.LIB_PATH)  # `make prof-sb`: 16 counter slots, the sub-block phases per wave
    o = 16 if sb else 8
    m = o + 3 * (WAVE_REC + 5 * WAVE_REC_CAP)
    buf = (ctypes.c_uint64 * m)()
    ctx.set_timing(True)
    batch.decode_async(outs)
    torch.cuda.synchronize()
    if lib.heifgpu_debug_counters(buf, m) <= 0:
        raise SystemExit("library has no counters: build with `make -C heif_amd/csrc prof`")
    reps = []
    for _ in range(3):  # the measured decodes (nothing else in flight)
        batch.decode_async(outs)
        torch.cuda.synchronize()
        reps.append(ctx.stage_times()[0])
        lib.heifgpu_debug_counters(buf, m)  # (the last decode's records stay in buf)
    perms = {}

    def src_tile(p):
        s, k = divmod(p, ntiles)
        if s not in perms:
            perms[s] = permutation(ntiles, s)
        return perms[s][k]

    rec = []
    for w in range(waves):
        t0, x1, x = buf[o + 3 * w], buf[o + 1 + 3 * w], buf[o + 2 + 3 * w]
        dur, place = x1 & 0xffffffff, x1 >> 32
        pics = [p for p in ((x >> s) & 0xffff for s in (16, 32, 48)) if p != 0xffff]
        hw = place & 0xffff
        rec.append({"t0": t0, "dur": dur / 1e5, "passes": x & 0xffff, "tiles": [src_tile(p) for p in pics],
                    "simd": (place >> 16 & 0xf, hw >> 13 & 7, hw >> 12 & 1, hw >> 8 & 15, hw >> 4 & 3)})
    for w, r in enumerate(rec):
        if w >= WAVE_REC_CAP:
            break
        b = [buf[o + 3 * (WAVE_REC + j * WAVE_REC_CAP + w) + i] for j in range(5) for i in range(3)]
        if b[0] == 0:
            continue
        kc = [(b[7] >> s) & 0xffff for s in (0, 16, 32, 48)] + [(b[8] >> s) & 0xffff for s in (0, 16, 32)]
        r["cycles"] = {"wave": b[0], "ctu": b[1], "tree": b[2], "tb": b[3], "sb": b[4], "ctu_end": b[5],
                       "pass_start": b[6]}
        r["kind_passes"] = dict(zip(KINDS, kc))
        r["lane_units"] = 4 * (b[8] >> 48)
        if sb:  # header, sig loop, greater1/2, signs + remainders + record (cycles, one lane per run), sig bins
            r["sb_phases"] = dict(zip(["head", "sig", "g1g2", "rest", "sig_bins"], b[9:14]))
    base = min(r["t0"] for r in rec)
    for r in rec:
        r["end"] = (r["t0"] - base) / 1e5 + r["dur"]
    q = sorted(r["end"] for r in rec)
    pct = {f"p{p}": round(q[min(len(q) - 1, int(p / 100 * len(q)))], 3) for p in (0, 10, 50, 90, 99, 100)}
    comp = {}
    for r in rec:
        comp.setdefault(tuple(r["tiles"]), []).append(r)
    by_comp = sorted(((k, v) for k, v in comp.items()), key=lambda kv: -statistics.mean(r["end"] for r in kv[1]))
    simds = {}
    for w, r in enumerate(rec):
        simds.setdefault(r["simd"], []).append(w)
    pairs = {}
    for ws in simds.values():
        key = tuple(sorted(tuple(rec[w]["tiles"]) for w in ws))
        pairs[key] = pairs.get(key, 0) + 1
    res = {
        "images": n, "geometry": geom, "waves": waves, "parse_ms_hip_events": [round(x, 3) for x in reps],
        "env": {k: v for k, v in os.environ.items() if k.startswith("HEIFGPU_")},
        "wave_end_ms": pct,
        "passes": {"min": min(r["passes"] for r in rec), "mean": round(statistics.mean(r["passes"] for r in rec), 1),
                   "max": max(r["passes"] for r in rec)},
        "waves_per_simd": {str(k): sum(1 for v in simds.values() if len(v) == k) for k in (1, 2, 3, 4)},
        "compositions": [{"tiles": list(k), "waves": len(v), "passes": v[0]["passes"],
                          "end_ms_mean": round(statistics.mean(r["end"] for r in v), 3),
                          "end_ms_max": round(max(r["end"] for r in v), 3),
                          "dur_ms_mean": round(statistics.mean(r["dur"] for r in v), 3),
                          "us_per_pass": round(1e3 * statistics.mean(r["dur"] for r in v) / max(v[0]["passes"], 1), 3)}
                         for k, v in by_comp],
        # wave-index offsets of the waves sharing a SIMD (the dispatcher's pairing rule)
        "simd_pair_offsets": dict(sorted(collections.Counter(
            max(ws) - min(ws) for ws in simds.values() if len(ws) == 2).most_common(8))),
        "simd_pairs_top": [{"pair": [list(t) for t in k], "simds": c} for k, c in
                           sorted(pairs.items(), key=lambda kv: -kv[1])[:40]],
        # the 8 waves ending last and 8 around the median: their own s_memtime
        # breakdown (cycles per unit kind group, pass starts) and the passes that
        # ran each unit kind, i.e. the cycles per run of each kind
        "slowest": [breakdown(r) for r in sorted(rec, key=lambda r: -r["end"])[:8] if "cycles" in r],
        "median": [breakdown(r) for r in sorted(rec, key=lambda r: r["end"])[len(rec) // 2 - 4:len(rec) // 2 + 4]
                   if "cycles" in r],
        "note": "s_memrealtime 100 MHz; tiles = source tiles of the wave's pictures (dealing order)",
    }
    print(json.dumps({k: res[k] for k in ("wave_end_ms", "passes", "parse_ms_hip_events", "waves_per_simd",
                                          "simd_pair_offsets")}))
    if len(sys.argv) > 2:
        pathlib.Path(sys.argv[2]).write_text(json.dumps(res, indent=1) + "\n")


def breakdown(r):
    c, kp = r["cycles"], r["kind_passes"]
    runs = {"ctu": kp["ctu"], "tree": kp["cqt"] + kp["cu"] + kp["tt"], "tb": kp["tb"], "sb": kp["sb"],
            "ctu_end": kp["ctu_end"]}
    return {"tiles": r["tiles"], "end_ms": round(r["end"], 3), "passes": r["passes"],
            "share": {k: round(v / max(c["wave"], 1), 3) for k, v in c.items() if k != "wave"},
            "cycles_per_pass": round(c["wave"] / max(r["passes"], 1)), "kind_passes": kp,
            "cycles_per_run": {k: round(c[k] / max(n, 1)) for k, n in runs.items()},
            "lanes_per_pass": round(r["lane_units"] / max(r["passes"], 1), 2),
            **({"sb_phase_cycles_per_run": {k: round(v / max(kp["sb"], 1)) for k, v in r["sb_phases"].items()}}
               if "sb_phases" in r else {})}


if __name__ == "__main__":
    main()
