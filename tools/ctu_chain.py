"""WPP critical path of the solo / spread parse (tuning only).

usage: HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so python tools/ctu_chain.py [spread|solo] [out.json]

Decodes one halfmoonbay image (48 tile pictures of 16 x 16 CTBs) with the
counter-instrumented library (`make -C heif_amd/csrc prof`), which records
per CTU the s_memrealtime (100 MHz, chip-wide) of the first time its wave wanted to start it, the
start of its U_CTU unit (the WPP wait over) and the end of its U_CTU_END
unit.  From the per-CTU work (end - start) it replays the WPP schedule with
zero hand-off latency (row r CTU c after row r CTU c - 1 and row r - 1 CTU
min(c + 1, last)) and compares that critical path with the measured span of
each picture: the difference is what the progress hand-off costs.
"""
import ctypes
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import heif_amd as H  # noqa: E402
from heif_amd import _lib  # noqa: E402

CAP = 1 << 17
ROWS, COLS = 16, 16  # CTB rows / columns of a halfmoonbay tile (512 x 512, CTB 32)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "spread"
    src = (ROOT / "tests/golden/halfmoonbay.heic").read_bytes()
    img = H.HeifImage.parse(src)
    ctx = H.DecodeContext(0)
    outs = ctx.alloc_outputs([img])
    b = ctx.prepare([img], parse=mode)
    lib = _lib.lib
    n = 8 + 3 * CAP
    buf = (ctypes.c_uint64 * n)()
    for rep in range(3):  # warm, then the measured decode
        b.decode_async(outs)
        torch.cuda.synchronize()
        k = lib.heifgpu_debug_counters(buf, n)
        if k <= 8:
            raise SystemExit("library has no CTU times: build with `make -C heif_amd/csrc prof`")
    assert b.status() == [0]
    t = np.frombuffer(bytes(buf), np.uint64)[8:].reshape(CAP, 3).astype(np.int64)
    spans, crits, works, waits, t0s, t1s, raw = [], [], [], [], [], [], []
    for p in range(48):
        rows = [t[(p * ROWS + r) * 128:(p * ROWS + r) * 128 + COLS] for r in range(ROWS)]
        want = np.array([r[:, 0] for r in rows])
        start = np.array([r[:, 1] for r in rows])
        end = np.array([r[:, 2] for r in rows])
        if (end == 0).any():
            raise SystemExit(f"picture {p}: missing CTU times")
        work = end - start
        sim = np.zeros((ROWS, COLS))
        for r in range(ROWS):
            for c in range(COLS):
                dep = 0.0
                if c > 0:
                    dep = sim[r, c - 1]
                if r > 0:
                    dep = max(dep, sim[r - 1, min(c + 1, COLS - 1)])
                sim[r, c] = dep + work[r, c]
        t0 = start[0, 0]
        raw.append((want, start, end))
        t0s.append(int(want.min()))
        t1s.append(int(end.max()))
        spans.append(int(end.max() - t0))
        crits.append(float(sim.max()))
        works.append(int(work.sum()))
        waits.append(int((start - want).sum()))
    spans, crits = np.array(spans), np.array(crits)
    h = int(np.argmax(spans))
    res = {
        "mode": mode,
        "pictures": 48,
        "heaviest": h,
        "heaviest_span_ticks": int(spans[h]),
        "heaviest_zero_latency_critical_path_ticks": int(crits[h]),
        "heaviest_handoff_overhead": round(1 - crits[h] / spans[h], 3),
        "max_critical_path_ticks": int(crits.max()),
        "mean_span_over_critical_path": round(float((spans / crits).mean()), 3),
        "global_span_ticks": int(max(t1s) - min(t0s)),
        "picture_first_want_offsets_ticks": sorted(int(v - min(t0s)) for v in t0s),
        "last_picture": int(np.argmax(t1s)),
        "last_picture_start_offset_ticks": int(t0s[int(np.argmax(t1s))] - min(t0s)),
        "heaviest_work_ticks_sum": works[h],
        "heaviest_wait_ticks_sum": waits[h],
        "note": "s_memrealtime ticks (10 ns) of the instrumented build",
    }
    g0 = min(t0s)
    for name, q in (("last", int(np.argmax(t1s))), ("heaviest", h)):
        w_, s_, e_ = raw[q]
        res[f"{name}_picture_rows"] = {"want": (w_ - g0).tolist(), "start": (s_ - g0).tolist(), "end": (e_ - g0).tolist()}
    print(json.dumps(res))
    if len(sys.argv) > 2:
        pathlib.Path(sys.argv[2]).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
