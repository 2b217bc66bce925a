"""Per-queue kernel timeline of a `rocprofv3 --kernel-trace` run of bench.py:
the steady-state decodes (parse launches 7..11 of the run), each kernel's
start / end relative to the first parse, and the gap on the parse queue
between one parse's end and the next one's start (what k_parse waits for).

usage: python tools/timeline.py gpurun_out/prof_r04/kt/kt_kernel_trace.csv [first_parse] [n]
"""
import csv
import sys

KINDS = ["k_parse", "k_transform", "k_intra_fused", "k_intra_stream", "k_intra", "k_sao", "k_deblock", "k_rbsp",
         "k_status_fold", "k_loopfilter", "fillBuffer", "copyBuffer"]


def kind(name):
    for k in KINDS:
        if k in name:
            return k
    return name[:24]


def main():
    path = sys.argv[1]
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    parses = [r for r in rows if "k_parse" in r["Kernel_Name"]]
    if len(parses) < first + n + 1:
        raise SystemExit(f"only {len(parses)} parse launches in the trace")
    t0 = int(parses[first]["Start_Timestamp"])
    lo, hi = t0, int(parses[first + n]["End_Timestamp"])
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e < lo or s > hi or kind(r["Kernel_Name"]) == "copyBuffer":
            continue
        print(f"q{r['Queue_Id']:>2} {kind(r['Kernel_Name']):16s} {(s - t0) / 1e6:9.2f} {(e - t0) / 1e6:9.2f} "
              f"{(e - s) / 1e6:8.2f} ms")
    gaps = [(int(parses[i + 1]["Start_Timestamp"]) - int(parses[i]["End_Timestamp"])) / 1e6
            for i in range(first, first + n)]
    period = (int(parses[first + n]["Start_Timestamp"]) - t0) / 1e6 / n
    dur = sum((int(p["End_Timestamp"]) - int(p["Start_Timestamp"])) / 1e6 for p in parses[first:first + n]) / n
    print(f"parse period {period:.2f} ms = parse {dur:.2f} ms + gap {sum(gaps) / n:.2f} ms "
          f"(gaps {', '.join(f'{g:.2f}' for g in gaps)})")


if __name__ == "__main__":
    main()
