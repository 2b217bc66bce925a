"""Copies a tools/profile_round.sh run into profiles/<tag>/ and derives the
per-launch HBM traffic of every kernel (MI355X_MICROARCH.md §HBM: FETCH_SIZE
and WRITE_SIZE are KiB; FETCH_SIZE is doubled for gfx950's half-count of
streamed reads — an upper-bound correction for k_parse's byte-wide loads,
whose width the guide leaves uncalibrated).  Writes profiles/pmc_traffic.json,
which bench.py reads for roofline.traffic.

usage: python tools/summarize_profile.py <tag> [round]
  (profiles/<round>/ receives the files; a config-5 run's are suffixed _config5)
"""
import collections
import csv
import json
import pathlib
import shutil
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]


def per_launch(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    src = ROOT / "gpurun_out" / f"prof_{tag}"
    dst = ROOT / "profiles" / (sys.argv[2] if len(sys.argv) > 2 else tag)
    dst.mkdir(parents=True, exist_ok=True)
    bench = json.loads((src / "bench.json").read_text().strip().splitlines()[-1])
    sfx = "_config5" if bench["config"]["workload"].startswith("config5") else ""
    shutil.copy(src / "kt" / "kt_kernel_stats.csv", dst / f"kernel_stats{sfx}.csv")
    (dst / f"bench{sfx}.json").write_text(json.dumps(bench, indent=2) + "\n")
    fetch = per_launch(src / "fetch" / "fetch_counter_collection.csv", "FETCH_SIZE")
    write = per_launch(src / "write" / "write_counter_collection.csv", "WRITE_SIZE")
    stats = {r["Name"]: float(r["AverageNs"]) for r in csv.DictReader(open(src / "kt" / "kt_kernel_stats.csv"))}
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith(("hg::", "void hg::")):
            continue
        f, w = fetch.get(k, 0.0) * 1024, write.get(k, 0.0) * 1024
        hbm = 2 * f + w
        ns = stats.get(k)
        kernels[k] = {"fetch_bytes_raw": f, "write_bytes": w, "hbm_bytes_corrected": hbm, "avg_ns": ns,
                      "hbm_gbs": hbm / ns if ns else None}
    parse = next(v for k, v in kernels.items() if "k_parse" in k)
    out = {
        "tag": tag,
        "batch": bench["config"]["images_per_gpu"],
        "parse_mode": bench["roofline"].get("parse_geometry", {}).get("mode", "lanes"),
        "k_parse_hbm_bytes_per_launch": round(parse["hbm_bytes_corrected"]),
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of "
                  "`bench.py --steps 1 --warmup 1`; bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per launch",
        "kernels": kernels,
    }
    (dst / f"pmc_traffic{sfx}.json").write_text(json.dumps(out, indent=2) + "\n")
    print(json.dumps(out, indent=2))


if __name__ == "__main__":
    main()
