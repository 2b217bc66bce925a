#!/bin/bash
# Kernel timeline of a short pipelined bench run (rocprofv3 kernel trace):
# prints each dispatch's start / end relative to the first, in ms.
# usage: tools/trace_timeline.sh [bench args]   -> gpurun_out/timeline/
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/timeline" -o tl --output-format csv -- \
    python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --verify 0 "$@" > "$R/gpurun_out/timeline.log" 2>&1 || exit 1
python3 - "$R/gpurun_out/timeline/tl_kernel_trace.csv" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "hg::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hg::", "")
    print(f"{name:28s} {s:9.2f} {e:9.2f} {e - s:8.2f}")
PY
