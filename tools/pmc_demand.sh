#!/bin/bash
# Issue / LDS demand per kernel (what a kernel takes from the SIMDs and LDS it
# shares with the other stream's kernel), per library variant (tuning).
# usage: tools/pmc_demand.sh V1 V2 ...   ("base" = libheifgpu.so)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
    lib=$R/heif_amd/libheifgpu_$v.so; [ "$v" = base ] && lib=$R/heif_amd/libheifgpu.so
    out=$R/gpurun_out/dem_$v
    HEIFGPU_LIBRARY=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES \
        -d "$out" -o p --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --verify 0 > "$out.log" 2>&1 || exit 1
    python3 - "$out" "$v" <<'PY'
import csv, collections, glob, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hg::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k, c in acc.items():
    if "k_" in k:
        d = len(n[k])
        print(sys.argv[2], k, {a.replace("SQ_", ""): round(b / d / 1e6, 1) for a, b in sorted(c.items())}, "M/dispatch")
PY
done
