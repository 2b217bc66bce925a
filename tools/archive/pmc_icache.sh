#!/bin/bash
# Instruction-cache / fetch counters of k_parse per library variant (tuning).
# usage: tools/pmc_icache.sh V1 V2 ...   ("base" = libheifgpu.so)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
    lib=$R/heif_amd/libheifgpu_$v.so; [ "$v" = base ] && lib=$R/heif_amd/libheifgpu.so
    out=$R/gpurun_out/icache_$v
    HEIFGPU_LIBRARY=$lib timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQC_TC_INST_REQ SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU \
        -d "$out" -o p --output-format csv -- python3 "$R/bench.py" --batch 64 --steps 1 --warmup 1 --no-cpu-baseline --verify 0 > "$out.log" 2>&1 || exit 1
    python3 - "$out" "$v" <<'PY'
import csv, collections, glob, sys
acc = collections.defaultdict(float); d = set()
for f in glob.glob(sys.argv[1] + "/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_parse" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); d.add(r["Dispatch_Id"])
bins = 64 * 15358022 * len(d)
print(sys.argv[2], {k: round(v / bins, 3) for k, v in sorted(acc.items())}, "per bin")
PY
done
