#!/bin/bash
# SQ instruction-mix / wait counters per kernel of one bench step (tuning).
# usage: tools/pmc_kernels.sh [tag]  -> gpurun_out/pmck_<tag>/ and a per-kernel table
T=${1:-base}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmck_$T
mkdir -p "$O"
i=0
for set in "SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_SMEM SQ_BUSY_CU_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS"; do
    i=$((i + 1))
    timeout -k 10 300 rocprofv3 --pmc $set -d "$O/s$i" -o p --output-format csv -- \
        python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --verify 0 > "$O/s$i.log" 2>&1 || exit 1
done
python3 - "$O" <<'PY'
import csv, collections, glob, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float)); nd = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/s*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hg::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); nd[k].add((f, r["Dispatch_Id"]))
for k, c in acc.items():
    n = max(1, len(nd[k]) // 2)
    print(k, {a: f"{v / n:.3e}" for a, v in sorted(c.items())})
PY
