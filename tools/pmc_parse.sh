#!/bin/bash
# SQ instruction-mix counters of k_parse for one library variant (tuning).
# usage: tools/pmc_parse.sh <variant-suffix or ''>  -> gpurun_out/pmc_<v>/
V=$1
# extra environment (e.g. HEIFGPU_PARSE=lanes) is inherited by the profiled process
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
LIB=$R/heif_amd/libheifgpu${V:+_$V}.so
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/pmc_$V"
for set in "SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_SMEM SQ_BUSY_CU_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS"; do
    tag=$(echo $set | cut -c1-12 | tr ' ' '_')
    HEIFGPU_LIBRARY=$LIB timeout -k 10 300 rocprofv3 --pmc $set -d "$R/gpurun_out/pmc_$V/$tag" -o p --output-format csv -- \
        python3 "$R/bench.py" --batch 64 --steps 1 --warmup 1 --no-cpu-baseline --verify 0 > "$R/gpurun_out/pmc_$V/$tag.log" 2>&1 || exit 1
done
python3 - "$R/gpurun_out/pmc_$V" <<'PY'
import csv, collections, glob, sys
acc = collections.defaultdict(float); disp = set()
for f in glob.glob(sys.argv[1] + "/*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_parse" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add((f, r["Dispatch_Id"]))
nd = len(disp) / 2
bins = 64 * 15358022
print({k: round(v / nd / bins, 2) for k, v in sorted(acc.items())}, "per bin")
PY
