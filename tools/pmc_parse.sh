#!/bin/bash
# SQ counters of the parse kernel (one rocprofv3 --pmc pass per counter set,
# each within the 8-SQ-counter limit), reduced to per-launch and per-bin
# figures in gpurun_out/pmc_parse_<mode><sfx>/parse_counters_<mode><sfx>.json
# (bench.py reads profiles/<round>/ copies of them).
# usage: [PARSE=lanes|solo|spread] [WORKLOAD=config4|config5] [PMC_BATCH=n] tools/pmc_parse.sh [library-suffix]
#        (on the GPU box, repo root)
V=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
LIB=$R/heif_amd/libheifgpu${V:+_$V}.so
BATCH=${PMC_BATCH:-128}
MODE=${PARSE:-lanes}
WL=${WORKLOAD:-config4}
SFX=$([ "$WL" = config5 ] && echo _config5)
OUT=$R/gpurun_out/pmc_parse_${MODE}${SFX}${V:+_$V}
cd /tmp && export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH" \
           "SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA" \
           "SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_IFETCH"; do
    i=$((i + 1))
    HEIFGPU_LIBRARY=$LIB timeout -s KILL 300 rocprofv3 --pmc $set -d "$OUT/set$i" -o p --output-format csv -- \
        python3 "$R/bench.py" --batch "$BATCH" --parse "$MODE" --workload "$WL" --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --verify 0 > "$OUT/set$i.log" 2>&1 || { [ $i -eq 3 ] || exit 1; }
done
python3 - "$OUT" "$BATCH" "$MODE" "$WL" "$SFX" "$R" <<'PY'
import csv, collections, glob, json, sys
out, batch, mode, wl, sfx, root = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5], sys.argv[6]
sys.path.insert(0, root)
acc = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in glob.glob(out + "/set*/**/p_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_parse" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
per_launch = {k: v / len(disp[k]) for k, v in sorted(acc.items())}
if wl == "config5":  # bins of one config-5 image (every image permutes the same 135 tiles): the oracle's count
    from heif_amd import synth_encoder as S
    from oracle import oracle
    p5 = S.CONFIG5["params"]
    pool = [S.picture(p5, 5000 + k) for k in range(135)]
    img = S.grid_heic(S.CONFIG5["out_w"], S.CONFIG5["out_h"], p5, pictures=pool)
    bpi = sum(c["bins"] for c in oracle.decode_heic(img, with_checks=True).checks)
else:
    bpi = 15358022  # bins per halfmoonbay image (oracle count)
bins = batch * bpi
res = {
    "kernel": "k_parse_" + mode,
    "parse_mode": mode,
    "workload": wl,
    "batch_images": batch,
    "bins_per_image": bpi,
    "bins_per_launch": bins,
    "per_launch": {k: round(v) for k, v in per_launch.items()},
    "per_bin": {k: round(v / bins, 4) for k, v in per_launch.items()},
    "note": "SQ_*_CYCLES / WAIT / ACTIVE count quad-cycles (MI355X_MICROARCH.md); one pass per counter set",
}
w = per_launch.get("SQ_WAVES")
if w:
    res["per_wave"] = {k: round(v / w, 1) for k, v in per_launch.items()}
json.dump(res, open(out + f"/parse_counters_{mode}{sfx}.json", "w"), indent=1)
print(json.dumps(res["per_bin"]))
PY
