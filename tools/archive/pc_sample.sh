#!/bin/bash
# PC sampling of the single-image (spread) parse: which instructions the waves
# sit on.  usage: tools/pc_sample.sh [method] [unit] [interval]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pcs
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$OUT/list.txt" 2>&1
grep -i -B2 -A8 "pc_sampl\|PC Sampling" "$OUT/list.txt" | head -60
M=${1:-stochastic}; U=${2:-cycles}; I=${3:-65536}
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit $U \
    --pc-sampling-interval $I -d "$OUT/run" -o pcs --output-format csv -- \
    python3 "$R/bench.py" --batch 1 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --verify 0 > "$OUT/bench.log" 2>&1
rc=$?
echo "rocprofv3 rc=$rc"
tail -5 "$OUT/bench.log"
find "$OUT/run" -type f | head -20
for f in $(find "$OUT/run" -name "*.csv"); do echo "$f $(wc -l < $f)"; head -3 "$f"; done
exit $rc
