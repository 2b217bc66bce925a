#!/bin/bash
# Parse-mode latency / throughput matrix: bench.py per (batch, mode).
# usage: tools/lat_modes.sh "1 8 128" "solo lanes" [steps]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/modes
for b in ${1:-1 128}; do
  for m in ${2:-solo lanes}; do
    timeout -k 10 240 python3 bench.py --batch $b --parse $m --steps ${3:-10} --warmup 2 --no-cpu-baseline --no-e2e --verify 1 \
        > gpurun_out/modes/${TAG}b${b}_${m}.json 2> gpurun_out/modes/${TAG}b${b}_${m}.err || { tail -5 gpurun_out/modes/${TAG}b${b}_${m}.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], 'lat', d['latency_ms_one_step'], 'alone', d['stage_ms_alone'], 'pipe', d['stage_ms_per_step'], d['verified_images'])" gpurun_out/modes/${TAG}b${b}_${m}.json
  done
done
