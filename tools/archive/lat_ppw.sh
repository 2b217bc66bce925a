#!/bin/bash
# Small-batch (config 3) latency: bench.py at each batch size, with the
# adaptive pictures per parse wave (default) and forced values.
# usage: tools/lat_ppw.sh "1 8 32" "0 4"     (0 = adaptive default)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/lat
for b in ${1:-1 8}; do
  for p in ${2:-0 4}; do
    e=""; [ "$p" != 0 ] && e="HEIFGPU_LANES_PPW=$p"
    timeout -k 10 200 env $e python3 bench.py --batch $b --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --verify 1 > gpurun_out/lat/b${b}_p${p}.json 2> gpurun_out/lat/b${b}_p${p}.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['latency_ms_one_step'], d['stage_ms_alone'], d['verified_images'])" gpurun_out/lat/b${b}_p${p}.json
  done
done
