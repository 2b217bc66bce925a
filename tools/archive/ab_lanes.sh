#!/bin/bash
# b128 lanes A/B over library variants: tools/ab_lanes.sh v1 v2 ...  ("base" = product); AB_STEPS, AB_BATCH, AB_PARSE
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out/ab_lanes
for v in "$@"; do
  lib=heif_amd/libheifgpu.so; [ "$v" != base ] && lib=heif_amd/libheifgpu_$v.so
  HEIFGPU_LIBRARY=$lib timeout -k 10 200 python3 bench.py --batch ${AB_BATCH:-128} --parse ${AB_PARSE:-auto} --steps ${AB_STEPS:-10} --warmup 2 \
      --no-cpu-baseline --no-e2e --verify ${AB_VERIFY:-2} > gpurun_out/ab_lanes/$v.json 2> gpurun_out/ab_lanes/$v.err || { echo "$v FAILED"; tail -3 gpurun_out/ab_lanes/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], 'parse pipe', d['stage_ms_per_step']['parse'], 'alone', d['stage_ms_alone']['parse'], 'lat', d['latency_ms_one_step'])" gpurun_out/ab_lanes/$v.json $v
done
