#!/bin/bash
# Single-image solo-parse A/B over library variants: tools/ab_solo.sh v1 v2 ...  ("base" = product)
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out/ab_solo
for v in "$@"; do
  lib=heif_amd/libheifgpu.so; [ "$v" != base ] && lib=heif_amd/libheifgpu_$v.so
  HEIFGPU_LIBRARY=$lib timeout -k 10 120 python3 bench.py --batch ${AB_BATCH:-1} --parse ${AB_PARSE:-solo} --steps 10 --warmup 2 \
      --no-cpu-baseline --no-e2e --verify 1 > gpurun_out/ab_solo/$v.json 2> gpurun_out/ab_solo/$v.err || { echo "$v FAILED"; tail -3 gpurun_out/ab_solo/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], 'parse', d['stage_ms_alone']['parse'], 'lat', d['latency_ms_one_step'])" gpurun_out/ab_solo/$v.json $v
done
