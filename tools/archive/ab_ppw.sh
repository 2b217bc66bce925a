#!/bin/bash
# lanes-parse occupancy A/B: (variant, pics per wave) pairs, e.g. tools/ab_ppw.sh base:0 wpe3:2
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out/ab_ppw
for spec in "$@"; do
  v=${spec%%:*}; p=${spec#*:}
  lib=heif_amd/libheifgpu.so; [ "$v" != base ] && lib=heif_amd/libheifgpu_$v.so
  HEIFGPU_LIBRARY=$lib timeout -k 10 200 python3 bench.py --batch 128 --parse lanes --ppw $p --steps ${AB_STEPS:-20} --warmup 2 \
      --no-cpu-baseline --no-e2e --verify 2 > gpurun_out/ab_ppw/${v}_$p.json 2> gpurun_out/ab_ppw/${v}_$p.err || { echo "$spec FAILED"; tail -3 gpurun_out/ab_ppw/${v}_$p.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], 'parse pipe', d['stage_ms_per_step']['parse'], 'alone', d['stage_ms_alone']['parse'], 'pipe', d['stage_ms_per_step'])" gpurun_out/ab_ppw/${v}_$p.json $spec
done
