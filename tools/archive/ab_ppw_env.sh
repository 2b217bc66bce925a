#!/bin/bash
# like ab_ppw.sh with an environment per run: tools/ab_ppw_env.sh variant:ppw:VAR=v,VAR2=w ...
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out/ab_ppw
for spec in "$@"; do
  v=${spec%%:*}; rest=${spec#*:}; p=${rest%%:*}; envs=""; [ "$rest" != "$p" ] && envs=${rest#*:}
  lib=heif_amd/libheifgpu.so; [ "$v" != base ] && lib=heif_amd/libheifgpu_$v.so
  tag=$(echo "$spec" | tr ':,=' '___')
  env HEIFGPU_LIBRARY=$lib ${envs//,/ } timeout -k 10 200 python3 bench.py --batch 128 --parse lanes --ppw $p --steps ${AB_STEPS:-20} --warmup 2 \
      --no-cpu-baseline --no-e2e --verify 2 > gpurun_out/ab_ppw/$tag.json 2> gpurun_out/ab_ppw/$tag.err || { echo "$spec FAILED"; tail -3 gpurun_out/ab_ppw/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], 'parse pipe', d['stage_ms_per_step']['parse'], 'alone', d['stage_ms_alone']['parse'], 'pipe', d['stage_ms_per_step'])" gpurun_out/ab_ppw/$tag.json $spec
done
