#!/bin/bash
# spread-mode bring-up: emulation-verified kernel on the GPU (single image parity via bench verify),
# then single-image A/B of solo / spread for the product library and the nouni variant
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out/ab_solo
for m in spread solo; do
  for v in base nouni; do
    lib=heif_amd/libheifgpu.so; [ "$v" != base ] && lib=heif_amd/libheifgpu_$v.so
    HEIFGPU_LIBRARY=$lib timeout -k 10 120 python3 bench.py --batch ${AB_BATCH:-1} --parse $m --steps 10 --warmup 2 \
        --no-cpu-baseline --no-e2e > gpurun_out/ab_solo/${m}_$v.json 2> gpurun_out/ab_solo/${m}_$v.err || { echo "$m $v FAILED"; tail -3 gpurun_out/ab_solo/${m}_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], 'parse', d['stage_ms_alone']['parse'], 'lat', d['latency_ms_one_step'], 'verified', d['verified_images'])" gpurun_out/ab_solo/${m}_$v.json "$m $v"
  done
done
