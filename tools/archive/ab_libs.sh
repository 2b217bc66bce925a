#!/bin/bash
# Same-box A/B of in-tree library builds: tools/ab_libs.sh old new old new ...
# ("new" = heif_amd/libheifgpu.so, X = heif_amd/libheifgpu_X.so); bench value,
# stage ms in the pipeline and alone.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out"
i=0
for v in "$@"; do
    i=$((i+1))
    lib=$R/heif_amd/libheifgpu_$v.so; [ "$v" = new ] && lib=$R/heif_amd/libheifgpu.so
    HEIFGPU_LIBRARY=$lib timeout -k 10 300 python3 "$R/bench.py" --steps ${AB_STEPS:-10} --warmup 2 \
        --verify 1 --no-cpu-baseline --no-e2e ${AB_ARGS:-} > "$R/gpurun_out/ab_${i}_$v.log" 2>&1 || { echo "$v FAILED"; tail -3 "$R/gpurun_out/ab_${i}_$v.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], 'pipe', d['stage_ms_per_step'], 'alone', d.get('stage_ms_alone'))" "$R/gpurun_out/ab_${i}_$v.log" "$v"
done
