#!/bin/bash
# A/B the in-tree library variants heif_amd/libheifgpu_<V>.so on the bench.
# usage: tools/ab_bench.sh A B C ...   (prints value and stage ms per variant)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for v in "$@"; do
    lib=$R/heif_amd/libheifgpu_$v.so; [ "$v" = base ] && lib=$R/heif_amd/libheifgpu.so
    HEIFGPU_LIBRARY=$lib timeout -k 10 300 python3 "$R/bench.py" --steps ${AB_STEPS:-3} --warmup 1 \
        --verify 1 --no-cpu-baseline ${AB_ARGS:-} > "$R/gpurun_out/ab_$v.log" 2>&1 || { echo "$v FAILED"; tail -3 "$R/gpurun_out/ab_$v.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['stage_ms_per_step'])" "$R/gpurun_out/ab_$v.log" "$v"
done
