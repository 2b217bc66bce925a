#!/bin/bash
# A/B environment settings of the default library on the bench.
# usage: tools/ab_env.sh name:VAR=v,VAR2=w name2:...   ("base" = no extra env)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for spec in "$@"; do
    name=${spec%%:*}; envs=""; [ "$spec" != "$name" ] && envs=${spec#*:}
    timeout -k 10 300 env ${envs//,/ } python3 "$R/bench.py" --steps ${AB_STEPS:-3} --warmup 1 \
        --verify 1 --no-cpu-baseline ${AB_ARGS:-} > "$R/gpurun_out/abe_$name.log" 2>&1 || { echo "$name FAILED"; tail -5 "$R/gpurun_out/abe_$name.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['stage_ms_per_step'])" "$R/gpurun_out/abe_$name.log" "$name"
done
