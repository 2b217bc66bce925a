#!/bin/bash
# A/B of environment settings on the bench (same box, variants interleaved).
# usage: tools/ab.sh [-r ROUNDS] name:VAR=v,VAR2=w name2 ...   ("name" alone = no extra env)
# env: AB_STEPS (10), AB_ARGS (extra bench.py arguments)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUNDS=1
if [ "$1" = "-r" ]; then ROUNDS=$2; shift 2; fi
mkdir -p "$R/gpurun_out"
for ((k = 0; k < ROUNDS; ++k)); do
    for spec in "$@"; do
        name=${spec%%:*}; envs=""; [ "$spec" != "$name" ] && envs=${spec#*:}
        log="$R/gpurun_out/ab_${name}_$k.log"
        timeout -k 10 300 env ${envs//,/ } python3 "$R/bench.py" --steps ${AB_STEPS:-10} --warmup 2 \
            --verify 0 --no-cpu-baseline --no-e2e ${AB_ARGS:-} > "$log" 2>&1 || { echo "$name FAILED"; tail -5 "$log"; exit 1; }
        python3 - "$log" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s, a = d["stage_ms_per_step"], d["stage_ms_alone"]
print(f"{sys.argv[2]:>12} {d['value']:9.1f} Mpix/s {d['ms_per_step']:7.2f} ms/step | pipe " +
      " ".join(f"{k[:5]} {v:6.2f}" for k, v in s.items()) + " | alone " + " ".join(f"{v:6.2f}" for v in a.values()) +
      f" | lat {d['latency_ms_one_step']:6.2f} | geom {d['roofline']['parse_geometry']}", flush=True)
PY
    done
done
