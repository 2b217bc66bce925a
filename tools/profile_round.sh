#!/bin/bash
# Round profile on the GPU box: kernel-trace stats of the default bench run,
# then separate FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md §HBM:
# never combined with tracing; one TCC counter group per pass).
# usage: [BENCH_ARGS="--workload config5 --batch 1"] tools/profile_round.sh <tag>
#        (writes gpurun_out/prof_<tag>/; BENCH_ARGS go to every bench.py run)
set -euo pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
    python3 "$R/bench.py" ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- \
    python3 "$R/bench.py" ${BENCH_ARGS:-} --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --verify 0 > "$OUT/fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- \
    python3 "$R/bench.py" ${BENCH_ARGS:-} --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --verify 0 > "$OUT/write.log" 2>&1
echo "profile $TAG done"
