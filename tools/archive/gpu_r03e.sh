#!/bin/bash
# GPU parity tests, single-image latency with k_intra spread vs workgroup mode,
# then the round profile under tag $1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  for b in 1 4; do
    HEIFGPU_INTRA_SPREAD=$v timeout -k 10 120 python3 bench.py --batch $b --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/lat_s${v}_b$b.json 2> gpurun_out/lat_s${v}_b$b.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/lat_s${v}_b$b.json')); print('intra_spread=$v batch=$b', d['value'], d.get('latency_ms_one_step'), d.get('stage_ms_alone'))"
  done
done
[ -n "$1" ] || exit 0
tools/profile_round.sh $1 || exit 1
python3 -c "import json,sys; d=json.load(open('gpurun_out/prof_$1/bench.json')); print(d['value'], d['ms_per_step'], d.get('stage_ms_per_step'), d.get('verified_images'))"
