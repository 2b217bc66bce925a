#!/bin/bash
# r03 (session 2): GPU parity tests, then the round profile (kernel-trace stats
# + FETCH/WRITE passes of the default bench) under tag $1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
tools/profile_round.sh ${1:-r03c} || exit 1
python3 -c "import json,sys; d=json.load(open('gpurun_out/prof_${1:-r03c}/bench.json')); print(d['value'], d['ms_per_step'], d.get('stage_ms_per_step'), d.get('verified_images'))"
