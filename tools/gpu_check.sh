#!/bin/bash
# GPU parity tests, then a short bench (the iteration loop of a round).
# usage: tools/gpu_check.sh [bench args...]   (on the GPU box, from the repo root)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
cat gpurun_out/bench.json
exit $rc
