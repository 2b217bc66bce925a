#!/bin/bash
# GPU parity tests, then a same-box single-image latency A/B of library builds
# (tools/ab_libs.sh at --batch 1): tools/gpu_lat_ab.sh old new old new
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--batch 1" tools/ab_libs.sh "$@"
