#!/bin/bash
# Round-3 closing evidence: GPU parity suite, then the profile set of tools/gpu_profile_r03.sh.
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
tools/gpu_profile_r03.sh
echo "latency $(date +%T)"
TAG=f_ tools/lat_modes.sh "1 4" "spread" 10
