#!/bin/bash
# GPU tests, then the parse-mode matrix (tools/lat_modes.sh)
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
tools/lat_modes.sh "${1:-1 8 128}" "${2:-solo lanes}" 10
