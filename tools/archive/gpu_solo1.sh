#!/bin/bash
# GPU tests, then the parse-mode matrix (tools/lat_modes.sh)
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
[ -n "$1" ] && tools/lat_modes.sh "$1" "${2:-solo lanes}" 10; exit 0
