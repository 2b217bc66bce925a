#!/bin/bash
# engine change check: parity subset, then b1 (solo, spread; product and nouni) and b128 lanes
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "halfmoonbay or bench_shard or synthetic_bit_exact" > gpurun_out/gpu_tests_eng.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_eng.log
[ $rc -eq 0 ] || exit $rc
tools/gpu_spread.sh || exit 1
tools/lat_modes.sh "128" "lanes" 10
