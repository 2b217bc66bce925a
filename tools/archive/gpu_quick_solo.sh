#!/bin/bash
# solo-parse parity subset, then the single-image A/B over the given variants
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "solo or halfmoonbay or ring or nowpp" > gpurun_out/gpu_tests_solo.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_solo.log
[ $rc -eq 0 ] || exit $rc
tools/ab_solo.sh "$@"
