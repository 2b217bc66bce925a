#!/bin/bash
# GPU parity tests, same-box single-image latency A/B of the given library variants, spread-parse phase profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--batch 1" tools/ab_libs.sh "$@" || exit 1
HEIFGPU_LIBRARY=heif_amd/libheifgpu_profsb.so timeout -k 10 120 python3 tools/parse_prof.py 1 gpurun_out/profsb_spread_b1.json spread || exit 1
