#!/bin/bash
# GPU parity tests, then same-box A/B of library variants at one image (spread parse)
# and at the bench batch (lanes parse): tools/gpu_ab_both.sh head new head new
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
echo "== batch 1"
AB_ARGS="--batch 1" tools/ab_libs.sh "$@" || exit 1
echo "== batch 128"
tools/ab_libs.sh "$@" || exit 1
