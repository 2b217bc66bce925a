#!/bin/bash
# GPU parity tests on the default library, then an A/B of library variants
# (tools/ab_bench.sh) at AB_STEPS steps.  usage: tools/gpu_ab.sh V1 V2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do tools/ab_bench.sh "$@" || exit 1; done
