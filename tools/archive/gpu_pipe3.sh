#!/bin/bash
# Three parse-output sets by default: GPU parity suite, then same-box A/B
# against two sets and with the reconstruction streams at high priority.
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS=20 tools/ab_env.sh two:HEIFGPU_PIPELINE=2 three three_rprio:HEIFGPU_RECON_PRIORITY=1 two:HEIFGPU_PIPELINE=2 three three_rprio:HEIFGPU_RECON_PRIORITY=1
