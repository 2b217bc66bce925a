#!/bin/bash
# GPU parity tests + a short bench + the k_parse_lanes cycle breakdown (tuning loop).
# usage: tools/gpu_quick.sh   (on the GPU box, from the repo root)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS=3 tools/ab_env.sh base || exit 1
if [ -f heif_amd/libheifgpu_prof.so ]; then
    HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so timeout -k 10 120 python3 tools/parse_prof.py 128
fi
