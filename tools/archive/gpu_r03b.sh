#!/bin/bash
# r03: IPC gather test, solo A/B (scalar-state hint vs not), solo counters.
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out
timeout -k 10 150 python -u -m pytest tests/test_gpu_ipc.py -x -s -q --timeout 120 --timeout-method thread > gpurun_out/gpu_ipc.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_ipc.log
[ $rc -eq 0 ] || exit $rc
tools/lat_modes.sh "1" "solo" 10 || exit 1
TAG=nouni_ HEIFGPU_LIBRARY=heif_amd/libheifgpu_nouni.so tools/lat_modes.sh "1" "solo" 10 || exit 1
HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so timeout -k 10 120 python3 tools/parse_prof.py 1 gpurun_out/prof_solo_b1.json solo || exit 1
HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so timeout -k 10 120 python3 tools/parse_prof.py 1 gpurun_out/prof_lanes_b1.json lanes || exit 1
PARSE=solo PMC_BATCH=1 tools/pmc_parse.sh
