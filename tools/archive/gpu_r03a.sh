#!/bin/bash
# r03 solo-mode bring-up: GPU tests (the cross-process IPC test on its own),
# then the parse-mode matrix for the product library and the variant without
# the scalar-state hint.
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread --deselect tests/test_gpu_ipc.py::test_ipc_tile_split_gather > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
tools/lat_modes.sh "1 128" "solo lanes" 10 || exit 1
TAG=nouni_ HEIFGPU_LIBRARY=heif_amd/libheifgpu_nouni.so tools/lat_modes.sh "1 128" "solo" 10 || exit 1
timeout -k 10 150 python -u -m pytest tests/test_gpu_ipc.py -x -s -q --timeout 120 --timeout-method thread > gpurun_out/gpu_ipc.log 2>&1; rc=$?
tail -15 gpurun_out/gpu_ipc.log
exit $rc
