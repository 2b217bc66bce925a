#!/bin/bash
# solo / spread parse phase breakdown (libheifgpu_profsb.so, libheifgpu_prof.so) for one image
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out
HEIFGPU_LIBRARY=heif_amd/libheifgpu_profsb.so timeout -k 10 120 python3 tools/parse_prof.py 1 gpurun_out/profsb_spread_b1.json spread || exit 1
HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so timeout -k 10 120 python3 tools/parse_prof.py 1 gpurun_out/prof_spread_b1.json spread || exit 1
