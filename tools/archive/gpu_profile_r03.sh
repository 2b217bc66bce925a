#!/bin/bash
# r03 evidence run: kernel-trace stats + FETCH/WRITE passes of the default bench
# (tools/profile_round.sh), SQ counters of the lanes parse at the bench batch and of
# the spread parse of one image, and the s_memtime unit breakdowns (prof library).
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
R=$(pwd)
mkdir -p gpurun_out
echo "profile_round $(date +%T)"
tools/profile_round.sh r03 || exit 1
echo "pmc lanes $(date +%T)"
PARSE=lanes PMC_BATCH=128 tools/pmc_parse.sh > gpurun_out/pmc_lanes.log 2>&1 || { tail -5 gpurun_out/pmc_lanes.log; exit 1; }
echo "pmc spread $(date +%T)"
mv gpurun_out/pmc_parse gpurun_out/pmc_parse_lanes
PARSE=spread PMC_BATCH=1 tools/pmc_parse.sh > gpurun_out/pmc_spread.log 2>&1 || { tail -5 gpurun_out/pmc_spread.log; exit 1; }
mv gpurun_out/pmc_parse gpurun_out/pmc_parse_spread
echo "unit breakdowns $(date +%T)"
HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so timeout -k 10 120 python3 tools/parse_prof.py 128 gpurun_out/prof_lanes_b128.json lanes || exit 1
HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so timeout -k 10 120 python3 tools/parse_prof.py 1 gpurun_out/prof_spread_b1.json spread || exit 1
echo "done $(date +%T)"
