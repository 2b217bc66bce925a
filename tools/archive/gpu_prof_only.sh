#!/bin/bash
# Kernel-trace stats + FETCH/WRITE passes of the default bench (tools/profile_round.sh).
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out
tools/profile_round.sh ${1:-r03}
