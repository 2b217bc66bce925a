#!/bin/bash
# Same-box A/B of the reconstruction-stream priority and the 3-set pipeline.
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out
AB_STEPS=10 tools/ab_env.sh base rprio:HEIFGPU_RECON_PRIORITY=1 pipe3:HEIFGPU_PIPELINE=3 base rprio:HEIFGPU_RECON_PRIORITY=1 pipe3:HEIFGPU_PIPELINE=3
