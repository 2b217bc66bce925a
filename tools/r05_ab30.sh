# r05: fewer k_transform waves beside the parse, by a VGPR floor (xa 96: one wave in the 160
# VGPRs the two parse waves leave per SIMD; xb 128) against the current build, 128 images
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 2 cur xa:${V}_xa.so xb:${V}_xb.so > gpurun_out/r05/ab_b128_xfloor.txt 2>&1
