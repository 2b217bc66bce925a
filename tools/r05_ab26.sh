# r05: the lanes parse held to 2 waves per SIMD (a VGPR floor of 176), alone (f0) and with the
# SLP cost threshold that took its VGPRs below the 3-wave line (f1 -3, f2 -10; f4 / f5 with a
# 256-VGPR budget) against the current build: 128 images, one image
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 2 cur f0:${V}_f0.so f1:${V}_f1.so f2:${V}_f2.so f4:${V}_f4.so f5:${V}_f5.so \
    > gpurun_out/r05/ab_b128_floor.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 400 bash tools/ab.sh -r 1 cur f0:${V}_f0.so f1:${V}_f1.so \
    > gpurun_out/r05/ab_b1_floor.txt 2>&1
