# r05: the lanes translation unit under the VGPR floor with other code-generation flags
# (a1 max-ilp scheduler, a3 unroll threshold 1000, a4 SLP threshold -5, a5 SLP -2) against
# the current build at 128 images
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 2 cur a1:${V}_a1.so a3:${V}_a3.so a4:${V}_a4.so a5:${V}_a5.so \
    > gpurun_out/r05/ab_b128_lanesflags.txt 2>&1
