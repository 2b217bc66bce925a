# r05: k_intra without scalarized global loads (ig: its uniform loads as vector loads, fewer SGPRs)
# against the current build: 128 images and one image
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 2 cur ig:${V}_ig.so > gpurun_out/r05/ab_b128_ig.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 400 bash tools/ab.sh -r 1 cur ig:${V}_ig.so > gpurun_out/r05/ab_b1_ig.txt 2>&1
