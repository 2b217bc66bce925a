# r05: vectorizer / unroller off per TU (v1 parse no SLP, v2 parse no loop unrolling, v3 intra
# no SLP, v4 intra no loop unrolling) against the current build: 128 images, one image
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 2 cur v1:${V}_v1.so v2:${V}_v2.so v3:${V}_v3.so v4:${V}_v4.so \
    > gpurun_out/r05/ab_b128_vu.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 400 bash tools/ab.sh -r 1 cur v1:${V}_v1.so v2:${V}_v2.so v4:${V}_v4.so \
    > gpurun_out/r05/ab_b1_vu.txt 2>&1
