# r05: SLP vectorizer cost threshold per TU (s1 parse -3, s2 parse -10, s4 parse +3, s3 intra -3)
# against the current build: 128 images, one image
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 2 cur s1:${V}_s1.so s2:${V}_s2.so s3:${V}_s3.so s4:${V}_s4.so \
    > gpurun_out/r05/ab_b128_slp.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 400 bash tools/ab.sh -r 1 cur s1:${V}_s1.so s2:${V}_s2.so s4:${V}_s4.so \
    > gpurun_out/r05/ab_b1_slp.txt 2>&1
