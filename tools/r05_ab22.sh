# r05: machine schedulers for the reconstruction TUs on top of the parse's iterative-ilp
# (i5: intra iterative-minreg, i3: intra iterative-ilp, l1: transform + loop filter max-ilp,
# l5: transform + loop filter iterative-minreg) against the current build: 128 images, one image
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 2 cur i5:${V}_i5.so i3:${V}_i3.so l1:${V}_l1.so l5:${V}_l5.so \
    > gpurun_out/r05/ab_b128_rsched.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 400 bash tools/ab.sh -r 1 cur i5:${V}_i5.so i3:${V}_i3.so \
    > gpurun_out/r05/ab_b1_rsched.txt 2>&1
