# r05: transform stages as packed int16 dot products (libheifgpu_dot4.so): GPU suite on that
# build, then A/B at 128 images and one image against the current build
# (and k_intra at 5 / 4 waves per SIMD: HG_INTRA_WPE)
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
HEIFGPU_LIBRARY=heif_amd/libheifgpu_dot4.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests_dot4.log 2>&1 &&
AB_STEPS=10 timeout -k 10 600 bash tools/ab.sh -r 2 cur dot4:${V}_dot4.so wpe5:${V}_wpe5.so wpe4:${V}_wpe4.so > gpurun_out/r05/ab_b128_dot4.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 300 bash tools/ab.sh -r 2 cur dot4:${V}_dot4.so \
    > gpurun_out/r05/ab_b1_dot4.txt 2>&1
