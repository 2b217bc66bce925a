# r05: transform stages as packed int16 dot products (libheifgpu_dot.so): GPU suite on that
# build, then A/B at 128 images and one image against the current build
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
HEIFGPU_LIBRARY=heif_amd/libheifgpu_dot.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests_dot.log 2>&1 &&
AB_STEPS=10 timeout -k 10 600 bash tools/ab.sh -r 2 cur dot:${V}_dot.so > gpurun_out/r05/ab_b128_dot.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 300 bash tools/ab.sh -r 2 cur dot:${V}_dot.so \
    > gpurun_out/r05/ab_b1_dot.txt 2>&1
