# r05: SAO four samples per load (sao_quad) on top of the 4x4 dot transforms and k_intra at
# 5 waves per SIMD: GPU suite on that build, then A/B at 128 images against the same build
# without sao_quad (wpe5)
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
HEIFGPU_LIBRARY=heif_amd/libheifgpu_sao5.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests_sao5.log 2>&1 &&
AB_STEPS=10 timeout -k 10 600 bash tools/ab.sh -r 2 wpe5:${V}_wpe5.so sao5:${V}_sao5.so cur \
    > gpurun_out/r05/ab_b128_sao.txt 2>&1
