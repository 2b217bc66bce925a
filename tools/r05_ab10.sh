# r05: k_intra's chroma-pair gather with selects (ipx2) and two-wave k_transform workgroups on
# top of it (xf2): GPU suite on ipx2, A/B at 128 images against the current build
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
HEIFGPU_LIBRARY=heif_amd/libheifgpu_ipx2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests_ipx2.log 2>&1 &&
AB_STEPS=10 timeout -k 10 800 bash tools/ab.sh -r 2 cur ipx2:${V}_ipx2.so xf2:${V}_xf2.so \
    > gpurun_out/r05/ab_b128_ipx2.txt 2>&1
