# r05: k_intra's reference filter with selects (flt): GPU suite on flt, A/B at 128 images
# against the current build, then the current build's per-kernel instruction mix
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
HEIFGPU_LIBRARY=heif_amd/libheifgpu_flt.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests_flt.log 2>&1 &&
AB_STEPS=10 timeout -k 10 600 bash tools/ab.sh -r 2 cur flt:${V}_flt.so > gpurun_out/r05/ab_b128_flt.txt 2>&1 &&
timeout -k 10 700 bash tools/pmc_kernels.sh r05b > gpurun_out/r05/pmc_kernels_b.txt 2>&1
