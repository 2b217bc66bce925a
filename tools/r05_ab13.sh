# r05: k_transform's 4x4 rounds over the coded 4x4 TBs only (pa, on top of tbb): GPU suite on pa,
# A/B at 128 images against tbb and one image against the current build
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
HEIFGPU_LIBRARY=heif_amd/libheifgpu_pa.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests_pa.log 2>&1 &&
AB_STEPS=10 timeout -k 10 700 bash tools/ab.sh -r 2 tbb:${V}_tbb.so pa:${V}_pa.so > gpurun_out/r05/ab_b128_pa.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 300 bash tools/ab.sh -r 2 cur pa:${V}_pa.so > gpurun_out/r05/ab_b1_pa.txt 2>&1
