# r05: the transposed transform tables from a compile-time constant table (mtc), and k_transform's
# larger TBs picked from a ballot over 64 coalesced records (tbb, on top of mtc): GPU suite on
# tbb, A/B at 128 images against the current build
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
HEIFGPU_LIBRARY=heif_amd/libheifgpu_tbb.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests_tbb.log 2>&1 &&
AB_STEPS=10 timeout -k 10 700 bash tools/ab.sh -r 2 cur mtc:${V}_mtc.so tbb:${V}_tbb.so > gpurun_out/r05/ab_b128_tbb.txt 2>&1
