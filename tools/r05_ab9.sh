# r05: k_intra's small-TB neighbour gather with selects and one-pass prediction (ipx), luma
# deblocking by 4-sample words (dbw, on top of ipx): GPU suite on dbw, A/B at 128 images vs rp
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
HEIFGPU_LIBRARY=heif_amd/libheifgpu_dbw.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests_dbw.log 2>&1 &&
AB_STEPS=10 timeout -k 10 800 bash tools/ab.sh -r 2 rp:${V}_rp.so ipx:${V}_ipx.so dbw:${V}_dbw.so \
    > gpurun_out/r05/ab_b128_ipx.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 300 bash tools/ab.sh -r 2 rp:${V}_rp.so dbw:${V}_dbw.so \
    > gpurun_out/r05/ab_b1_ipx.txt 2>&1
