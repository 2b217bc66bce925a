# r05: DC sums by ds_swizzle (dc), k_rbsp at the parse's issue priority (rp), one k_intra wave
# per picture (iw1): GPU suite on rp, then A/B at 128 images against sao5 and one image
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
HEIFGPU_LIBRARY=heif_amd/libheifgpu_rp.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests_rp.log 2>&1 &&
AB_STEPS=10 timeout -k 10 800 bash tools/ab.sh -r 2 sao5:${V}_sao5.so dc:${V}_dc.so rp:${V}_rp.so \
    iw1:${V}_rp.so,HEIFGPU_INTRA_WAVES=1 > gpurun_out/r05/ab_b128_rp.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 300 bash tools/ab.sh -r 2 sao5:${V}_sao5.so rp:${V}_rp.so \
    > gpurun_out/r05/ab_b1_rp.txt 2>&1
