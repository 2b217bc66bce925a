# r05: k_intra waves per picture and the luma / chroma split at 128 images with the final code
set -o pipefail
mkdir -p gpurun_out/r05
AB_STEPS=10 timeout -k 10 1000 bash tools/ab.sh -r 2 cur iw4:HEIFGPU_INTRA_WAVES=4 iw8:HEIFGPU_INTRA_WAVES=8 \
    iw16:HEIFGPU_INTRA_WAVES=16 sp0:HEIFGPU_INTRA_SPLIT=0 sp1:HEIFGPU_INTRA_SPLIT=1 > gpurun_out/r05/ab_b128_iwaves.txt 2>&1
