# r05: pictures per lanes wave and the pipeline depth re-checked on the final code, 128 images
set -o pipefail
mkdir -p gpurun_out/r05
AB_STEPS=10 timeout -k 10 1000 bash tools/ab.sh -r 2 cur ppw2:HEIFGPU_LANES_PPW=2 ppw4:HEIFGPU_LANES_PPW=4 \
    pipe2:HEIFGPU_PIPELINE=2 > gpurun_out/r05/ab_b128_ppw.txt 2>&1
