# r05: the lanes parse's bit window topped up once per pass (topup) against the same build
# without it (notu): GPU suite on topup, A/B at 128 images and one image
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
HEIFGPU_LIBRARY=heif_amd/libheifgpu_topup.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests_topup.log 2>&1 &&
AB_STEPS=10 timeout -k 10 700 bash tools/ab.sh -r 2 notu:${V}_notu.so topup:${V}_topup.so > gpurun_out/r05/ab_b128_topup.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 300 bash tools/ab.sh -r 1 notu:${V}_notu.so topup:${V}_topup.so > gpurun_out/r05/ab_b1_topup.txt 2>&1
