# r05: MFMA transform with B operands packed from the int16 table (no extra LDS): GPU suite on
# mfd (every 16x16 / 32x32 TB, 6 waves per SIMD), A/B at 128 images of mfd, mfe (32x32 with >= 8
# columns, 16x16 >= 12), mff (as mfd at 7 waves per SIMD, one spilled VGPR) against the current build
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
HEIFGPU_LIBRARY=heif_amd/libheifgpu_mfd.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests_mfd.log 2>&1 &&
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 2 cur mfd:${V}_mfd.so mfe:${V}_mfe.so mff:${V}_mff.so \
    > gpurun_out/r05/ab_b128_mfd.txt 2>&1
