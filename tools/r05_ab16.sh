# r05: SAO / deblocking index math by f32-reciprocal division (fd), and k_intra's 4x4 / 8x8
# residual loaded one TB ahead (pf, on top of fd): GPU suite on pf, A/B at 128 images against
# the current build, one image against it
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
HEIFGPU_LIBRARY=heif_amd/libheifgpu_pf.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests_pf.log 2>&1 &&
AB_STEPS=10 timeout -k 10 700 bash tools/ab.sh -r 2 cur fd:${V}_fd.so pf:${V}_pf.so > gpurun_out/r05/ab_b128_pf.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 300 bash tools/ab.sh -r 1 cur pf:${V}_pf.so > gpurun_out/r05/ab_b1_pf.txt 2>&1
