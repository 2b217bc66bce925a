# r05: the parse TU alone under a machine scheduler (p3 iterative-ilp, p1 max-ilp, p4
# iterative-maxocc, p5 iterative-minreg; the rest default) against the current build:
# GPU suite on p3, 128 images and one image
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
HEIFGPU_LIBRARY=heif_amd/libheifgpu_p3.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests_p3.log 2>&1 &&
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 2 cur p3:${V}_p3.so p1:${V}_p1.so p4:${V}_p4.so p5:${V}_p5.so \
    > gpurun_out/r05/ab_b128_psched.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 400 bash tools/ab.sh -r 2 cur p3:${V}_p3.so p4:${V}_p4.so p5:${V}_p5.so \
    > gpurun_out/r05/ab_b1_psched.txt 2>&1
