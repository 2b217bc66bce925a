# r05: GPU suite on the rebuilt library (parse iterative-ilp, intra iterative-minreg), then
# o2 (parse TU at -O2), xf1 (transform max-ilp), lf1 (loop filter max-ilp) against it
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05/gpu_tests.log 2>&1 &&
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 2 cur o2:${V}_o2.so xf1:${V}_xf1.so lf1:${V}_lf1.so \
    > gpurun_out/r05/ab_b128_o2.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 400 bash tools/ab.sh -r 1 cur o2:${V}_o2.so \
    > gpurun_out/r05/ab_b1_o2.txt 2>&1
