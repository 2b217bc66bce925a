# r05: GPU suite on the rebuilt library (lanes and solo parse as separate translation units;
# lanes: VGPR floor 176, 256-VGPR budget, SLP threshold -3), A/B against the previous
# configuration (prev) at 128 images and one image
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05/gpu_tests.log 2>&1 &&
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 3 cur prev:${V}_prev.so > gpurun_out/r05/ab_b128_tu.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 400 bash tools/ab.sh -r 2 cur prev:${V}_prev.so \
    > gpurun_out/r05/ab_b1_tu.txt 2>&1
