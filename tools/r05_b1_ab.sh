# r05: GPU tests of the current tree, then one-image latency A/B (same box):
# current (agent release/acquire hand-offs), r04 relaxed hand-offs, no scalar state hint
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05/gpu_tests.log 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 900 bash tools/ab.sh -r 3 cur relaxed:HEIFGPU_LIBRARY=heif_amd/libheifgpu_relaxed.so \
    nouni:HEIFGPU_LIBRARY=heif_amd/libheifgpu_nouni.so > gpurun_out/r05/ab_b1.txt 2>&1
