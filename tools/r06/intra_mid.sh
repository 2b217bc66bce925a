# r06: GPU suite on the k_intra window refactor, its A/B at 128 images, and
# the mid-size batches (spread with / without the scalar state hint, lanes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r06/gpu_tests_intra.log 2>&1 &&
tail -1 gpurun_out/r06/gpu_tests_intra.log &&
timeout -k 10 600 bash tools/ab.sh -r 2 base:HEIFGPU_LIBRARY=heif_amd/libheifgpu_base.so intra_frame &&
AB_ARGS="--batch 16 --parse spread" timeout -k 10 300 bash tools/ab.sh sp16 sp16_nouni:HEIFGPU_LIBRARY=heif_amd/libheifgpu_nouni.so &&
AB_ARGS="--batch 32 --parse spread" timeout -k 10 300 bash tools/ab.sh sp32 sp32_nouni:HEIFGPU_LIBRARY=heif_amd/libheifgpu_nouni.so &&
AB_ARGS="--batch 16 --parse lanes" timeout -k 10 300 bash tools/ab.sh la16 &&
AB_ARGS="--batch 32 --parse lanes" timeout -k 10 300 bash tools/ab.sh la32
