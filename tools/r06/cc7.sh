# r06: context states as 7-bit fields of one 64-bit word in the sub-block's sig loop (lanes engine: the
# library; scalar engine's 4x4 loop: libheifgpu_solo7.so), against the HEAD build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
B=HEIFGPU_LIBRARY=heif_amd/libheifgpu_base.so
S=HEIFGPU_LIBRARY=heif_amd/libheifgpu_solo7.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r06/gpu_tests_cc7.log 2>&1 &&
tail -1 gpurun_out/r06/gpu_tests_cc7.log &&
HEIFGPU_LIBRARY=heif_amd/libheifgpu_solo7.so timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_synth.py -m gpu -x -q --timeout 240 --timeout-method thread -k "spread or b1 or stream or one_image or config3" > gpurun_out/r06/gpu_tests_solo7.log 2>&1 &&
tail -1 gpurun_out/r06/gpu_tests_solo7.log &&
timeout -k 10 900 bash tools/ab.sh -r 2 base:$B cc7 &&
AB_ARGS="--batch 1" timeout -k 10 600 bash tools/ab.sh -r 2 b1_base:$B b1_cc7 b1_solo7:$S &&
AB_ARGS="--batch 16" timeout -k 10 600 bash tools/ab.sh b16_base:$B b16_cc7 b16_solo7:$S
