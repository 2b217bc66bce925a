# r06: GPU suite with row-major spread as the default, then the AUTO geometry at 1..64 images
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r06/gpu_tests_rows.log 2>&1 &&
tail -1 gpurun_out/r06/gpu_tests_rows.log &&
TAG=r06auto_ timeout -k 10 900 bash tools/lat_modes.sh "1 4 8 16 24 32 48 64" "auto" 10 &&
timeout -k 10 700 bash tools/pmc_kernels.sh r06 > gpurun_out/r06/pmc_kernels_b128.txt 2>&1 &&
tail -12 gpurun_out/r06/pmc_kernels_b128.txt
