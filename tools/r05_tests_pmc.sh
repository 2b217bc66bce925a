# r05: GPU suite on the current build, then the per-kernel SQ instruction mix of one bench step
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05/gpu_tests.log 2>&1 &&
timeout -k 10 700 bash tools/pmc_kernels.sh r05 > gpurun_out/r05/pmc_kernels.txt 2>&1
