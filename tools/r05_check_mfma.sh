# r05: GPU suite and the default bench on the rebuilt library (MFMA transform default)
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05/gpu_tests.log 2>&1 &&
timeout -k 10 400 python3 bench.py > gpurun_out/r05/bench_mfma.json 2> gpurun_out/r05/bench_mfma.err
