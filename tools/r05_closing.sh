# r05 closing check on the final tree: smoke(), the GPU suite, the default bench line
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05/smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05/gpu_tests.log 2>&1 &&
timeout -k 10 400 python3 bench.py > gpurun_out/r05/bench_closing.json 2> gpurun_out/r05/bench_closing.err
