# r06 (session 2) first call: GPU suite, the default bench, one-image latency
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r06/gpu_tests.log 2>&1 &&
tail -2 gpurun_out/r06/gpu_tests.log &&
timeout -k 10 300 python3 bench.py > gpurun_out/r06/bench.json 2> gpurun_out/r06/bench.err &&
tail -c 1500 gpurun_out/r06/bench.json &&
timeout -k 10 200 python3 bench.py --batch 1 --no-cpu-baseline --no-e2e > gpurun_out/r06/bench_b1.json 2> gpurun_out/r06/bench_b1.err &&
tail -c 400 gpurun_out/r06/bench_b1.json &&
HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so timeout -k 10 200 python -u tools/wave_times.py 128 gpurun_out/r06/wave_times_b128.json > gpurun_out/r06/wave_times.log 2>&1 &&
tail -30 gpurun_out/r06/wave_times.log
