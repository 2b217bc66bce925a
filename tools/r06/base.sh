# r06 first call: GPU suite, the default bench, per-wave parse times (counter build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r06/gpu_tests.log 2>&1 &&
tail -2 gpurun_out/r06/gpu_tests.log &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-e2e > gpurun_out/r06/bench_base.json 2> gpurun_out/r06/bench_base.err &&
tail -c 600 gpurun_out/r06/bench_base.json &&
HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so timeout -k 10 200 python -u tools/wave_times.py 128 gpurun_out/r06/wave_times_b128.json
