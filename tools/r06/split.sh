# r06: split dealing (HEIFGPU_LANES_SPLIT=1: heaviest pictures two per wave, the rest four) — correctness
# (every image verified), per-wave times, bench pairs, distinct-tile control
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
HEIFGPU_LANES_SPLIT=1 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/r06/split_verify.json 2>&1 &&
python3 -c "import json; d=json.loads(open('gpurun_out/r06/split_verify.json').read().strip().splitlines()[-1]); print('split verified', d['verified_images'], d['roofline']['parse_geometry'])" &&
HEIFGPU_LANES_SPLIT=1 HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so timeout -k 10 200 python -u tools/wave_times.py 128 gpurun_out/r06/wave_b128_split.json > gpurun_out/r06/wave_split.log 2>&1 && tail -1 gpurun_out/r06/wave_split.log &&
timeout -k 10 900 bash tools/ab.sh -r 2 base split:HEIFGPU_LANES_SPLIT=1 &&
AB_ARGS="--workload config4u" timeout -k 10 600 bash tools/ab.sh u_base u_split:HEIFGPU_LANES_SPLIT=1
