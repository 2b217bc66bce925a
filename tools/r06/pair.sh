# r06: which waves share a SIMD (per-wave records, counter build), and the heavy-with-light slot order
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
P=heif_amd/libheifgpu_prof.so
HEIFGPU_LIBRARY=$P timeout -k 10 200 python -u tools/wave_times.py 128 gpurun_out/r06/wave_b128_base2.json > gpurun_out/r06/wave_base2.log 2>&1 && tail -1 gpurun_out/r06/wave_base2.log &&
HEIFGPU_LANES_PAIR=1 HEIFGPU_LIBRARY=$P timeout -k 10 200 python -u tools/wave_times.py 128 gpurun_out/r06/wave_b128_pair.json > gpurun_out/r06/wave_pair.log 2>&1 && tail -1 gpurun_out/r06/wave_pair.log &&
timeout -k 10 900 bash tools/ab.sh -r 2 base pair:HEIFGPU_LANES_PAIR=1 &&
AB_ARGS="--workload config4u" timeout -k 10 600 bash tools/ab.sh u_base u_pair:HEIFGPU_LANES_PAIR=1
