# r06: coefficient-free TBs and empty sub-blocks inside one unit run: A/B against HEAD, then the per-wave breakdown
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
bash tools/r06/ab_lib.sh loops &&
HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so timeout -k 10 300 python -u tools/wave_times.py 128 gpurun_out/r06/wave_bd_loops_b128.json > gpurun_out/r06/wave_bd_loops.log 2>&1
