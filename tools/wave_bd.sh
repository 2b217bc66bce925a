# Per-wave cycle breakdown of the lanes parse at 128 images (tools/wave_times.py): the counter
# build (`make -C heif_amd/csrc prof`: units per wave) and the prof-sb build (+ sub-block phases).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so timeout -k 10 300 python -u tools/wave_times.py 128 gpurun_out/r06/wave_bd_b128.json > gpurun_out/r06/wave_bd.log 2>&1 &&
HEIFGPU_LIBRARY=heif_amd/libheifgpu_profsb.so timeout -k 10 300 python -u tools/wave_times.py 128 gpurun_out/r06/wave_bd_sb_b128.json > gpurun_out/r06/wave_bd_sb.log 2>&1
