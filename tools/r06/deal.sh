# r06: lanes dealing variants (HEIFGPU_LANES_DEAL) — per-wave times (counter build), then bench A/B
# pairs on the halfmoonbay shard and on the distinct-tile control (config4u)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
P=heif_amd/libheifgpu_prof.so
B=HEIFGPU_LIBRARY=heif_amd/libheifgpu_base.so  # the GPU-verified HEAD build
for d in chain light chain_light; do
  HEIFGPU_LANES_DEAL=$d HEIFGPU_LIBRARY=$P timeout -k 10 200 python -u tools/wave_times.py 128 gpurun_out/r06/wave_b128_$d.json > gpurun_out/r06/wave_$d.log 2>&1 || exit 1
  tail -1 gpurun_out/r06/wave_$d.log
done &&
timeout -k 10 900 bash tools/ab.sh -r 2 base:$B deal_chain:$B,HEIFGPU_LANES_DEAL=chain deal_light:$B,HEIFGPU_LANES_DEAL=light deal_cl:$B,HEIFGPU_LANES_DEAL=chain_light &&
AB_ARGS="--workload config4u" timeout -k 10 900 bash tools/ab.sh u_base:$B u_chain:$B,HEIFGPU_LANES_DEAL=chain u_light:$B,HEIFGPU_LANES_DEAL=light u_cl:$B,HEIFGPU_LANES_DEAL=chain_light
