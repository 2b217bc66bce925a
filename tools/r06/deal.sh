# r06: lanes dealing variants — per-wave times (counter build), then bench A/B pairs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
P=heif_amd/libheifgpu_prof.so
HEIFGPU_LIBRARY=$P timeout -k 10 200 python -u tools/wave_times.py 1 gpurun_out/r06/wave_b1_ppw1.json 1 &&
for d in bytes chain light chain_light; do
  HEIFGPU_LANES_DEAL=$d HEIFGPU_LIBRARY=$P timeout -k 10 200 python -u tools/wave_times.py 128 gpurun_out/r06/wave_b128_$d.json || exit 1
done &&
timeout -k 10 900 bash tools/ab.sh -r 2 base deal_chain:HEIFGPU_LANES_DEAL=chain deal_light:HEIFGPU_LANES_DEAL=light deal_cl:HEIFGPU_LANES_DEAL=chain_light
