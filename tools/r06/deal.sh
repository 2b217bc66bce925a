# r06: lanes dealing variants — per-wave times (counter build), then bench A/B pairs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
P=heif_amd/libheifgpu_prof.so
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "failed_reload or rows_mode_removed or status_sticky" > gpurun_out/r06/gpu_new_tests.log 2>&1 && tail -1 gpurun_out/r06/gpu_new_tests.log &&
HEIFGPU_LIBRARY=$P timeout -k 10 200 python -u tools/wave_times.py 1 gpurun_out/r06/wave_b1_ppw1.json 1 &&
for d in bytes chain light chain_light; do
  HEIFGPU_LANES_DEAL=$d HEIFGPU_LIBRARY=$P timeout -k 10 200 python -u tools/wave_times.py 128 gpurun_out/r06/wave_b128_$d.json || exit 1
done &&
timeout -k 10 900 bash tools/ab.sh -r 1 base deal_chain:HEIFGPU_LANES_DEAL=chain deal_light:HEIFGPU_LANES_DEAL=light deal_cl:HEIFGPU_LANES_DEAL=chain_light
AB_ARGS="--batch 16 --parse spread" timeout -k 10 300 bash tools/ab.sh sp16 sp16_rows:HEIFGPU_SPREAD_ORDER=rows &&
AB_ARGS="--batch 32 --parse spread" timeout -k 10 300 bash tools/ab.sh sp32_rows:HEIFGPU_SPREAD_ORDER=rows &&
AB_ARGS="--batch 64 --parse spread" timeout -k 10 300 bash tools/ab.sh sp64_rows:HEIFGPU_SPREAD_ORDER=rows &&
AB_ARGS="--batch 1" timeout -k 10 300 bash tools/ab.sh b1 b1_rows:HEIFGPU_SPREAD_ORDER=rows
