# r06: parse cycle breakdowns on the final parse code (counter builds): lanes at 128 images per unit kind,
# spread at one image per unit kind and per sub-block phase
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so timeout -k 10 300 python -u tools/parse_prof.py 128 gpurun_out/r06/parse_units_lanes_b128.json lanes > gpurun_out/r06/units_lanes.log 2>&1 && tail -3 gpurun_out/r06/units_lanes.log &&
HEIFGPU_LIBRARY=heif_amd/libheifgpu_prof.so timeout -k 10 200 python -u tools/parse_prof.py 1 gpurun_out/r06/parse_units_spread_b1.json spread > gpurun_out/r06/units_spread.log 2>&1 && tail -3 gpurun_out/r06/units_spread.log &&
HEIFGPU_LIBRARY=heif_amd/libheifgpu_profsb.so timeout -k 10 200 python -u tools/parse_prof.py 1 gpurun_out/r06/profsb_spread_b1.json spread > gpurun_out/r06/profsb_spread.log 2>&1 && tail -3 gpurun_out/r06/profsb_spread.log
