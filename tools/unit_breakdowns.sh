# The counter builds' cycle breakdowns on the current code (make -C heif_amd/csrc prof prof-sb first):
# lanes at 128 images and spread at one image, by unit kind (prof) and by sub-block phase (prof-sb),
# plus the per-wave records (tools/wave_times.py).  Writes gpurun_out/units/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/units
P=heif_amd/libheifgpu_prof.so S=heif_amd/libheifgpu_profsb.so
HEIFGPU_LIBRARY=$P timeout -k 10 300 python -u tools/parse_prof.py 128 gpurun_out/units/parse_units_lanes_b128.json > gpurun_out/units/u1.log 2>&1 &&
HEIFGPU_LIBRARY=$P timeout -k 10 300 python -u tools/parse_prof.py 1 gpurun_out/units/parse_units_spread_b1.json > gpurun_out/units/u2.log 2>&1 &&
HEIFGPU_LIBRARY=$S timeout -k 10 300 python -u tools/parse_prof.py 128 gpurun_out/units/profsb_lanes_b128.json > gpurun_out/units/u3.log 2>&1 &&
HEIFGPU_LIBRARY=$S timeout -k 10 300 python -u tools/parse_prof.py 1 gpurun_out/units/profsb_spread_b1.json > gpurun_out/units/u4.log 2>&1 &&
HEIFGPU_LIBRARY=$P timeout -k 10 300 python -u tools/wave_times.py 128 gpurun_out/units/wave_bd_b128.json > gpurun_out/units/u5.log 2>&1 &&
HEIFGPU_LIBRARY=$S timeout -k 10 300 python -u tools/wave_times.py 128 gpurun_out/units/wave_bd_sb_b128.json > gpurun_out/units/u6.log 2>&1 &&
tail -n 2 gpurun_out/units/u*.log
