# r05: instrumented parse builds (s_memtime per unit kind / sub-block phase), same box
set -o pipefail
mkdir -p gpurun_out/r05
P=heif_amd/libheifgpu_prof.so; PSB=heif_amd/libheifgpu_profsb.so
HEIFGPU_LIBRARY=$P timeout -k 10 200 python -u tools/parse_prof.py 1 gpurun_out/r05/parse_units_spread_b1.json spread > gpurun_out/r05/pp1.log 2>&1 &&
HEIFGPU_LIBRARY=$PSB timeout -k 10 200 python -u tools/parse_prof.py 1 gpurun_out/r05/profsb_spread_b1.json spread > gpurun_out/r05/pp2.log 2>&1 &&
HEIFGPU_LIBRARY=$P timeout -k 10 300 python -u tools/parse_prof.py 128 gpurun_out/r05/parse_units_lanes_b128.json lanes > gpurun_out/r05/pp3.log 2>&1 &&
HEIFGPU_LIBRARY=$P timeout -k 10 300 python -u tools/parse_prof.py 128 gpurun_out/r05/parse_units_rows_b128.json rows > gpurun_out/r05/pp4.log 2>&1
