# r06: the lanes sub-block unit's phases (prof-sb build: header, sig loop, greater1/2, rest), 128 images
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
HEIFGPU_LIBRARY=heif_amd/libheifgpu_profsb.so timeout -k 10 300 python -u tools/parse_prof.py 128 gpurun_out/r06/profsb_lanes_b128.json lanes > gpurun_out/r06/profsb_lanes.log 2>&1; rc=$?; tail -3 gpurun_out/r06/profsb_lanes.log; exit $rc
