# r06: lanes-only unit loops and sub-block gating (odd passes run the sub-block unit only with N lanes or more):
# GPU suite on the loops build, then 20-step bench pairs against HEAD (libheifgpu_base.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r06/gpu_tests_gate.log 2>&1 &&
tail -1 gpurun_out/r06/gpu_tests_gate.log &&
AB_STEPS=20 timeout -k 10 900 bash tools/ab.sh -r 2 base:HEIFGPU_LIBRARY=heif_amd/libheifgpu_base.so loops \
  gate8:HEIFGPU_LIBRARY=heif_amd/libheifgpu_gate8.so gate16:HEIFGPU_LIBRARY=heif_amd/libheifgpu_gate16.so &&
AB_ARGS="--batch 1" timeout -k 10 300 bash tools/ab.sh b1_base:HEIFGPU_LIBRARY=heif_amd/libheifgpu_base.so b1_loops
