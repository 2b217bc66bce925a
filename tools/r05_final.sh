# r05 final: the round profile (tools/r05_profile.sh) and the per-kernel instruction mix
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
timeout -k 10 900 bash tools/r05_profile.sh > gpurun_out/r05_final_profile.log 2>&1 &&
cd "$R" && timeout -k 10 300 bash tools/pmc_kernels.sh b128_final2 > gpurun_out/pmc_kernels_b128_final2.txt 2>&1
