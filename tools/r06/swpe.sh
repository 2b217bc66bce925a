# r06: spread kernel at a 6-waves-per-SIMD register budget (80 VGPRs, 36 B/lane scratch) against 5 (89 VGPRs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu_swpe6.so
for b in 16 32 1; do
  AB_ARGS="--batch $b" timeout -k 10 600 bash tools/ab.sh -r 2 b${b}:HEIFGPU_PARSE=spread b${b}_w6:HEIFGPU_PARSE=spread,$V || exit 1
done
