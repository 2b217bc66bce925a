# r06: spread parse in row-major job order (HEIFGPU_SPREAD_ORDER=rows) against picture-major spread and
# lanes, at 4..128 images (halfmoonbay permutations) and on the distinct-tile control at 16 / 32
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for b in 4 8 16 32 64 128; do
  AB_ARGS="--batch $b" timeout -k 10 900 bash tools/ab.sh b${b}_spread:HEIFGPU_PARSE=spread b${b}_rows:HEIFGPU_PARSE=spread,HEIFGPU_SPREAD_ORDER=rows b${b}_lanes:HEIFGPU_PARSE=lanes || exit 1
done
for b in 16 32; do
  AB_ARGS="--batch $b --workload config4u" timeout -k 10 900 bash tools/ab.sh u${b}_spread:HEIFGPU_PARSE=spread u${b}_rows:HEIFGPU_PARSE=spread,HEIFGPU_SPREAD_ORDER=rows u${b}_lanes:HEIFGPU_PARSE=lanes || exit 1
done
