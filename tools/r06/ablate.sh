# r06: co-run cost of each reconstruction stage on the pipelined step (measurement build: wrong pixels)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=HEIFGPU_LIBRARY=heif_amd/libheifgpu_ablate.so
timeout -k 10 900 bash tools/ab.sh -r 2 full:$L no_xf:$L,HEIFGPU_ABLATE=1 no_intra:$L,HEIFGPU_ABLATE=2 no_lf:$L,HEIFGPU_ABLATE=12 parse_only:$L,HEIFGPU_ABLATE=15
