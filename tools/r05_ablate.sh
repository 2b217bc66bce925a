# r05: co-run cost of each reconstruction stage on the 128-image step (measurement build
# libheifgpu_ablate.so: HEIFGPU_ABLATE bits drop stages, wrong pixels, --verify 0)
set -o pipefail
mkdir -p gpurun_out/r05
L=HEIFGPU_LIBRARY=heif_amd/libheifgpu_ablate.so
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 1 all:$L none:$L,HEIFGPU_ABLATE=15 noxf:$L,HEIFGPU_ABLATE=1 \
    nointra:$L,HEIFGPU_ABLATE=2 nolf:$L,HEIFGPU_ABLATE=12 nosao:$L,HEIFGPU_ABLATE=8 \
    > gpurun_out/r05/ab_ablate.txt 2>&1
