# r05: where k_intra's time goes (measurement builds, wrong pixels): no neighbour gather (ablg),
# no prediction (ablp), predict_tb returning at once (ablt), against the current build
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 700 bash tools/ab.sh -r 1 cur ablg:${V}_ablg.so ablp:${V}_ablp.so ablt:${V}_ablt.so \
    > gpurun_out/r05/ab_b128_iabl.txt 2>&1
