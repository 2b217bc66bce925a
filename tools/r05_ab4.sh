# r05: k_intra register pressure A/B at 128 images: windows built per use (iw), and with the
# window block's address in a VGPR (iwv), against the current build
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 600 bash tools/ab.sh -r 2 cur iw:${V}_iw.so iwv:${V}_iwv.so \
    > gpurun_out/r05/ab_b128_intra.txt 2>&1
