# r05: the int8 MFMA transform only for TBs with many coded columns (mfa: 32x32 with >= 16
# columns; mfb: 32x32 >= 8, 16x16 >= 12; mfc: 32x32 >= 24), A/B at 128 images
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 2 cur mfa:${V}_mfa.so mfb:${V}_mfb.so mfc:${V}_mfc.so \
    > gpurun_out/r05/ab_b128_mfx.txt 2>&1
