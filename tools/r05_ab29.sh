# r05: code-generation flags of the solo / spread translation unit (sv1 iterative-minreg, sv2 SLP
# threshold +2, sv3 no SLP, sv4 unroll threshold 100) against the current build, one image
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 600 bash tools/ab.sh -r 2 cur sv1:${V}_sv1.so sv2:${V}_sv2.so sv3:${V}_sv3.so sv4:${V}_sv4.so \
    > gpurun_out/r05/ab_b1_soloflags.txt 2>&1
