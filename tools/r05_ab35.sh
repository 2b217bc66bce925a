# r05: SLP cost threshold -3 for the transform (t3) and loop-filter (l3) units, 128 images
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 2 cur t3:${V}_t3.so l3:${V}_l3.so > gpurun_out/r05/ab_b128_slp_xl.txt 2>&1
