# r05: the parse's issue priority re-checked on the final code (pr2: s_setprio 2, pr0: none), 128 images
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 2 cur pr2:${V}_pr2.so pr0:${V}_pr0.so > gpurun_out/r05/ab_b128_prio.txt 2>&1
