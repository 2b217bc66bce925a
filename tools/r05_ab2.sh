# r05: queue select as explicit v_cndmask (HG_QSEL_ASM) A/B at 128 images and one image;
# co-run ablation of the reconstruction stages
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 600 bash tools/ab.sh -r 2 cur qasm:${V}_qasm.so row256:${V}_row256.so > gpurun_out/r05/ab_b128_qasm.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 300 bash tools/ab.sh -r 1 cur qasm:${V}_qasm.so row256:${V}_row256.so \
    > gpurun_out/r05/ab_b1_qasm.txt 2>&1 &&
bash tools/r05_ablate.sh
