# r05: pass scheduling of k_parse_lanes A/B at 128 images: tree / TB units wanted by fewer than
# 3 lanes held back (HG_DEFER_MIN=3), and two sub-block slots per pass (HG_SB_SLOTS=2)
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 600 bash tools/ab.sh -r 2 cur d3:${V}_d3.so s2:${V}_s2.so \
    > gpurun_out/r05/ab_b128_sched.txt 2>&1
