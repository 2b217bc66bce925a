# r05: the compiler's scheduling strategies on the whole library (sch1 max-ilp, sch2
# max-memory-clause, sch3 iterative-ilp) against the current build: 128 images and one image
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
AB_STEPS=10 timeout -k 10 900 bash tools/ab.sh -r 2 cur sch1:${V}_sch1.so sch2:${V}_sch2.so sch3:${V}_sch3.so \
    > gpurun_out/r05/ab_b128_sched_strat.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 400 bash tools/ab.sh -r 1 cur sch1:${V}_sch1.so sch2:${V}_sch2.so sch3:${V}_sch3.so \
    > gpurun_out/r05/ab_b1_sched_strat.txt 2>&1
