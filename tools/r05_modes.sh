# r05: GPU suite; lanes-engine A/B at 128 images (32x32 scan tables, context-indexed
# state rows, branch-free sig loop, queue select) and one image (spread)
set -o pipefail
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05/gpu_tests.log 2>&1 &&
AB_STEPS=10 timeout -k 10 800 bash tools/ab.sh -r 2 cur noscan:${V}_noscan.so rowctx:${V}_rowctx.so \
    rs:${V}_rs.so qsel:${V}_qsel.so > gpurun_out/r05/ab_b128_engine.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 400 bash tools/ab.sh -r 2 cur noscan:${V}_noscan.so \
    rs:${V}_rs.so > gpurun_out/r05/ab_b1_engine.txt 2>&1
