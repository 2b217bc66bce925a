# r05: the whole GPU suite on the current tree, the default bench line, then one-image A/B of two scalar-state sets
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r05/bench_check.json 2> gpurun_out/r05/bench_check.err &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 600 bash tools/ab.sh -r 2 cur lean:HEIFGPU_LIBRARY=heif_amd/libheifgpu_lean.so \
    tbset:HEIFGPU_LIBRARY=heif_amd/libheifgpu_tbset.so > gpurun_out/r05/ab_b1_sets.txt 2>&1
