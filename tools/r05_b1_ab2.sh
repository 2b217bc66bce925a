# r05: scalar-engine variants, one-image latency (same box): cur (s_cselect decision),
# old (r04 decision), eng / hot (fewer state fields made scalar)
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread \
    -k "parse_modes or streaming or halfmoonbay_bit_exact" > gpurun_out/r05/gpu_b1ab2.log 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 900 bash tools/ab.sh -r 3 cur old:HEIFGPU_LIBRARY=heif_amd/libheifgpu_old.so \
    eng:HEIFGPU_LIBRARY=heif_amd/libheifgpu_eng.so hot:HEIFGPU_LIBRARY=heif_amd/libheifgpu_hot.so > gpurun_out/r05/ab_b1_engine.txt 2>&1
