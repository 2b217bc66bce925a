# r05: 16x16 / 32x32 inverse transforms on the int8 MFMA (mfma): GPU suite on mfma, A/B at 128
# images against the current build, one image, and kernel traces of both at 128 images
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r05
V=HEIFGPU_LIBRARY=heif_amd/libheifgpu
HEIFGPU_LIBRARY=heif_amd/libheifgpu_mfma.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests_mfma.log 2>&1 &&
AB_STEPS=10 timeout -k 10 700 bash tools/ab.sh -r 2 cur mfma:${V}_mfma.so > gpurun_out/r05/ab_b128_mfma.txt 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 300 bash tools/ab.sh -r 1 cur mfma:${V}_mfma.so > gpurun_out/r05/ab_b1_mfma.txt 2>&1 &&
mkdir -p gpurun_out/r05/kt_cur gpurun_out/r05/kt_mfma && cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r05/kt_cur" -o kt --output-format csv -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-e2e > "$R/gpurun_out/r05/kt_cur/bench.json" 2>&1 &&
HEIFGPU_LIBRARY=$R/heif_amd/libheifgpu_mfma.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r05/kt_mfma" -o kt --output-format csv -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-e2e > "$R/gpurun_out/r05/kt_mfma/bench.json" 2>&1
