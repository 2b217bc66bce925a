# r05: sub-block tail trims (positions past the first eight from the greater1 loop, greater2 nibble
# by shift, s_bitreplicate nibble spreading) against the previous build, one image and 128 images
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_synth.py -x -q --timeout 200 --timeout-method thread \
    -k "parse_modes or streaming or halfmoonbay_bit_exact or solo or spread or lanes" > gpurun_out/r05/gpu_b1ab4.log 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 600 bash tools/ab.sh -r 2 cur base:HEIFGPU_LIBRARY=heif_amd/libheifgpu_base.so \
    nobr:HEIFGPU_LIBRARY=heif_amd/libheifgpu_nobr.so > gpurun_out/r05/ab_b1_tail.txt 2>&1 &&
AB_STEPS=10 timeout -k 10 600 bash tools/ab.sh -r 2 cur base:HEIFGPU_LIBRARY=heif_amd/libheifgpu_base.so > gpurun_out/r05/ab_b128_tail.txt 2>&1
