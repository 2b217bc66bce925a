# r05: scalar engine (spread / solo parse) variants, one-image latency, same box; GPU parity first.
# cur: s_cselect decision, 4-slot sig context word above 4x4, engine + tree state scalar, seq table
# in VGPR lanes, greater1 position after the loop; each other build undoes one of these
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_synth.py -x -q --timeout 200 --timeout-method thread \
    -k "parse_modes or streaming or halfmoonbay_bit_exact or solo or spread" > gpurun_out/r05/gpu_b1ab3.log 2>&1 &&
AB_ARGS="--batch 1" AB_STEPS=20 timeout -k 10 1000 bash tools/ab.sh -r 2 cur generic:HEIFGPU_LIBRARY=heif_amd/libheifgpu_generic.so \
    seqlds:HEIFGPU_LIBRARY=heif_amd/libheifgpu_seqlds.so uniall:HEIFGPU_LIBRARY=heif_amd/libheifgpu_uniall.so \
    tbset:HEIFGPU_LIBRARY=heif_amd/libheifgpu_tbset.so lean:HEIFGPU_LIBRARY=heif_amd/libheifgpu_lean.so > gpurun_out/r05/ab_b1_sig4.txt 2>&1
