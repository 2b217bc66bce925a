# r06: the tuning knobs re-checked on the current kernels (bench pairs at 128 images)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
timeout -k 10 1200 bash tools/ab.sh base iw1:HEIFGPU_INTRA_WAVES=1 iw3:HEIFGPU_INTRA_WAVES=3 iw4:HEIFGPU_INTRA_WAVES=4 \
    isplit:HEIFGPU_INTRA_SPLIT=1 dbk1:HEIFGPU_DBK_BLOCKS=1 dbk4:HEIFGPU_DBK_BLOCKS=4 sao2:HEIFGPU_SAO_BLOCKS=2 \
    sao8:HEIFGPU_SAO_BLOCKS=8 prep:HEIFGPU_PREP_STREAM=1 base2
