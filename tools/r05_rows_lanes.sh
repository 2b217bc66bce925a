# r05: rows parse, pictures per row wave (HEIFGPU_ROWS_LANES) x dealing (HEIFGPU_ROWS_DEAL), same box
set -o pipefail
mkdir -p gpurun_out/r05
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --verify 8 \
      > gpurun_out/r05/rl_$name.json 2> gpurun_out/r05/rl_$name.err
}
run lanes HEIFGPU_PARSE=lanes &&
run k16_l64 HEIFGPU_PARSE=rows HEIFGPU_ROWS_DEAL=16 &&
run k16_l32 HEIFGPU_PARSE=rows HEIFGPU_ROWS_DEAL=16 HEIFGPU_ROWS_LANES=32 &&
run k16_l16 HEIFGPU_PARSE=rows HEIFGPU_ROWS_DEAL=16 HEIFGPU_ROWS_LANES=16 &&
run k1_l32 HEIFGPU_PARSE=rows HEIFGPU_ROWS_LANES=32 &&
run copies_l32 HEIFGPU_PARSE=rows HEIFGPU_ROWS_DEAL=copies HEIFGPU_ROWS_LANES=32 &&
run copies_l64 HEIFGPU_PARSE=rows HEIFGPU_ROWS_DEAL=copies
