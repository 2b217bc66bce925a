# r05: rows parse with repeated bitstreams spread over K sizes per group (HEIFGPU_ROWS_DEAL), same box
set -o pipefail
mkdir -p gpurun_out/r05
run() {  # name, env..., then bench args
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --verify 8 \
      > gpurun_out/r05/deal_$name.json 2> gpurun_out/r05/deal_$name.err
}
run lanes HEIFGPU_PARSE=lanes &&
run k1 HEIFGPU_PARSE=rows &&
run k2 HEIFGPU_PARSE=rows HEIFGPU_ROWS_DEAL=2 &&
run k4 HEIFGPU_PARSE=rows HEIFGPU_ROWS_DEAL=4 &&
run k8 HEIFGPU_PARSE=rows HEIFGPU_ROWS_DEAL=8 &&
run k16 HEIFGPU_PARSE=rows HEIFGPU_ROWS_DEAL=16
