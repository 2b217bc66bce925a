# r05: distinct-tile control (config4u): lanes vs rows parse, same box
set -o pipefail
mkdir -p gpurun_out/r05
export BENCH_C4U_CACHE=/tmp/c4u_$$.npz
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload config4u --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
      --verify 16 > gpurun_out/r05/c4u_$name.json 2> gpurun_out/r05/c4u_$name.err
}
run lanes HEIFGPU_PARSE=lanes &&
run rows64 HEIFGPU_PARSE=rows &&
run rows32 HEIFGPU_PARSE=rows HEIFGPU_ROWS_LANES=32 &&
run lanes2 HEIFGPU_PARSE=lanes
rc=$?; rm -f $BENCH_C4U_CACHE; exit $rc
