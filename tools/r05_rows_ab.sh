# r05: rows-parse bring-up on the GPU: parity of the new mode, then bench A/B
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread \
    -k "parse_modes or bench_shard_every_image or status_sticky" > gpurun_out/r05/gpu_rows.log 2>&1 &&
for m in lanes rows; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --parse $m > gpurun_out/r05/ab_$m.json 2> gpurun_out/r05/ab_$m.err || exit 1
done &&
HEIFGPU_ROWS_DEAL=copies timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --parse rows > gpurun_out/r05/ab_rows_copies.json 2> gpurun_out/r05/ab_rows_copies.err
