set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r05/bench_default.json 2> gpurun_out/r05/bench_default.err &&
timeout -k 10 200 python -u bench.py --workload config5 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05/config5_b1.json 2> gpurun_out/r05/config5_b1.err &&
timeout -k 10 200 python -u bench.py --workload config5 --batch 1 --split tiles --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05/config5_split_w1.json 2> gpurun_out/r05/config5_split_w1.err
