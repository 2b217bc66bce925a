# Closing lines on the final code, after profiles/<round>/ holds this round's counter files: the default
# bench (config 4, with roofline.traffic and issue), one image, config 5 (cpu_baseline, traffic, issue),
# the config-5 tile split at world 1 (per-rank parse, chain floor), the distinct-tile control, the GPU
# suite and smoke()
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/final
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1 &&
tail -1 gpurun_out/final/gpu_tests.log &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 && cat gpurun_out/final/smoke.log &&
timeout -k 10 300 python3 bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err &&
timeout -k 10 200 python3 bench.py --batch 1 --no-e2e > gpurun_out/final/bench_b1.json 2> gpurun_out/final/bench_b1.err &&
timeout -k 10 300 python3 bench.py --workload config5 --batch 1 --no-e2e > gpurun_out/final/config5_b1.json 2> gpurun_out/final/config5_b1.err &&
timeout -k 10 300 python3 bench.py --workload config5 --batch 1 --split tiles --no-e2e --no-cpu-baseline > gpurun_out/final/config5_split_w1.json 2> gpurun_out/final/config5_split_w1.err &&
timeout -k 10 300 python3 bench.py --workload config4u --no-e2e --no-cpu-baseline > gpurun_out/final/bench_config4u.json 2> gpurun_out/final/bench_config4u.err &&
for f in bench bench_b1 config5_b1 config5_split_w1 bench_config4u; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d.get('latency_ms_one_step'), d['roofline']['traffic'], (d['roofline'].get('issue') or {}).get('wave_instr_per_bin'), (d.get('cpu_baseline') or {}).get('value'), d.get('verified_images'))" gpurun_out/final/$f.json
done
