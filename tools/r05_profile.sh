# r05 round profile with the final code (on the GPU box, repo root):
#  1. tools/profile_round.sh r05: kernel-trace stats of the default bench, FETCH_SIZE / WRITE_SIZE passes
#  2. the parse's SQ counters, lanes (128 images) and spread (1 image)
#  3. kernel trace of the one-image bench (config 3)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
timeout -k 10 1200 bash tools/profile_round.sh r05 > gpurun_out/r05_profile_round.log 2>&1 &&
PARSE=lanes timeout -k 10 600 bash tools/pmc_parse.sh > gpurun_out/r05_pmc_lanes.log 2>&1 &&
PARSE=spread PMC_BATCH=1 timeout -k 10 400 bash tools/pmc_parse.sh > gpurun_out/r05_pmc_spread.log 2>&1 &&
mkdir -p gpurun_out/prof_r05_b1 && cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r05_b1/kt" -o kt --output-format csv -- \
    python3 "$R/bench.py" --batch 1 --steps 20 --warmup 2 --no-e2e > "$R/gpurun_out/prof_r05_b1/bench.json" 2> "$R/gpurun_out/prof_r05_b1/bench.err"
# 4. the plain bench line (no profiler) and the one-image line
cd "$R" && timeout -k 10 400 python3 bench.py > gpurun_out/r05_bench_plain.json 2> gpurun_out/r05_bench_plain.err &&
timeout -k 10 300 python3 bench.py --batch 1 --steps 20 --warmup 2 > gpurun_out/r05_bench_b1.json 2> gpurun_out/r05_bench_b1.err
