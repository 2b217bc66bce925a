# Round profile (run on the final code; tags from ROUND, default r06): kernel-trace stats + corrected HBM traffic of the default bench
# (config 4) and of config 5, the parse's SQ counters (lanes at 128 images, spread at one image, spread on
# config 5), and the one-image kernel trace.  tools/summarize_profile.py copies them into profiles/<round>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
RD=${ROUND:-r06}
timeout -k 10 900 bash tools/profile_round.sh $RD &&
BENCH_ARGS="--workload config5 --batch 1" timeout -k 10 600 bash tools/profile_round.sh ${RD}c5 &&
timeout -k 10 600 bash tools/pmc_parse.sh &&
PARSE=spread PMC_BATCH=1 timeout -k 10 400 bash tools/pmc_parse.sh &&
PARSE=spread WORKLOAD=config5 PMC_BATCH=1 timeout -k 10 400 bash tools/pmc_parse.sh &&
mkdir -p gpurun_out/prof_${RD}b1 && cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${RD}b1/kt" -o kt --output-format csv -- \
    python3 "$R/bench.py" --batch 1 --no-e2e > "$R/gpurun_out/prof_${RD}b1/bench.json" 2> "$R/gpurun_out/prof_${RD}b1/bench.err" &&
echo final profile done
