# r05: instruction-cache counters of one 128-image bench step (per kernel; --pmc serialises
# the kernels, so these are each kernel alone).  Lists the gfx950 counters first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r05_icache"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/r05_icache/counters.txt" 2>&1 || true
grep -q SQC_ICACHE_MISSES "$R/gpurun_out/r05_icache/counters.txt" &&
timeout -s KILL 240 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES \
    -d "$R/gpurun_out/r05_icache/ic" -o ic --output-format csv -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --verify 0 > "$R/gpurun_out/r05_icache/ic.log" 2>&1
