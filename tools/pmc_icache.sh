# Instruction-cache counters per kernel (each kernel alone: --pmc serialises dispatches): 128 images and one image
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/icache
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ -d $R/gpurun_out/icache/b128 -o p --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --verify 0 > $R/gpurun_out/icache/b128.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ -d $R/gpurun_out/icache/b1 -o p --output-format csv -- python3 $R/bench.py --batch 1 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --verify 0 > $R/gpurun_out/icache/b1.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_IFETCH SQC_TC_INST_REQ SQ_WAVES SQ_WAIT_INST_ANY -d $R/gpurun_out/icache/b128t -o p --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --verify 0 > $R/gpurun_out/icache/b128t.log 2>&1
