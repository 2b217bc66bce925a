# r06: mixed-parse feasibility probe (tools/r06/mixed_parse.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
timeout -k 10 600 python3 -u tools/r06/mixed_parse.py 16,16,1 24,8,1 8,24,1 32,16,1 32,32,2 16,48,2 > gpurun_out/r06/mixed_parse.log 2>&1; rc=$?; cat gpurun_out/r06/mixed_parse.log; exit $rc
