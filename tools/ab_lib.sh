# A library change against the HEAD build (libheifgpu_base.so): GPU suite on the new build, same-box
# bench pairs at 128 images (and one image), and one SQ instruction-mix pass per kernel for both builds.
# usage: bash tools/ab_lib.sh <name> [extra ab.sh specs...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
N=${1:-new}; shift
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r06/gpu_tests_$N.log 2>&1 &&
tail -1 gpurun_out/r06/gpu_tests_$N.log &&
timeout -k 10 700 bash tools/ab.sh -r 2 base:HEIFGPU_LIBRARY=heif_amd/libheifgpu_base.so $N "$@" &&
AB_ARGS="--batch 1" timeout -k 10 300 bash tools/ab.sh b1_base:HEIFGPU_LIBRARY=heif_amd/libheifgpu_base.so b1_$N &&
cd /tmp && export TMPDIR=/tmp &&
for v in base $N; do
  lib=$R/heif_amd/libheifgpu.so; [ $v = base ] && lib=$R/heif_amd/libheifgpu_base.so
  HEIFGPU_LIBRARY=$lib timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_BUSY_CU_CYCLES \
    -d $R/gpurun_out/r06/sq_$v -o p --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --verify 0 > $R/gpurun_out/r06/sq_$v.log 2>&1 || exit 1
done &&
python3 - "$R/gpurun_out/r06" base $N <<'PY'
import csv, collections, glob, sys
for v in sys.argv[2:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); nd = collections.defaultdict(set)
    for f in glob.glob(f"{sys.argv[1]}/sq_{v}/**/p_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hg::", "")
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); nd[k].add((f, r["Dispatch_Id"]))
    for k in sorted(acc):
        if not k.startswith("k_"): continue
        n = max(1, len(nd[k]))
        c = acc[k]
        print(f"{v:>6} {k:34s} VALU {c['SQ_INSTS_VALU']/n/1e9:6.3f} G  SALU {c['SQ_INSTS_SALU']/n/1e9:6.3f} G  LDS {c['SQ_INSTS_LDS']/n/1e9:6.3f} G  BR {c['SQ_INSTS_BRANCH']/n/1e9:6.3f} G")
PY
