# r06: where k_intra's instructions go: SQ instruction counts and k_intra alone for measurement builds that
# drop the TB's work (HG_IABL_TB), the neighbour gather (HG_IABL_GATHER) or the prediction (HG_IABL_PRED)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
timeout -k 10 600 bash tools/ab.sh full iabl_TB:HEIFGPU_LIBRARY=heif_amd/libheifgpu_iabl_TB.so iabl_GATHER:HEIFGPU_LIBRARY=heif_amd/libheifgpu_iabl_GATHER.so iabl_PRED:HEIFGPU_LIBRARY=heif_amd/libheifgpu_iabl_PRED.so &&
cd /tmp && export TMPDIR=/tmp &&
for v in full iabl_TB iabl_GATHER iabl_PRED; do
  lib=$R/heif_amd/libheifgpu.so; [ $v != full ] && lib=$R/heif_amd/libheifgpu_$v.so
  HEIFGPU_LIBRARY=$lib timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_BUSY_CU_CYCLES \
    -d $R/gpurun_out/r06/sqi_$v -o p --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --verify 0 > $R/gpurun_out/r06/sqi_$v.log 2>&1 || exit 1
done &&
python3 - "$R/gpurun_out/r06" <<'PY'
import csv, collections, glob, sys
for v in ("full", "iabl_TB", "iabl_GATHER", "iabl_PRED"):
    acc = collections.defaultdict(float); nd = set()
    for f in glob.glob(f"{sys.argv[1]}/sqi_{v}/**/p_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_intra" in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"]); nd.add((f, r["Dispatch_Id"]))
    n = max(1, len(nd))
    print(f"{v:>12} k_intra per launch: " + "  ".join(f"{k[9:]} {x / n / 1e9:.3f} G" for k, x in sorted(acc.items())))
PY
cd "$R" && timeout -k 10 600 python3 -u tools/r06/mixed_parse.py 16,16,1 24,8,1 32,16,1 32,32,2 16,48,2 > gpurun_out/r06/mixed_parse.log 2>&1; cat gpurun_out/r06/mixed_parse.log
