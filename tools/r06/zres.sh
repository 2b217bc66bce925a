# r06: residual runs by CTB in z-order (k_transform -> k_intra): GPU suite, same-box A/B against the
# previous layout (libheifgpu_base.so), and FETCH_SIZE / WRITE_SIZE per kernel for both
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r06/gpu_tests_zres.log 2>&1 &&
tail -1 gpurun_out/r06/gpu_tests_zres.log &&
timeout -k 10 600 bash tools/ab.sh -r 2 base:HEIFGPU_LIBRARY=heif_amd/libheifgpu_base.so zres &&
AB_ARGS="--batch 1" timeout -k 10 300 bash tools/ab.sh b1_base:HEIFGPU_LIBRARY=heif_amd/libheifgpu_base.so b1_zres &&
cd /tmp && export TMPDIR=/tmp &&
for v in base zres; do
  lib=heif_amd/libheifgpu.so; [ $v = base ] && lib=heif_amd/libheifgpu_base.so
  for c in FETCH_SIZE WRITE_SIZE; do
    HEIFGPU_LIBRARY=$R/$lib timeout -s KILL 300 rocprofv3 --pmc $c -d $R/gpurun_out/r06/pmc_$v/$c -o p --output-format csv -- \
      python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --verify 0 > $R/gpurun_out/r06/pmc_${v}_$c.log 2>&1 || exit 1
  done
done &&
python3 - "$R/gpurun_out/r06" <<'PY'
import csv, collections, glob, sys
for v in ("base", "zres"):
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        acc = collections.defaultdict(list)
        for f in glob.glob(f"{sys.argv[1]}/pmc_{v}/{c}/**/p_counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == c:
                    acc[r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hg::", "")].append(float(r["Counter_Value"]))
        print(v, c, {k: round(sum(x) / len(x) * 1024 / 1e9, 3) for k, x in acc.items()}, "(GB per launch, raw KiB x 1024 / 1e9)")
PY
cd "$R" &&
timeout -k 10 300 python3 bench.py --workload config5 --batch 1 --split tiles --steps 10 --warmup 3 --no-e2e > gpurun_out/r06/config5_split_w1.json 2> gpurun_out/r06/config5_split_w1.err &&
tail -c 1200 gpurun_out/r06/config5_split_w1.json &&
AB_ARGS="--batch 16 --parse spread" timeout -k 10 300 bash tools/ab.sh sp16 sp16_nouni:HEIFGPU_LIBRARY=heif_amd/libheifgpu_nouni.so &&
AB_ARGS="--batch 32 --parse spread" timeout -k 10 300 bash tools/ab.sh sp32 sp32_nouni:HEIFGPU_LIBRARY=heif_amd/libheifgpu_nouni.so &&
AB_ARGS="--batch 16 --parse spread" timeout -k 10 300 bash tools/ab.sh sp16_rows:HEIFGPU_SPREAD_ORDER=rows &&
AB_ARGS="--batch 1" timeout -k 10 300 bash tools/ab.sh b1_rows:HEIFGPU_SPREAD_ORDER=rows
