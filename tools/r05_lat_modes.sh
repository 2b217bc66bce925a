# r05: one decode's latency and the pipelined rate per parse geometry and batch size
# (bench.py --batch B --parse MODE), collected into gpurun_out/r05/latency_modes.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r05/lat
mkdir -p $O
for run in 1:spread 1:solo 1:lanes 1:auto 4:spread 4:lanes 4:auto 16:spread 16:lanes 16:auto 128:lanes 128:spread; do
    b=${run%%:*}; m=${run##*:}
    steps=10; [ "$b" = 128 ] && steps=5
    timeout -k 10 300 python3 bench.py --batch $b --parse $m --steps $steps --warmup 2 --no-cpu-baseline --no-e2e \
        > $O/b${b}_${m}.json 2> $O/b${b}_${m}.err || exit 1
done
python3 - "$O" <<'PY'
import json, pathlib, sys
o = pathlib.Path(sys.argv[1]); runs = {}
for f in sorted(o.glob("b*.json")):
    d = json.loads(f.read_text().strip().splitlines()[-1])
    runs[f.stem] = {k: d.get(k) for k in ("value", "ms_per_step", "latency_ms_one_step")}
    runs[f.stem]["geometry"] = d.get("roofline", {}).get("parse_geometry")
    runs[f.stem]["stage_ms_alone"] = d.get("stage_ms_alone")
json.dump({"what": "bench.py --batch B --parse MODE --steps 10 (5 at B = 128) --warmup 2 --no-cpu-baseline "
           "--no-e2e (tools/r05_lat_modes.sh) on one MI355X; halfmoonbay permutations; Mpixels/s, ms; "
           "latency_ms_one_step = wall clock of one decode alone", "runs": runs},
          open(o.parent / "latency_modes.json", "w"), indent=1)
PY
