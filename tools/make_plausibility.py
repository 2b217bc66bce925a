"""Writes tests/golden/plausibility.json: the tests/plausibility.py metrics of
the oracle's halfmoonbay decode (primary luma + HDR gain map item 52)."""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import plausibility  # noqa: E402
from oracle import oracle  # noqa: E402

data = (ROOT / "tests/golden/halfmoonbay.heic").read_bytes()
luma = oracle.decode_heic(data, with_checks=False).y
tiles, (ho, hl) = oracle.list_tiles(data, 52)
o, n = tiles[0]
gain, _, _ = oracle.decode_tile(data[ho:ho + hl], data[o:o + n], 2016, 1512)
m = plausibility.metrics(luma, gain)
plausibility.check(m)
out = {"generator": "tools/make_plausibility.py", "thresholds": plausibility.THRESHOLDS,
       "metrics": {k: round(v, 6) if isinstance(v, float) else v for k, v in m.items()}}
(ROOT / "tests/golden/plausibility.json").write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out["metrics"]))
