"""Guard on the occupancy the kernels are tuned for.

The measured step rests on register budgets that a compiler or ROCm change
could silently move:
- k_parse_lanes at exactly 2 waves per SIMD (the inline-asm v175 floor plus
  amdgpu_waves_per_eu(2)): at 3 the reconstruction kernels of the previous
  decode find no room beside it and the step loses 6-8 %;
- k_transform at 7 waves per SIMD (its co-run residency beside the parse);
- k_intra at 5 or more (amdgpu_waves_per_eu(5));
- no product kernel touching scratch memory (a spill to scratch is a
  per-lane memory round trip inside a hot loop).

The product objects are compiled here exactly as the library Makefile builds
them (per-TU flags included: `make resource-usage`), with the AMDGPU
resource-usage remarks, and parsed.  A second build without the parse's VGPR
floor (-DHG_PARSE_NO_VGPR_FLOOR) shows the guard catches its removal.
No GPU is needed: hipcc cross-compiles gfx950.
"""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "heif_amd" / "csrc"

pytestmark = pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None and shutil.which("hipcc") is None,
                                reason="no hipcc")


def _usage(tmp: Path, extra: str = "", objs=None) -> dict:
    """{demangled-ish kernel name: {field: int}} from the remarks of one build."""
    build = tmp / "ru"
    if objs is None:
        r = subprocess.run(["make", "-s", "-C", str(CSRC), "-j8", "resource-usage", f"RU_BUILD={build}"]
                           + ([f"CXXFLAGS=-O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter {extra}"]
                              if extra else []),
                           capture_output=True, text=True, timeout=900)
        text = r.stdout + r.stderr
    else:
        targets = [str(build / o) for o in objs]
        r = subprocess.run(["make", "-s", "-C", str(CSRC), "-j8", f"BUILD={build}",
                            "EXTRA=-Rpass-analysis=kernel-resource-usage " + extra] + targets,
                           capture_output=True, text=True, timeout=900)
        text = r.stdout + r.stderr
    assert r.returncode == 0, text[-3000:]
    out, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z][A-Za-z ]*?)(?: \[[^\]]*\])?: (\d+)", line)
        if m and cur:
            out[cur][m.group(1).strip()] = int(m.group(2))
    assert out, text[-3000:]
    return out


def _find(usage: dict, pattern: str) -> dict:
    hits = {k: v for k, v in usage.items() if re.search(pattern, k)}
    assert hits, f"no kernel matches {pattern}: {sorted(usage)}"
    return hits


@pytest.fixture(scope="module")
def usage(tmp_path_factory):
    return _usage(tmp_path_factory.mktemp("ru_product"))


def test_parse_lanes_two_waves_per_simd(usage):
    for name, u in _find(usage, r"k_parse_lanes").items():
        assert u["Occupancy"] == 2, (name, u)
        assert u["VGPRs"] > 168, (name, u)  # the floor: at <= 168 a SIMD holds 3


def test_transform_seven_waves_per_simd(usage):
    for name, u in _find(usage, r"k_transform").items():
        assert u["Occupancy"] == 7, (name, u)


def test_intra_at_least_five_waves_per_simd(usage):
    for name, u in _find(usage, r"k_intraIL|k_intra[^_]").items():
        assert u["Occupancy"] >= 5, (name, u)


def test_no_product_kernel_uses_scratch(usage):
    bad = {k: v for k, v in usage.items() if v.get("ScratchSize", 0) != 0 or v.get("VGPRs Spill", 0) != 0}
    assert not bad, bad


def test_guard_catches_removed_vgpr_floor(tmp_path):
    """Without the v175 clobber the lanes parse fits 3 waves per SIMD, which the
    first test above would reject."""
    u = _usage(tmp_path, "-DHG_PARSE_NO_VGPR_FLOOR", objs=["kernels/parse_lanes.o"])
    occ = [v["Occupancy"] for k, v in u.items() if "k_parse_lanes" in k]
    assert occ and all(o != 2 for o in occ), u
