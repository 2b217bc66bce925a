"""A plain C program compiled with gcc against include/heifgpu.h and linked
with libheifgpu.so: the ABI as a non-Python host sees it (struct layouts,
error codes, parse -> info -> tile_params; on the GPU the one-shot decode and
the tile-split + gather path, hashed against the golden planes)."""
import hashlib
import json
import pathlib
import subprocess

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
SRC = ROOT / "tests" / "c_caller" / "heifgpu_caller.c"
GOLDEN = ROOT / "tests" / "golden" / "halfmoonbay.heic"


@pytest.fixture(scope="module")
def caller(tmp_path_factory):
    exe = tmp_path_factory.mktemp("c_caller") / "heifgpu_caller"
    cmd = ["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
           f"-I{ROOT / 'include'}", "-I/opt/rocm/include", str(SRC),
           f"-L{ROOT / 'heif_amd'}", "-lheifgpu", "-L/opt/rocm/lib", "-lamdhip64",
           f"-Wl,-rpath,{ROOT / 'heif_amd'}", "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_c_host_parse_info_tile_params(caller):
    r = subprocess.run([str(caller), str(GOLDEN)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "host ABI ok: 4032x3024 grid 6x8, 48 tiles" in r.stdout


@pytest.mark.gpu
def test_c_host_decode_and_tile_gather(caller, tmp_path):
    out = tmp_path / "planes.bin"
    r = subprocess.run([str(caller), str(GOLDEN), "--decode", str(out)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    raw = np.fromfile(out, dtype=np.uint8)
    ny, nc = 4032 * 3024, 2016 * 1512
    assert raw.size == 2 * (ny + 2 * nc)
    full, merged = raw[: ny + 2 * nc], raw[ny + 2 * nc:]
    gold = json.loads((ROOT / "tests" / "golden" / "halfmoonbay_planes.json").read_text())["planes"]
    planes = {"y": full[:ny], "cb": full[ny:ny + nc], "cr": full[ny + nc:]}
    for name, arr in planes.items():
        assert hashlib.sha256(arr.tobytes()).hexdigest() == gold[name], name
    assert np.array_equal(full, merged), "two tile subsets gathered differ from the one-shot decode"
