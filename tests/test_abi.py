"""The C-ABI boundary: the library loads without a GPU, exports exactly what
include/heifgpu.h declares, and the product never touches the oracle."""
import pathlib
import re
import subprocess
import sys

from heif_amd import _lib

ROOT = pathlib.Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "heifgpu.h"


def header_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return set(re.findall(r"\b(heifgpu_[a-z0-9_]+)\s*\(", text))


def test_header_functions_are_exported():
    names = header_functions()
    assert len(names) >= 20
    for n in sorted(names):
        assert hasattr(_lib.lib, n), f"{n} declared in heifgpu.h but not exported"


def test_binding_covers_header():
    assert header_functions() == set(_lib.EXPORTS)


def test_exported_symbols_are_c_linkage():
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for n in header_functions():
        assert n in syms  # unmangled: extern "C"


def test_library_is_gfx950_code():
    # the fat binary embeds the gfx950 code-object target id
    assert b"amdgcn-amd-amdhsa--gfx950" in _lib.LIB_PATH.read_bytes()


def test_product_does_not_reference_oracle():
    pkg = ROOT / "heif_amd"
    for p in list(pkg.rglob("*.py")) + list(pkg.rglob("*.cpp")) + list(pkg.rglob("*.hpp")) + list(pkg.rglob("*.hip")):
        if "emu" in p.parts:  # the host-emulation checker links the oracle by design (test-only)
            continue
        text = p.read_text()
        assert "import oracle" not in text and "from oracle" not in text and "oracle.h" not in text, p
    deps = subprocess.run(["ldd", str(_lib.LIB_PATH)], capture_output=True, text=True).stdout
    assert "oracle" not in deps


def test_missing_library_fails_loudly(tmp_path):
    code = "import heif_amd"
    env = {"HEIFGPU_LIBRARY": str(tmp_path / "nope.so"), "PATH": "/usr/bin:/bin"}
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True)
    assert r.returncode != 0
    assert "no CPU fallback" in r.stderr


def test_last_error_after_failure():
    import ctypes

    h = ctypes.c_void_p()
    rc = _lib.lib.heifgpu_image_parse(_lib.u8buf(b"junk"), 4, ctypes.byref(h))
    assert rc == _lib.HEIFGPU_E_PARSE
    assert _lib.last_error()
