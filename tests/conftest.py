"""Shared fixtures. `-m "not gpu"` runs everywhere; `-m gpu` needs an MI355X."""
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))


def make_emu(target: str = "emu-fast") -> None:
    """Build a host-emulation target of heif_amd/csrc under an exclusive file
    lock, so parallel test workers (pytest -n) never run make on the same
    build directory at once."""
    import fcntl
    import subprocess

    csrc = ROOT / "heif_amd" / "csrc"
    (csrc / "build").mkdir(exist_ok=True)
    with open(csrc / "build" / ".emu.lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", str(csrc), target], check=True, capture_output=True)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) — run with -m gpu")


@pytest.fixture(scope="session")
def halfmoonbay() -> bytes:
    return (GOLDEN / "halfmoonbay.heic").read_bytes()


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle

    return oracle


@pytest.fixture(scope="session")
def oracle_halfmoonbay(oracle_mod, halfmoonbay):
    return oracle_mod.decode_heic(halfmoonbay)
