"""Shared fixtures. `-m "not gpu"` runs everywhere; `-m gpu` needs an MI355X."""
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))


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
