"""The GPU kernels' own source, compiled for the host (HG_HOST_EMU: one host
thread per wave, kWave = 1), decoding halfmoonbay and diffed against the
oracle.  This runs the kernels' syntax, transform, prediction and loop-filter
logic on CPU, so kernel-logic regressions surface before a GPU is involved;
it is test infrastructure (it links the oracle), never a product path."""
import os
import pathlib
import subprocess

import pytest

from heif_amd.synthetic import permuted_heic
from conftest import make_emu

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "heif_amd" / "csrc"
EXE = CSRC / "build" / "emu_fast" / "emu_check"


@pytest.fixture(scope="module")
def emu_check():
    make_emu("emu-fast")
    return EXE


def _run(exe, path, env_extra=None):
    env = dict(os.environ)
    env.update(env_extra or {})
    r = subprocess.run([str(exe), str(path), "5"], capture_output=True, text=True, env=env, timeout=600)
    return r.returncode, r.stdout + r.stderr


# (k_intra: a single image runs luma / chroma wave pairs; "ppw1" forces the
# unsplit kernel.)
# k_parse_solo (one substream per wave), k_parse_solo<true> (spread: the
# automatic choice for a single image), k_parse_lanes (one substream per lane)
# with its adaptive geometry (one picture per wave for a single image), the
# full 64-lane packing of large batches (four 16-row pictures per wave) and
# batch (unsorted) wave order
LANES = {"HEIFGPU_PARSE": "lanes"}
PARSERS = {"solo": {"HEIFGPU_PARSE": "solo"}, "spread": {"HEIFGPU_PARSE": "spread"}, "lanes": LANES,
           "packed": {**LANES, "HEIFGPU_PARSE_ADAPT": "0"},
           "ppw1": {**LANES, "HEIFGPU_LANES_PPW": "1", "HEIFGPU_INTRA_SPLIT": "0"},
           # spread with k_intra_stream giving every picture up to its second launch, and without streaming
           "spread_redo": {"HEIFGPU_PARSE": "spread", "HEIFGPU_STREAM_PATIENCE_US": "0"},
           "spread_nostream": {"HEIFGPU_PARSE": "spread", "HEIFGPU_STREAM": "0"},
           "order0": {**LANES, "HEIFGPU_PARSE_ORDER": "0"}}


@pytest.mark.parametrize("parser", list(PARSERS))
def test_emulated_kernels_match_oracle(emu_check, parser):
    rc, out = _run(emu_check, ROOT / "tests/golden/halfmoonbay.heic", PARSERS[parser])
    assert rc == 0 and "EMU PARITY OK" in out, out[-2000:]


@pytest.mark.parametrize("parser", ["solo", "spread", "lanes", "packed"])
def test_emulated_kernels_permuted_image(emu_check, tmp_path, halfmoonbay, parser):
    p = tmp_path / "perm.heic"
    p.write_bytes(permuted_heic(halfmoonbay, 42))
    rc, out = _run(emu_check, p, PARSERS[parser])
    assert rc == 0 and "EMU PARITY OK" in out, out[-2000:]


def _corrupt(data: bytes, mode: str) -> bytes:
    import random

    from oracle import oracle

    d = bytearray(data)
    tiles, _ = oracle.list_tiles(data)
    if mode == "random":
        rng = random.Random(1)
        for k in (3, 20, 40):
            o, n = tiles[k]
            for _ in range(50):
                d[o + 40 + rng.randrange(n - 40)] = rng.randrange(256)
    else:  # zero the second half of tile 7's slice data
        o, n = tiles[7]
        d[o + n // 2:o + n] = bytes(n - n // 2)
    return bytes(d)


@pytest.mark.parametrize("parser", ["solo", "spread", "spread_redo", "lanes", "packed"])
@pytest.mark.parametrize("mode", ["random", "zeroed"])
def test_emulated_kernels_survive_corrupt_streams(emu_check, tmp_path, halfmoonbay, mode, parser):
    """Corrupt slice data must end in status bits, never in a crash (the same
    bounds protect the GPU: ring index masks, TU/coefficient caps, clamped
    geometry).  The ASan build (`make emu`) was run on the same inputs."""
    p = tmp_path / f"{mode}.heic"
    p.write_bytes(_corrupt(halfmoonbay, mode))
    rc, out = _run(emu_check, p, PARSERS[parser])
    assert rc in (0, 1), out[-2000:]
    line = next(l for l in out.splitlines() if l.startswith("parse: status"))
    assert int(line.split()[2].rstrip(","), 16) != 0


@pytest.mark.parametrize("split", [(2, 0), (2, 1), (3, 0), (3, 1), (3, 2), (8, 5)])
def test_emulated_tile_split_subsets(emu_check, split):
    """Row e2 (single-image tile split): rank g of G decodes only
    tiles k % G == g.  Its windows must equal the oracle's decode of the whole
    image and nothing else may be written, so the union over g — what
    heifgpu_gather_tiles assembles — is the single-rank decode bit for bit."""
    G, g = split
    r = subprocess.run([str(emu_check), str(ROOT / "tests/golden/halfmoonbay.heic"), "5", str(G), str(g)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "EMU PARITY OK" in r.stdout, (r.stdout + r.stderr)[-2000:]
    line = next(l for l in r.stdout.splitlines() if l.startswith("parse: status"))
    tbs = int(line.split()[3])
    assert 0 < tbs < 207654  # a strict subset of the image's TBs
