"""Pixel plausibility pin independent of the oracle's own arithmetic
(tests/plausibility.py): gain-map correlation with a permuted-tile negative
control, and CTB / tile edge-step ratios.  CPU: the oracle decode (which the
GPU matches bit for bit); GPU: the same metrics on the GPU's planes."""
import json

import numpy as np
import pytest

import plausibility
from conftest import GOLDEN

EXPECTED = json.loads((GOLDEN / "plausibility.json").read_text())["metrics"]


def _gain(oracle_mod, data):
    tiles, (ho, hl) = oracle_mod.list_tiles(data, 52)
    o, n = tiles[0]
    return oracle_mod.decode_tile(data[ho:ho + hl], data[o:o + n], 2016, 1512)[0]


def _compare(m):
    plausibility.check(m)
    for k, v in EXPECTED.items():
        assert m[k] == pytest.approx(v, abs=1e-6), k


def test_oracle_decode_is_plausible(oracle_mod, oracle_halfmoonbay, halfmoonbay):
    _compare(plausibility.metrics(oracle_halfmoonbay.y, _gain(oracle_mod, halfmoonbay)))


def test_control_detects_a_broken_decode(oracle_mod, oracle_halfmoonbay, halfmoonbay):
    """The metric discriminates: one tile replaced by a mid-grey block (a tile
    that failed to reconstruct) drops that tile's correlation to nothing."""
    y = oracle_halfmoonbay.y.copy()
    gain = _gain(oracle_mod, halfmoonbay)
    y[1024:1536, 1536:2048] = 128
    with pytest.raises(AssertionError):
        plausibility.check(plausibility.metrics(y, gain))


@pytest.mark.gpu
def test_gpu_decode_is_plausible(halfmoonbay):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import heif_amd as H

    y = H.HeicDecoder.decode(halfmoonbay).y.cpu().numpy()
    aux = H.HeifImage.parse(halfmoonbay).info.aux_item_id
    g = H.HeicDecoder.decode(halfmoonbay, item_id=aux).y.cpu().numpy()
    _compare(plausibility.metrics(np.asarray(y), np.asarray(g)))
