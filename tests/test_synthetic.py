"""Synthetic config-4 batches: mt19937_64 Fisher-Yates
permutations of halfmoonbay's 48 grid tiles."""
import pytest

import heif_amd as H
from heif_amd.synthetic import MT19937_64, find_dimg, permutation, permuted_heic


def test_mt19937_64_known_answer():
    # C++11 [rand.predef]: the 10000th output of a default-constructed mt19937_64
    rng = MT19937_64(5489)
    for _ in range(9999):
        rng()
    assert rng() == 9981545732273789042


@pytest.mark.parametrize("seed", [0, 1, 7, 1023])
def test_permutation_is_a_permutation(seed):
    p = permutation(48, seed)
    assert sorted(p) == list(range(48))


def test_permutations_differ_by_seed():
    assert permutation(48, 0) != permutation(48, 1)


def test_permuted_file_reorders_only_dimg(halfmoonbay):
    off, w, cnt = find_dimg(halfmoonbay)
    assert (w, cnt) == (2, 48)
    f = permuted_heic(halfmoonbay, 3)
    assert len(f) == len(halfmoonbay)
    diff = [i for i in range(len(f)) if f[i] != halfmoonbay[i]]
    assert all(off <= i < off + w * cnt for i in diff)
    ids = [int.from_bytes(f[off + 2 * k: off + 2 * k + 2], "big") for k in range(cnt)]
    assert sorted(ids) == list(range(1, 49))


def test_permuted_image_parses_with_same_geometry(halfmoonbay):
    i = H.HeifImage.parse(permuted_heic(halfmoonbay, 5)).info
    assert (i.width, i.height, i.num_tiles, i.coded_bytes) == (4032, 3024, 48, 1_704_187)


def test_permuted_image_tiles_follow_permutation(halfmoonbay):
    perm = permutation(48, 11)
    a = H.HeifImage.parse(halfmoonbay)
    b = H.HeifImage.parse(permuted_heic(halfmoonbay, 11))
    for k in (0, 5, 47):
        assert b.tile_params(k)["payload_bytes"] == a.tile_params(perm[k])["payload_bytes"]
