"""Known-answer vectors of the reference's own unit tests, run against both the
product's host code (libheifgpu C ABI hooks) and the CPU oracle.

Vectors: src/hevc/rbsp_reader.rs:143-303 (Tables 9-2/9-3, emulation
prevention incl. the real-SPS overlapping case) and
src/cabac/decoder.rs:300-373 (Table 9-39 TR cMax=5 cRice=0, Table 9-41
intra_chroma_pred_mode).  No GPU needed.
"""
import ctypes

import pytest

import heif_amd as H
from heif_amd import _lib

UE = [(0b10000000, 0), (0b01000000, 1), (0b01100000, 2), (0b00100000, 3), (0b00101000, 4),
      (0b00110000, 5), (0b00111000, 6), (0b00010000, 7), (0b00010010, 8), (0b00010100, 9)]
SE = [(0b10000000, 0), (0b01000000, 1), (0b01100000, -1), (0b00100000, 2), (0b00101000, -2),
      (0b00110000, 3), (0b00111000, -3)]
EP = [
    ([0x01, 0x02, 0x03, 0x04, 0x05], [0x01, 0x02, 0x03, 0x04, 0x05]),      # no pattern
    ([0x01, 0x00, 0x02], [0x01, 0x00, 0x02]),                              # single zero
    ([0x01, 0x00, 0x00, 0x04], [0x01, 0x00, 0x00, 0x04]),                  # double zero
    ([0x00, 0x00, 0x03, 0x00], [0x00, 0x00, 0x00]),                        # basic
    ([0x00, 0x00, 0x03, 0x01], [0x00, 0x00, 0x01]),
    ([0x00, 0x00, 0x03, 0x02], [0x00, 0x00, 0x02]),
    ([0x00, 0x00, 0x03, 0x03], [0x00, 0x00, 0x03]),
    ([0x00, 0x00, 0x03, 0x04], [0x00, 0x00, 0x03, 0x04]),                  # invalid follower kept
    ([0x01, 0x00, 0x00, 0x03], [0x01, 0x00, 0x00]),                        # at end
    ([0x00, 0x00, 0x03, 0x00, 0xFF, 0x00, 0x00, 0x03, 0x01], [0x00, 0x00, 0x00, 0xFF, 0x00, 0x00, 0x01]),
    ([0x42, 0x01, 0x01, 0x03, 0x70, 0x00, 0x00, 0x03, 0x00], [0x42, 0x01, 0x01, 0x03, 0x70, 0x00, 0x00, 0x00]),
    ([0x01, 0x03, 0x70, 0x00, 0x00, 0x03, 0x00, 0xB0, 0x00, 0x00, 0x03, 0x00, 0x00, 0x03, 0x00, 0x5A, 0xA0, 0x04],
     [0x01, 0x03, 0x70, 0x00, 0x00, 0x00, 0xB0, 0x00, 0x00, 0x00, 0x00, 0x00, 0x5A, 0xA0, 0x04]),  # real SPS
    ([0x00, 0x00, 0x03, 0x00, 0x00, 0x03, 0x01], [0x00, 0x00, 0x00, 0x00, 0x01]),  # consecutive
    ([], []),                                                               # empty
]
TR5 = [([0], 0), ([1, 0], 1), ([1, 1, 0], 2), ([1, 1, 1, 0], 3), ([1, 1, 1, 1, 0], 4), ([1, 1, 1, 1, 1], 5)]
CHROMA = [([0], 4), ([1, 0, 0], 0), ([1, 0, 1], 1), ([1, 1, 0], 2), ([1, 1, 1], 3)]


def _bins(seq):
    return (ctypes.c_uint8 * max(len(seq), 1))(*seq)


@pytest.mark.parametrize("byte,val", UE)
def test_ue_table_9_2(byte, val, oracle_mod):
    assert H.RbspReader.read_ue(bytes([byte])) == val
    v = ctypes.c_uint32()
    assert oracle_mod.lib.oracle_read_ue(_bins([byte]), 1, ctypes.byref(v)) == 0 and v.value == val


@pytest.mark.parametrize("byte,val", SE)
def test_se_table_9_3(byte, val, oracle_mod):
    assert H.RbspReader.read_se(bytes([byte])) == val
    v = ctypes.c_int32()
    assert oracle_mod.lib.oracle_read_se(_bins([byte]), 1, ctypes.byref(v)) == 0 and v.value == val


@pytest.mark.parametrize("src,want", EP)
def test_emulation_prevention(src, want, oracle_mod):
    assert H.RbspReader.remove_emulation_prevention(bytes(src)) == bytes(want)
    out = (ctypes.c_uint8 * max(len(src), 1))()
    n = oracle_mod.lib.oracle_remove_emulation_prevention(_bins(src), len(src), out)
    assert list(out[:n]) == want


def test_ue_rejects_truncated():
    with pytest.raises(H.HeifGpuError):
        H.RbspReader.read_ue(bytes([0x00]))  # 8 leading zeros, no terminator


@pytest.mark.parametrize("bins,val", TR5)
def test_truncated_rice_table_9_39(bins, val, oracle_mod):
    used = ctypes.c_int()
    assert _lib.lib.heifgpu_bins_truncated_rice(_bins(bins), len(bins), 5, 0, ctypes.byref(used)) == val
    assert used.value == len(bins)
    used2 = ctypes.c_int()
    assert oracle_mod.lib.oracle_decode_tr_bins(_bins(bins), len(bins), 5, 0, ctypes.byref(used2)) == val
    assert used2.value == len(bins)


@pytest.mark.parametrize("bins,val", CHROMA)
def test_intra_chroma_pred_mode_table_9_41(bins, val, oracle_mod):
    used = ctypes.c_int()
    assert _lib.lib.heifgpu_bins_chroma_pred_mode(_bins(bins), len(bins), ctypes.byref(used)) == val
    assert used.value == len(bins)
    used2 = ctypes.c_int()
    assert oracle_mod.lib.oracle_decode_chroma_mode_bins(_bins(bins), len(bins), ctypes.byref(used2)) == val


def _tr_ref(value, c_max, k):
    """Table 9-39 construction of TR(cMax, cRice) bins for `value`."""
    prefix = value >> k
    if prefix < (c_max >> k):
        bins = [1] * prefix + [0]
    else:
        bins = [1] * (c_max >> k)
    if c_max > value and k:
        bins += [(value >> (k - 1 - i)) & 1 for i in range(k)]
    return bins


def _eg_ref(value, k):
    """9.3.3.3 EGk bins."""
    bins = []
    while value >= (1 << k):
        bins.append(1)
        value -= 1 << k
        k += 1
    bins.append(0)
    bins += [(value >> (k - 1 - i)) & 1 for i in range(k)]
    return bins


@pytest.mark.parametrize("k", range(5))
def test_coeff_abs_level_remaining_roundtrip(k, oracle_mod):
    """9.3.3.11: prefix TR(4<<k, k) then EG(k+1) escape, for values across the switch."""
    for value in list(range(0, 80)) + [255, 1000, 32767]:
        c_max = 4 << k
        if value < c_max:
            bins = _tr_ref(value, c_max, k)
        else:
            bins = [1] * 4 + _eg_ref(value - c_max, k + 1)
        used = ctypes.c_int()
        got = _lib.lib.heifgpu_bins_coeff_abs_level_remaining(_bins(bins), len(bins), k, ctypes.byref(used))
        assert (got, used.value) == (value, len(bins)), (value, k)
        used2 = ctypes.c_int()
        got2 = oracle_mod.lib.oracle_decode_coeff_abs_level_remaining_bins(_bins(bins), len(bins), k,
                                                                          ctypes.byref(used2))
        assert (got2, used2.value) == (value, len(bins)), (value, k)


@pytest.mark.parametrize("k", [0, 1, 2])
def test_exp_golomb(k):
    for value in [0, 1, 2, 3, 7, 8, 100, 4095]:
        bins = _eg_ref(value, k)
        used = ctypes.c_int()
        assert _lib.lib.heifgpu_bins_exp_golomb(_bins(bins), len(bins), k, ctypes.byref(used)) == value
        assert used.value == len(bins)


def test_binarization_underrun_reports_error():
    used = ctypes.c_int()
    assert _lib.lib.heifgpu_bins_truncated_rice(_bins([1, 1]), 2, 5, 0, ctypes.byref(used)) == -1
