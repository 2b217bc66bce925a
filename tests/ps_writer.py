"""Hand-written SPS / PPS / slice-header writer for the robustness tests.

The synthetic encoder (heif_amd/csrc/synth) only writes legal parameter
sets; these tests need out-of-range ones (negative conformance offsets,
block-size ladders the kernels cannot take, SliceQpY outside [-QpBdOffset,
51], 12-bit streams), so this writes the same syntax (H.265 7.3.2.2 /
7.3.2.3 / 7.3.6.1, in the field order of hevc_synth.c's synth_sps /
synth_pps) with every value overridable.  Test infrastructure only.
"""
from __future__ import annotations


class BitWriter:
    def __init__(self):
        self.bits = []

    def u(self, v: int, n: int):
        for i in range(n - 1, -1, -1):
            self.bits.append((v >> i) & 1)

    def ue(self, v: int):
        v += 1
        n = v.bit_length()
        self.u(0, n - 1)
        self.u(v, n)

    def se(self, v: int):
        self.ue(2 * v - 1 if v > 0 else -2 * v)

    def trailing(self):
        self.bits.append(1)
        while len(self.bits) % 8:
            self.bits.append(0)

    def bytes(self) -> bytes:
        out = bytearray()
        for i in range(0, len(self.bits), 8):
            b = 0
            for x in self.bits[i:i + 8]:
                b = (b << 1) | x
            out.append(b)
        return bytes(out)


def _ep(rbsp: bytes) -> bytes:
    out, z = bytearray(), 0
    for x in rbsp:
        if z >= 2 and x <= 3:
            out.append(3)
            z = 0
        out.append(x)
        z = z + 1 if x == 0 else 0
    return bytes(out)


def _nal(t: int, w: BitWriter) -> bytes:
    return bytes([t << 1, 1]) + _ep(w.bytes())


def _ptl(w: BitWriter, profile: int):
    w.u(0, 2)
    w.u(0, 1)
    w.u(profile, 5)
    w.u(1 << (31 - profile), 32)
    w.u(1, 1)
    w.u(0, 1)
    w.u(0, 1)
    w.u(1, 1)
    w.u(0, 32)
    w.u(0, 11)
    w.u(0, 1)
    w.u(183, 8)


SPS_DEFAULTS = dict(chroma_format=1, width=128, height=96, conf=None, bit_depth=8, log2_min_cb_minus3=0,
                    log2_diff_max_min_cb=2, log2_min_tb_minus2=0, log2_diff_max_min_tb=3, depth_inter=0,
                    depth_intra=1, sao=1, pcm=None)


def sps(**over) -> bytes:
    """conf = (left, right, top, bottom) in chroma units as coded (ue)."""
    p = {**SPS_DEFAULTS, **over}
    w = BitWriter()
    w.u(0, 4)
    w.u(0, 3)
    w.u(1, 1)
    _ptl(w, 4 if p["chroma_format"] == 0 or p["bit_depth"] > 10 else (2 if p["bit_depth"] > 8 else 1))
    w.ue(0)
    w.ue(p["chroma_format"])
    w.ue(p["width"])
    w.ue(p["height"])
    if p["conf"] is not None:
        w.u(1, 1)
        for v in p["conf"]:
            w.ue(v)
    else:
        w.u(0, 1)
    w.ue(p["bit_depth"] - 8)
    w.ue(p["bit_depth"] - 8)
    w.ue(4)
    w.u(1, 1)
    w.ue(0)
    w.ue(0)
    w.ue(0)
    w.ue(p["log2_min_cb_minus3"])
    w.ue(p["log2_diff_max_min_cb"])
    w.ue(p["log2_min_tb_minus2"])
    w.ue(p["log2_diff_max_min_tb"])
    w.ue(p["depth_inter"])
    w.ue(p["depth_intra"])
    w.u(0, 1)  # scaling_list_enabled
    w.u(0, 1)  # amp
    w.u(p["sao"], 1)
    if p["pcm"] is None:
        w.u(0, 1)  # pcm_enabled_flag
    else:  # (bit depth luma, chroma, log2_min_pcm_cb_size_minus3, log2_diff_max_min_pcm_cb_size)
        w.u(1, 1)
        bdy, bdc, mn, df = p["pcm"]
        w.u(bdy - 1, 4)
        w.u(bdc - 1, 4)
        w.ue(mn)
        w.ue(df)
        w.u(0, 1)  # pcm_loop_filter_disabled_flag
    w.ue(0)    # num_short_term_ref_pic_sets
    w.u(0, 1)
    w.u(0, 1)
    w.u(1, 1)  # strong intra smoothing
    w.u(0, 1)  # vui
    w.u(0, 1)  # extensions
    w.trailing()
    return _nal(33, w)


PPS_DEFAULTS = dict(init_qp_minus26=0, cu_qp_delta=1, diff_cu_qp_delta_depth=1, cb_qp_offset=0, cr_qp_offset=0,
                    wpp=1, beta=0, tc=0)


def pps(**over) -> bytes:
    p = {**PPS_DEFAULTS, **over}
    w = BitWriter()
    w.ue(0)
    w.ue(0)
    w.u(0, 1)
    w.u(0, 1)
    w.u(0, 3)
    w.u(1, 1)  # sign hiding
    w.u(0, 1)
    w.ue(0)
    w.ue(0)
    w.se(p["init_qp_minus26"])
    w.u(0, 1)
    w.u(0, 1)  # transform skip
    w.u(p["cu_qp_delta"], 1)
    if p["cu_qp_delta"]:
        w.ue(p["diff_cu_qp_delta_depth"])
    w.se(p["cb_qp_offset"])
    w.se(p["cr_qp_offset"])
    w.u(0, 1)
    w.u(0, 1)
    w.u(0, 1)
    w.u(0, 1)  # transquant bypass
    t = p.get("tiles")  # dict(cols, rows, uniform=1, col_w=(), row_h=(), across=0) or None
    w.u(1 if t else 0, 1)  # tiles_enabled_flag
    w.u(p["wpp"], 1)
    if t:
        w.ue(t["cols"] - 1)
        w.ue(t["rows"] - 1)
        w.u(t.get("uniform", 1), 1)
        if not t.get("uniform", 1):
            for v in t["col_w"]:
                w.ue(v - 1)
            for v in t["row_h"]:
                w.ue(v - 1)
        w.u(t.get("across", 0), 1)
    w.u(0, 1)
    w.u(1, 1)  # deblocking control present
    w.u(0, 1)
    w.u(0, 1)
    w.se(p["beta"])
    w.se(p["tc"])
    w.u(0, 1)
    w.u(0, 1)
    w.ue(0)
    w.u(0, 1)
    w.u(0, 1)
    w.trailing()
    return _nal(34, w)
