// cabac.hpp — CABAC arithmetic decoding engine + binarizations for gfx950.
//
// Reference: src/cabac/arithmetic.rs (engine :13-174, tables :176-255) and
// src/cabac/decoder.rs (binarizations :152-284). MI355X design: one wave
// decodes one WPP substream; every lane runs the engine in lock-step (the
// values are wave-uniform), so the 64 lanes are free to refill a per-wave
// LDS byte ring in one coalesced 64-byte load with emulation-prevention
// bytes dropped by a wave ballot + popcount compaction, instead of one
// serial global load per byte. Context states live in LDS as
// (pStateIdx << 1) | valMps, one byte each. The value register is the
// usual 16-bit-scaled window (range << 7) so a renormalisation never needs
// more than one byte refill.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define HG_HD __host__ __device__
#else
#define HG_HD
#endif

namespace hg {

// Flat context index layout (I slices; Table 9-4 order)
enum CtxId : int {
    CTX_SAO_MERGE = 0,
    CTX_SAO_TYPE = 1,
    CTX_SPLIT_CU = 2,
    CTX_TQ_BYPASS = 5,
    CTX_PART_MODE = 6,
    CTX_PREV_INTRA = 7,
    CTX_CHROMA_MODE = 8,
    CTX_SPLIT_TF = 9,
    CTX_CBF_LUMA = 12,
    CTX_CBF_CHROMA = 14,
    CTX_CU_QP_DELTA = 19,
    CTX_TS_FLAG = 21,
    CTX_LAST_X = 23,
    CTX_LAST_Y = 41,
    CTX_CSBF = 59,
    CTX_SIG = 63,
    CTX_GT1 = 107,
    CTX_GT2 = 131,
    CTX_NUM = 137,
    CTX_PAD = 144
};

// initType-0 init values (syntax_element.rs:90-242, Table 9-5..9-31)
#define HG_CTX_INIT_VALUES                                                                                       \
    153, 200, 139, 141, 157, 154, 184, 184, 63, 153, 138, 138, 111, 141, 94, 138, 182, 154, 154, 154, 154, 139, \
        139, 110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63, 110, 110, \
        124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63, 91, 171, 134, 141, 111,  \
        111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107, 125, 141, 179, 153, 125, 107, \
        125, 141, 179, 153, 125, 140, 139, 182, 182, 152, 136, 152, 136, 153, 136, 139, 111, 136, 139, 111, 141, \
        111, 140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152, 140, 179, 166, 182,   \
        140, 227, 122, 197, 138, 153, 136, 167, 152, 152

// Table 9-46 rangeTabLps[pStateIdx][qRangeIdx], row-major
#define HG_LPS_TABLE                                                                                         \
    128, 176, 208, 240, 128, 167, 197, 227, 128, 158, 187, 216, 123, 150, 178, 205, 116, 142, 169, 195, 111,  \
        135, 160, 185, 105, 128, 152, 175, 100, 122, 144, 166, 95, 116, 137, 158, 90, 110, 130, 150, 85, 104,  \
        123, 142, 81, 99, 117, 135, 77, 94, 111, 128, 73, 89, 105, 122, 69, 85, 100, 116, 66, 80, 95, 110, 62,  \
        76, 90, 104, 59, 72, 86, 99, 56, 69, 81, 94, 53, 65, 77, 89, 51, 62, 73, 85, 48, 59, 69, 80, 46, 56, 66, \
        76, 43, 53, 63, 72, 41, 50, 59, 69, 39, 48, 56, 65, 37, 45, 54, 62, 35, 43, 51, 59, 33, 41, 48, 56, 32,  \
        39, 46, 53, 30, 37, 43, 50, 29, 35, 41, 48, 27, 33, 39, 45, 26, 31, 37, 43, 24, 30, 35, 41, 23, 28, 33,  \
        39, 22, 27, 32, 37, 21, 26, 30, 35, 20, 24, 29, 33, 19, 23, 27, 31, 18, 22, 26, 30, 17, 21, 25, 28, 16,  \
        20, 23, 27, 15, 19, 22, 25, 14, 18, 21, 24, 14, 17, 20, 23, 13, 16, 19, 22, 12, 15, 18, 21, 12, 14, 17,  \
        20, 11, 14, 16, 19, 11, 13, 15, 18, 10, 12, 15, 17, 10, 12, 14, 16, 9, 11, 13, 15, 9, 11, 12, 14, 8, 10, \
        12, 14, 8, 9, 11, 13, 7, 9, 11, 12, 7, 9, 10, 12, 7, 8, 10, 11, 6, 8, 9, 11, 6, 7, 9, 10, 6, 7, 8, 9, 2, \
        2, 2, 2

// Table 9-45 transIdxLps
#define HG_TRANS_LPS                                                                                             \
    0, 0, 1, 2, 2, 4, 4, 5, 6, 7, 8, 9, 9, 11, 11, 12, 13, 13, 15, 15, 16, 16, 18, 18, 19, 19, 21, 21, 22, 22, 23, \
        24, 24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30, 31, 32, 32, 33, 33, 33, 34, 34, 35, 35, 35, 36, 36, 36,  \
        37, 37, 37, 38, 38, 63

// 9.3.2.2 preCtxState → packed state
HG_HD inline uint8_t ctx_init_state(int init_value, int slice_qp) {
    int q = slice_qp < 0 ? 0 : (slice_qp > 51 ? 51 : slice_qp);
    int m = (init_value >> 4) * 5 - 45, n = ((init_value & 15) << 3) - 16;
    int pre = ((m * q) >> 4) + n;
    pre = pre < 1 ? 1 : (pre > 126 ? 126 : pre);
    int mps = pre > 63 ? 1 : 0;
    int st = mps ? pre - 64 : 63 - pre;
    return uint8_t((st << 1) | mps);
}

// ---------------- binarizations over an abstract bin source ----------------
// decoder.rs:152-164
template <class F>
HG_HD inline uint32_t bin_fixed_length(F &&bin, int nbits) {
    uint32_t v = 0;
    for (int i = 0; i < nbits; ++i) v = (v << 1) | uint32_t(bin());
    return v;
}
// decoder.rs:166-190 (TR, cMax, cRiceParam)
template <class F>
HG_HD inline uint32_t bin_truncated_rice(F &&bin, uint32_t cmax, int crice) {
    uint32_t pmax = cmax >> crice, p = 0;
    while (p < pmax && bin()) ++p;
    uint32_t suf = 0;
    if (crice > 0 && p < pmax) suf = bin_fixed_length(bin, crice);
    return (p << crice) + suf;
}
// decoder.rs:206-222, accumulated in 32 bits (App. B item 9). Returns
// 0xffffffff when the prefix exceeds 31 ones (corrupt stream).
template <class F>
HG_HD inline uint32_t bin_exp_golomb(F &&bin, int k) {
    int ones = 0;
    while (bin()) {
        if (++ones > 31 - k) return 0xffffffffu;
    }
    return (((1u << ones) - 1u) << k) + bin_fixed_length(bin, ones + k);
}
// decoder.rs:230-261: prefix TR(cMax = 4 << k, k), escape EG(k+1)
template <class F>
HG_HD inline uint32_t bin_coeff_abs_level_remaining(F &&bin, int k) {
    uint32_t cmax = 4u << k;
    uint32_t pre = bin_truncated_rice(bin, cmax, k);
    if (pre == cmax) {
        uint32_t s = bin_exp_golomb(bin, k + 1);
        return s == 0xffffffffu ? s : cmax + s;
    }
    return pre;
}
// decoder.rs:192-204 (Table 9-41): bin0 context, then FL(2) bypass; "0" → 4
template <class F0, class F1>
HG_HD inline uint32_t bin_intra_chroma_pred_mode(F0 &&ctx_bin, F1 &&bypass_bin) {
    if (!ctx_bin()) return 4;
    return bin_fixed_length(bypass_bin, 2);
}

}  // namespace hg
