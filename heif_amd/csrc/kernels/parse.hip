// parse.hip — CABAC slice-data parser for gfx950 (pipeline stage 1).
//
// Replaces SliceSegmentReader::read_data / read_coding_tree_unit and the
// todo!() sao() / coding_quadtree() of src/hevc/slice.rs:206-256, with the
// engine of src/cabac/arithmetic.rs and the binarizations of
// src/cabac/decoder.rs, plus everything H.265 needs below them (7.3.8.3-14,
// 9.3.4.2 ctxInc, 8.4.2 MPM, 8.6.1 QP).
//
// Mapping to MI355X: one workgroup per picture (HEIF grid tile), one wave per
// WPP substream (= CTB row).  Row r may parse CTU c once row r-1 has finished
// CTU c+1 (the WPP 2-CTU lag, which also covers the above-CTB split depth and
// SAO merge-up data); the lag is enforced with per-wave progress counters in
// LDS (workgroup-scope release/acquire, so no cross-CU protocol is needed).
// All 64 lanes run the scalar syntax decode in lock-step; lanes fan out for
// the byte-ring refill (coalesced 64-byte loads, EP bytes removed by ballot),
// and for the map writes (QP, edges, modes, depths).
#include "cabac.hpp"
#include "kernels.hpp"
#include "tables.hpp"

#if !defined(HG_HOST_EMU)
// v_writelane_b32 (this clang exposes no builtin for it): lane `lane` of `old` := src
extern "C" __device__ int hg_writelane(int src, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
#endif

namespace hg {

__constant__ uint8_t c_lps[256] = {HG_LPS_TABLE};
__constant__ uint8_t c_trans_lps[64] = {HG_TRANS_LPS};
__constant__ uint8_t c_ctx_init[CTX_NUM] = {HG_CTX_INIT_VALUES};
#if defined(HG_PARSE_PROF) && !defined(HG_HOST_EMU)
__device__ uint64_t g_prof[16];
#endif

namespace {

#define HG_INLINE __device__ __attribute__((always_inline)) inline
// lane-parallel loop with a wave-uniform trip count; only the body is predicated
#define HG_LANE_LOOP(k, lane_, n)                                       \
    for (int k##_0 = 0, k = (lane_); k##_0 < (n); k##_0 += kWave, k = k##_0 + (lane_)) \
        if (k < (n))

__device__ __forceinline__ uint32_t uni(uint32_t v) { return HG_UNI(v); }

__device__ __forceinline__ int unis(int v) { return (int)HG_UNI((uint32_t)v); }

// Optional cycle/bin counters (build with -DHG_PARSE_PROF; read back with
// heifgpu_debug_counters).  Compiled out of the product library.
#if defined(HG_PARSE_PROF) && !defined(HG_HOST_EMU)
#define HG_PROF(x) x
__device__ __forceinline__ uint64_t prof_clock() { return __builtin_amdgcn_s_memtime(); }
#else
#define HG_PROF(x)
#endif
enum { PF_WAVE, PF_SPIN, PF_BINS, PF_BYPASS, PF_REFILL, PF_CQT, PF_RESID, PF_SAO, PF_N };

#if defined(__HIP_DEVICE_COMPILE__)
#define HG_GLOBAL __attribute__((address_space(1)))  // keeps LDS-held pointers global (not flat)
#else
#define HG_GLOBAL
#endif
struct PicConst {
    int W, H, wctb, hctb, minCb, minTb, maxTb, maxDepthIntra, chroma, bdY, bdC, qpbdY, qpbdC;
    int pcmMin, pcmMax, log2qg, cbOff, crOff, sliceQp, saoL, saoC, w4, h4;
    uint32_t tu_cap, coef_cap;
    HG_GLOBAL int8_t *gqpy;
    HG_GLOBAL uint8_t *gflags;
    HG_GLOBAL TuRec *tu_out;
    HG_GLOBAL Coef *coef_out;
};

struct alignas(16) WaveLds {
    PicConst pc;
    uint8_t ring[256 + 16];  // + trash byte for dropped lanes (ring_refill)
    uint8_t ipm[16][17];  // IntraPredModeY per 4x4 of the current CTB, column 0 = left CTB
    uint8_t depth[8][9];  // CtDepth per 8x8, column 0 = left CTB
    int8_t qpy[8][8];     // QpY per 8x8 of the current CTB
    uint32_t cqt[24];     // coding_quadtree stack
    uint64_t tt[24];      // transform_tree stack
    SaoParams sao_left;
    uint8_t pad_[2];
};


// ---------------------------------------------------------------- context registers
// The 137 context variables live in ONE VGPR of the wave: context i is byte
// (i >> 6) of lane (i & 63).  A bin reads its context with v_readlane (SGPR
// lane select) and writes it back with v_writelane, so the serial bin chain
// never waits on LDS.  rangeTabLps (Table 9-52) rides in a second VGPR (lane
// = pStateIdx, 4 bytes = qRangeIdx) and transIdxLps (Table 9-53) in a third.
// In the host emulation (kWave = 1) the same interface is plain arrays.
#if defined(HG_HOST_EMU)
struct CtxRegs {
    uint8_t b[256];
    uint8_t lps[64][4];
    uint8_t trans[64];
    void load_tables(int) {
        for (int st = 0; st < 64; ++st) {
            for (int q = 0; q < 4; ++q) lps[st][q] = c_lps[(st << 2) | q];
            trans[st] = c_trans_lps[st];
        }
    }
    uint32_t word(int ci) const { return b[ci]; }
    static uint32_t state(uint32_t w, int) { return w; }
    void put(int ci, uint32_t, uint32_t s) { b[ci] = (uint8_t)s; }
    uint32_t lps_of(uint32_t st, uint32_t q) const { return lps[st][q]; }
    uint32_t trans_of(uint32_t st) const { return trans[st]; }
    void init(int, int qp) {
        for (int i = 0; i < 256; ++i) b[i] = i < CTX_NUM ? ctx_init_state(c_ctx_init[i], qp) : 0;
    }
    void save(uint32_t *slot, int) const { std::memcpy(slot, b, 256); }
    void restore(const uint32_t *slot, int) { std::memcpy(b, slot, 256); }
};
#else
struct CtxRegs {
    uint32_t v;      // contexts
    uint32_t lpsv;   // rangeTabLps row of state = lane
    uint32_t transv; // transIdxLps of state = lane
    __device__ void load_tables(int lane) {
        lpsv = (uint32_t)c_lps[lane << 2] | ((uint32_t)c_lps[(lane << 2) | 1] << 8) |
               ((uint32_t)c_lps[(lane << 2) | 2] << 16) | ((uint32_t)c_lps[(lane << 2) | 3] << 24);
        transv = c_trans_lps[lane];
    }
    __device__ uint32_t word(int ci) const { return (uint32_t)__builtin_amdgcn_readlane((int)v, ci & 63); }
    static __device__ uint32_t state(uint32_t w, int ci) { return (w >> ((ci >> 6) << 3)) & 0xffu; }
    __device__ void put(int ci, uint32_t w, uint32_t s) {
        const int sh = (ci >> 6) << 3;
        w = (w & ~(0xffu << sh)) | (s << sh);
        v = (uint32_t)hg_writelane((int)w, ci & 63, (int)v);
    }
    __device__ uint32_t lps_of(uint32_t st, uint32_t q) const {
        return ((uint32_t)__builtin_amdgcn_readlane((int)lpsv, (int)st) >> (q << 3)) & 0xffu;
    }
    __device__ uint32_t trans_of(uint32_t st) const {
        return (uint32_t)__builtin_amdgcn_readlane((int)transv, (int)st);
    }
    __device__ void init(int lane, int qp) {
        uint32_t w = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int i = lane + 64 * k;
            if (i < CTX_NUM) w |= (uint32_t)ctx_init_state(c_ctx_init[i], qp) << (8 * k);
        }
        v = w;
    }
    __device__ void save(uint32_t *slot, int lane) const { slot[lane] = v; }
    __device__ void restore(const uint32_t *slot, int lane) { v = slot[lane]; }
};
#endif

struct Parser {
    // Cold per-picture constants and output pointers live in the wave's LDS
    // block (WaveLds::pc, read through PCV/PCP at their few use sites): the
    // register file is kept for the CABAC engine and the per-CU state, so the
    // bin loops do not spill SGPRs into VGPR lanes.
    int log2ctb, ctb;
    uint32_t flags;
    // engine (9.3.4.3) with a 16-bit-scaled value register
    uint32_t range, value;
    int bits_needed;
    // byte ring
    uint32_t rd, wr, src_pos, nal_end, prev1, prev2;
    const uint8_t *src;
    const uint8_t *depth_above;  // LDS line of the CTB row above (8x8 units)
#if !defined(HG_HOST_EMU)
    uint32_t cstage, cstage_n;  // coefficient staging (coef_put)
    uint32_t tstage[4], tstage_n;  // TU record staging (tu_put)
    uint32_t ringv;  // the ring, 4 bytes per lane
    uint32_t scanv;  // 8x8 diagonal scan: byte 0 = x | (y << 3) of sPos = lane, byte 1 = sPos of raster lane
#endif
    uint32_t status;
    WaveLds *w;
    CtxRegs cx;
    int lane;
    HG_PROF(uint64_t prof[PF_N];)
    // CTB
    int ctbx, ctby, rx, ry;
    // quantization groups (8.6.1)
    int qp_prev_last, qp_pred, cu_qp_delta_val, qpy_cur, qg_x, qg_y;
    bool is_cu_qp_delta_coded, qg_new, first_qg_in_slice;
    // coding unit
    bool cu_bypass;
    int cu_intra_split, cu_chroma_mode;
    // outputs
    uint32_t ntu, ncoef;
};
#define PCV(f) unis(p.w->pc.f)
#define PCP(f) (p.w->pc.f)

// ---------------------------------------------------------------- bytes
// The RBSP bytes of the substream flow through a 256-byte ring per wave.
// ring_refill converts the next 64 raw bytes (one per lane, emulation-
// prevention bytes dropped via ballot compaction) and appends them.  Refills
// happen only at a few syntax points (ensure_bytes): CTU start/end, every
// coding-quadtree and transform-tree node and every residual sub-block, each
// of which consumes at most ~175 bytes of a conforming stream (a 4x4
// sub-block: 42 context bins of <= 6 bits + 16 coeff_abs_level_remaining of
// <= 72 bypass bins).  next_byte is therefore branch-free.  On the GPU the
// ring also lives in a VGPR (byte rd of lane (rd >> 2) & 63), so the byte
// fetch of the bin loop is a v_readlane rather than an LDS round trip.
constexpr uint32_t kRingLowWater = 192;  // ring - 64: a refill never overwrites unread bytes
#if defined(HG_HOST_EMU)
HG_INLINE void ring_refill(Parser &p) {  // scalar equivalent of the 64-lane ballot refill
    for (int lane = 0; lane < 64; ++lane) {
        uint32_t pos = p.src_pos + lane;
        if (pos >= p.nal_end) break;
        uint32_t b = p.src[pos];
        uint32_t nb = pos + 1 < p.nal_end ? p.src[pos + 1] : 0xffu;
        bool ep = p.prev2 == 0 && p.prev1 == 0 && b == 3 && (pos + 1 >= p.nal_end || nb <= 3);
        if (!ep) p.w->ring[p.wr++ & 255] = (uint8_t)b;
        p.prev2 = p.prev1;
        p.prev1 = b;
    }
    p.src_pos += 64;
}
HG_INLINE uint32_t next_byte(Parser &p) { return p.w->ring[p.rd++ & 255]; }
#else
HG_INLINE void ring_refill(Parser &p) {
    const int lane = p.lane;
    uint32_t pos = p.src_pos + lane;
    bool valid = pos < p.nal_end;
    uint32_t b = valid ? p.src[pos] : 0xffu;
    uint32_t b64 = (p.src_pos + 64 < p.nal_end) ? p.src[p.src_pos + 64] : 0xffu;
    uint32_t nb = __shfl(b, (lane + 1) & 63, 64);
    if (lane == 63) nb = b64;
    uint32_t bm1 = __shfl(b, (lane + 63) & 63, 64);
    uint32_t bm2 = __shfl(b, (lane + 62) & 63, 64);
    bm1 = lane == 0 ? p.prev1 : bm1;
    bm2 = lane == 0 ? p.prev2 : (lane == 1 ? p.prev1 : bm2);
    // rbsp_reader.rs:11-39: 00 00 03 followed by a byte <= 3 (or the end)
    bool ep = valid && bm2 == 0 && bm1 == 0 && b == 3 && (pos + 1 >= p.nal_end || nb <= 3);
    bool keep = valid && !ep;
    uint64_t m = __ballot(keep);
    uint32_t idx = __popcll(m & ((1ull << lane) - 1ull));
    // no divergent branch around the store (it would make the compiler treat the
    // ring state, and so the whole engine, as divergent): dropped bytes go to ring[256]
    p.w->ring[keep ? (p.wr + idx) & 255 : 256] = (uint8_t)b;
    p.wr += __popcll(m);
    p.prev2 = uni(__shfl(b, 62, 64));
    p.prev1 = uni(__shfl(b, 63, 64));
    p.src_pos += 64;
    p.ringv = reinterpret_cast<const uint32_t *>(p.w->ring)[lane];  // same wave: LDS is in order
}
HG_INLINE uint32_t next_byte(Parser &p) {
    const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)p.ringv, (int)((p.rd >> 2) & 63));
    const uint32_t v = (d >> ((p.rd & 3) << 3)) & 0xffu;
    ++p.rd;
    return v;
}
#endif


// top up the ring to the low-water mark (or the end of the NAL unit)
HG_INLINE void ensure_bytes(Parser &p) {
    while (p.wr - p.rd < kRingLowWater && p.src_pos < p.nal_end) {
        ring_refill(p);
        HG_PROF(++p.prof[PF_REFILL]);
    }
}

// a conforming substream never reads past the bytes it was given
HG_INLINE void check_overrun(Parser &p) {
    if ((int32_t)(p.wr - p.rd) < 0) p.status |= ST_OVERRUN;
}

// 9.3.2.5 initialization of the arithmetic decoding engine at a raw offset
HG_INLINE void engine_init(Parser &p, uint32_t raw_start) {
    p.src_pos = raw_start;
    p.rd = p.wr = 0;
    p.prev1 = raw_start >= 1 ? p.src[raw_start - 1] : 0xffu;
    p.prev2 = raw_start >= 2 ? p.src[raw_start - 2] : 0xffu;
    p.prev1 = uni(p.prev1);
    p.prev2 = uni(p.prev2);
    p.range = 510;
    ensure_bytes(p);
    uint32_t b0 = next_byte(p);
    uint32_t b1 = next_byte(p);
    p.value = (b0 << 8) | b1;
    p.bits_needed = -8;
    if ((p.value >> 7) >= 510) p.status |= ST_CABAC_INIT;
}

// 9.3.2.2 context initialization
HG_INLINE void ctx_init(Parser &p) {
    p.cx.init(p.lane, PCV(sliceQp));
}

// ---------------------------------------------------------------- engine
// 9.3.4.3.2 DecodeDecision (arithmetic.rs:97-144)
HG_INLINE int dec_bin(Parser &p, int ci) {
    HG_PROF(++p.prof[PF_BINS]);
    // Branchy on purpose: at 6 waves/SIMD k_parse is issue-bound, and the MPS
    // path (the common one) is the shortest instruction sequence.  (Measured:
    // a branch-free select version, and a bit counter tested with `& 8`, both
    // cost +30 % on the bench.)
    const uint32_t w = p.cx.word(ci);
    const uint32_t s = CtxRegs::state(w, ci);
    uint32_t st = s >> 1, mps = s & 1;
    const uint32_t lps = p.cx.lps_of(st, (p.range >> 6) & 3);
    p.range -= lps;
    const uint32_t scaled = p.range << 7;
    int bin;
    if (p.value < scaled) {
        bin = (int)mps;
        st = st < 62 ? st + 1 : st;
        if (scaled < (256u << 7)) {
            p.range = scaled >> 6;
            p.value <<= 1;
            if (++p.bits_needed == 0) {
                p.bits_needed = -8;
                p.value |= next_byte(p);
            }
        }
    } else {
        p.value -= scaled;
        const uint32_t nbits = (uint32_t)__builtin_clz(lps) - 23u;
        p.value <<= nbits;
        p.range = lps << nbits;
        bin = (int)(mps ^ 1u);
        if (st == 0) mps ^= 1u;
        st = p.cx.trans_of(st);
        p.bits_needed += (int)nbits;
        if (p.bits_needed >= 0) {
            p.value |= next_byte(p) << p.bits_needed;
            p.bits_needed -= 8;
        }
    }
    p.cx.put(ci, w, (st << 1) | mps);
    return bin;
}

// 9.3.4.3.4 DecodeBypass (arithmetic.rs:146-157)
__device__ __forceinline__ int dec_bypass(Parser &p) {
    HG_PROF(++p.prof[PF_BYPASS]);
    p.value <<= 1;
    if (++p.bits_needed >= 0) {
        p.bits_needed = -8;
        p.value |= next_byte(p);
    }
    const uint32_t scaled = p.range << 7;
    if (p.value >= scaled) {
        p.value -= scaled;
        return 1;
    }
    return 0;
}

HG_INLINE uint32_t dec_bypass_bits(Parser &p, int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; ++i) v = (v << 1) | (uint32_t)dec_bypass(p);
    return v;
}

// 9.3.4.3.5 DecodeTerminate (arithmetic.rs:159-169)
HG_INLINE int dec_term(Parser &p) {
    p.range -= 2;
    uint32_t scaled = p.range << 7;
    if (p.value >= scaled) return 1;
    if (scaled < (256u << 7)) {
        p.range = scaled >> 6;
        p.value <<= 1;
        if (++p.bits_needed == 0) {
            p.bits_needed = -8;
            p.value |= next_byte(p);
        }
    }
    return 0;
}

// ---------------------------------------------------------------- helpers
__device__ __forceinline__ int chroma_qp_map(int qpi, int chroma) {
    if (chroma != 1) return qpi < 51 ? qpi : 51;
    if (qpi < 30) return qpi;
    if (qpi > 43) return qpi - 6;
    constexpr int t[14] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37};
    return t[qpi - 30];
}

__device__ __forceinline__ void update_qpy(Parser &p) {
    p.qpy_cur = ((p.qp_pred + p.cu_qp_delta_val + 52 + 2 * PCV(qpbdY)) % (52 + PCV(qpbdY))) - PCV(qpbdY);
}

// 8.6.1: qPY_PRED of the current quantization group
HG_INLINE void derive_qp_pred(Parser &p) {
    int prev;
    bool first_in_ctb = p.qg_x == p.ctbx && p.qg_y == p.ctby;
    if (p.first_qg_in_slice) {
        prev = PCV(sliceQp);
        p.first_qg_in_slice = false;
    } else if ((p.flags & SP_WPP) && first_in_ctb && p.rx == 0) {
        prev = PCV(sliceQp);
    } else {
        prev = p.qp_prev_last;
    }
    int mask = p.ctb - 1;
    int qa = (p.qg_x & mask) ? unis(p.w->qpy[(p.qg_y - p.ctby) >> 3][((p.qg_x - p.ctbx) >> 3) - 1]) : prev;
    int qb = (p.qg_y & mask) ? unis(p.w->qpy[((p.qg_y - p.ctby) >> 3) - 1][(p.qg_x - p.ctbx) >> 3]) : prev;
    p.qp_pred = (qa + qb + 1) >> 1;
}

// ---------------------------------------------------------------- SAO syntax (7.3.8.3)
HG_INLINE void parse_sao(Parser &p, SaoParams *sao_line_above, SaoParams *gsao) {
    ensure_bytes(p);
    SaoParams s;
    for (int c = 0; c < 3; ++c) {
        s.type[c] = 0;
        s.band_eo[c] = 0;
        for (int i = 0; i < 4; ++i) s.off[c][i] = 0;
    }
    int ml = 0, mu = 0;
    if (p.rx > 0) ml = dec_bin(p, CTX_SAO_MERGE);
    if (p.ry > 0 && !ml) mu = dec_bin(p, CTX_SAO_MERGE);
    if (ml) {
        s = p.w->sao_left;
    } else if (mu) {
        s = sao_line_above[p.rx];
    } else {
        // component loop fully unrolled: a runtime index into the private
        // SaoParams would keep it in scratch (and scratch loads are divergent)
        const int ncomp = PCV(chroma) ? 3 : 1;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            if (c >= ncomp) break;
            if (!((PCV(saoL) && c == 0) || (PCV(saoC) && c > 0))) continue;
            if (c < 2) {
                int t = 0;
                if (dec_bin(p, CTX_SAO_TYPE)) t = dec_bypass(p) ? 2 : 1;
                s.type[c] = (int8_t)t;
            } else {
                s.type[2] = s.type[1];
            }
            if (!s.type[c]) continue;
            int bd = c ? PCV(bdC) : PCV(bdY);
            uint32_t cmax = (1u << ((bd < 10 ? bd : 10) - 5)) - 1;
            int a[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = (int)bin_truncated_rice([&]() { return dec_bypass(p); }, cmax, 0);
            if (s.type[c] == 1) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (a[i] && dec_bypass(p)) a[i] = -a[i];
                s.band_eo[c] = (uint8_t)dec_bypass_bits(p, 5);
#pragma unroll
                for (int i = 0; i < 4; ++i) s.off[c][i] = (int16_t)a[i];
            } else {
                if (c < 2) s.band_eo[c] = (uint8_t)dec_bypass_bits(p, 2);
                else s.band_eo[2] = s.band_eo[1];
                s.off[c][0] = (int16_t)a[0];
                s.off[c][1] = (int16_t)a[1];
                s.off[c][2] = (int16_t)-a[2];
                s.off[c][3] = (int16_t)-a[3];
            }
        }
    }
    p.w->sao_left = s;  // every lane stores the same value: no divergent branch
    gsao[p.ry * PCV(wctb) + p.rx] = s;
}

// ---------------------------------------------------------------- scans (6.5.3-6.5.5)
// Per-coefficient lookups must not touch memory: 2x2 and 4x4 scans are packed
// 64-bit immediates, the 8x8 diagonal scan (32x32 TBs' sub-block order) sits
// in a VGPR read with v_readlane.  Results use kScanPos's x | (y << 4) form.
HG_INLINE int scan_pos(const Parser &p, int l, int scan, int i) {
#if defined(HG_HOST_EMU)
    return kScanPos[l][scan][i];
#else
    if (l == 3) {
        const uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)p.scanv, i) & 0xffu;
        return (int)((e & 7) | ((e >> 3) << 4));
    }
    if (l == 0) return 0;
    const uint64_t t = l == 2 ? (scan == 0 ? kScan4Pos[0] : scan == 1 ? kScan4Pos[1] : kScan4Pos[2])
                              : (scan == 0 ? kScan2Pos[0] : scan == 1 ? kScan2Pos[1] : kScan2Pos[2]);
    const uint32_t e = (uint32_t)(t >> (4 * i)) & 15u;
    return (int)((e & 3) | ((e >> 2) << 4));
#endif
}

HG_INLINE int scan_inv(const Parser &p, int l, int scan, int raster) {
#if defined(HG_HOST_EMU)
    return kScanInv[l][scan][raster];
#else
    if (l == 3) return (int)(((uint32_t)__builtin_amdgcn_readlane((int)p.scanv, raster) >> 8) & 0xffu);
    if (l == 0) return 0;
    const uint64_t t = l == 2 ? (scan == 0 ? kScan4Inv[0] : scan == 1 ? kScan4Inv[1] : kScan4Inv[2])
                              : (scan == 0 ? kScan2Inv[0] : scan == 1 ? kScan2Inv[1] : kScan2Inv[2]);
    return (int)((uint32_t)(t >> (4 * raster)) & 15u);
#endif
}

// sig_coeff_flag ctxInc patterns (9.3.4.2.5) per prevCsbf, byte per raster
// position e = x | (y << 2); and Table 9-50's ctxIdxMap for 4x4 TBs
constexpr uint64_t sig_pat_word(int pc, int half) {
    uint64_t w = 0;
    for (int k = 0; k < 8; ++k) {
        const int e = half * 8 + k, x = e & 3, y = e >> 2;
        const int v = pc == 0 ? (x + y == 0 ? 2 : (x + y < 3 ? 1 : 0))
                    : pc == 1 ? (y == 0 ? 2 : (y == 1 ? 1 : 0))
                    : pc == 2 ? (x == 0 ? 2 : (x == 1 ? 1 : 0)) : 2;
        w |= (uint64_t)v << (8 * k);
    }
    return w;
}
constexpr uint64_t sig_map4_word(int half) {
    uint64_t w = 0;
    for (int k = 0; k < 8; ++k) w |= ((kSigCtxMap4 >> (4 * (half * 8 + k))) & 15u) << (8 * k);
    return w;
}
constexpr uint64_t kSigPat[4][2] = {{sig_pat_word(0, 0), sig_pat_word(0, 1)}, {sig_pat_word(1, 0), sig_pat_word(1, 1)},
                                    {sig_pat_word(2, 0), sig_pat_word(2, 1)}, {sig_pat_word(3, 0), sig_pat_word(3, 1)}};
constexpr uint64_t kSigMap4Lo = sig_map4_word(0), kSigMap4Hi = sig_map4_word(1);

HG_INLINE uint64_t scan4_word(int scan) {
    return scan == 0 ? kScan4Pos[0] : (scan == 1 ? kScan4Pos[1] : kScan4Pos[2]);
}

// Coefficients leave k_parse 64 at a time: coefficient k of the pending group
// sits in lane k of a staging VGPR and one coalesced store writes the group.
// (A per-coefficient global store would make the next overwrite of its data
// VGPR wait for the store to complete: an s_waitcnt vmcnt(0) per coefficient.)
HG_INLINE void coef_flush(Parser &p) {
#if !defined(HG_HOST_EMU)
    if (p.cstage_n) {
        const uint32_t n = p.cstage_n;
        const uint32_t cap = PCV(coef_cap) - 1;  // the row's last slot is the trash slot
        if (p.ncoef + n <= cap) {
            // every lane stores (no divergent branch): lanes past n hit the trash slot
            const uint32_t idx = (uint32_t)p.lane < n ? p.ncoef + p.lane : cap;
            PCP(coef_out)[idx] = p.cstage;
            p.ncoef += n;
        } else {
            p.status |= ST_CAPACITY;
        }
        p.cstage_n = 0;
    }
#endif
}

HG_INLINE void coef_put(Parser &p, uint32_t packed) {
#if defined(HG_HOST_EMU)
    if (p.ncoef < PCV(coef_cap)) PCP(coef_out)[p.ncoef++] = packed;
    else p.status |= ST_CAPACITY;
#else
    p.cstage = (uint32_t)hg_writelane((int)packed, (int)p.cstage_n, (int)p.cstage);
    if (++p.cstage_n == 64) coef_flush(p);
#endif
}

// ---------------------------------------------------------------- residual_coding (7.3.8.11)
HG_INLINE void residual_coding(Parser &p, int log2n, int cidx, int mode, bool &ts, uint32_t &coef_first,
                                uint32_t &ncoef) {
    const int n = 1 << log2n;
    ts = false;
    if ((p.flags & SP_TRANSFORM_SKIP) && !p.cu_bypass && log2n == 2) ts = dec_bin(p, CTX_TS_FLAG + (cidx ? 1 : 0));
    // last_sig_coeff_{x,y}_prefix (decoder.rs:109-130), suffixes (bypass)
    int cmax = (log2n << 1) - 1;
    int off, shift;
    if (cidx == 0) {
        off = 3 * (log2n - 2) + ((log2n - 1) >> 2);
        shift = (log2n + 1) >> 2;
    } else {
        off = 15;
        shift = log2n - 2;
    }
    int px = 0, py = 0;
    while (px < cmax && dec_bin(p, CTX_LAST_X + off + (px >> shift))) ++px;
    while (py < cmax && dec_bin(p, CTX_LAST_Y + off + (py >> shift))) ++py;
    int lx = px, ly = py;
    if (px > 3) {
        int k = (px >> 1) - 1;
        lx = (1 << k) * (2 + (px & 1)) + (int)dec_bypass_bits(p, k);
    }
    if (py > 3) {
        int k = (py >> 1) - 1;
        ly = (1 << k) * (2 + (py & 1)) + (int)dec_bypass_bits(p, k);
    }
    // 7.4.9.11 scanIdx
    int scan = 0;
    if (log2n == 2 || (log2n == 3 && cidx == 0)) {
        if (mode >= 6 && mode <= 14) scan = 2;
        else if (mode >= 22 && mode <= 30) scan = 1;
    }
    if (scan == 2) {
        int t = lx;
        lx = ly;
        ly = t;
    }
    if (lx >= n || ly >= n) {
        p.status |= ST_SYNTAX;
        lx &= n - 1;
        ly &= n - 1;
    }
    const int sbl = log2n - 2, sbw = 1 << sbl;
    const int last_sub = scan_inv(p, sbl, scan, (ly >> 2) * sbw + (lx >> 2));
    const int last_pos = scan_inv(p, 2, scan, (ly & 3) * 4 + (lx & 3));
    uint64_t csbf = 0;  // coded_sub_block_flag bitmap, bit yS*8+xS
    int prev_c1 = 1;    // greater1Ctx state carried from the previous coded sub-block
    bool any_sb = false;
    coef_first = p.ncoef;
    ncoef = 0;
    for (int i = last_sub; i >= 0; --i) {
        ensure_bytes(p);
        const int sp = scan_pos(p, sbl, scan, i);
        const int xS = sp & 15, yS = sp >> 4;
        bool coded;
        bool infer_dc = false;
        int prev_csbf = 0;
        if (xS < sbw - 1) prev_csbf |= (int)((csbf >> (yS * 8 + xS + 1)) & 1);
        if (yS < sbw - 1) prev_csbf |= (int)((csbf >> ((yS + 1) * 8 + xS)) & 1) << 1;
        if (i < last_sub && i > 0) {
            int ctx = ((prev_csbf & 1) | (prev_csbf >> 1)) + (cidx ? 2 : 0);
            coded = dec_bin(p, CTX_CSBF + ctx);
            infer_dc = true;
        } else {
            coded = true;
        }
        if (coded) csbf |= 1ull << (yS * 8 + xS);
        uint32_t sig = 0;
        if (coded) {
            int nstart = 15;
            if (i == last_sub) {
                sig = 1u << last_pos;
                nstart = last_pos - 1;
            }
            // ctxInc of sig_coeff_flag (9.3.4.2.5) for every raster position e = xP | (yP << 2)
            // of this sub-block, one byte each in two words: the bin loop does one shift
            uint64_t t0, t1;
            if (log2n == 2) {
                t0 = kSigMap4Lo;
                t1 = kSigMap4Hi;
            } else {
                const int off = cidx == 0 ? ((xS | yS) ? 3 : 0) + (log2n == 3 ? (scan == 0 ? 9 : 15) : 21)
                                          : (log2n == 3 ? 9 : 12);
                const uint64_t rep = 0x0101010101010101ull * (uint64_t)off;
                t0 = (prev_csbf == 0 ? kSigPat[0][0] : prev_csbf == 1 ? kSigPat[1][0]
                      : prev_csbf == 2 ? kSigPat[2][0] : kSigPat[3][0]) + rep;
                t1 = (prev_csbf == 0 ? kSigPat[0][1] : prev_csbf == 1 ? kSigPat[1][1]
                      : prev_csbf == 2 ? kSigPat[2][1] : kSigPat[3][1]) + rep;
                if ((xS | yS) == 0) t0 &= ~0xffull;  // DC of the TB: sigCtx 0
            }
            const int cbase = CTX_SIG + (cidx ? 27 : 0);
            const uint64_t sw = scan4_word(scan);
            for (int nn = nstart; nn >= 0; --nn) {
                if (nn > 0 || !infer_dc) {
                    const int e = (int)((sw >> (4 * nn)) & 15u);
                    const uint64_t t = (e & 8) ? t1 : t0;
                    const int sc = (int)((t >> ((e & 7) * 8)) & 0xffu);
                    if (dec_bin(p, cbase + sc)) {
                        sig |= 1u << nn;
                        infer_dc = false;
                    }
                } else {
                    sig |= 1u;  // inferred DC of a coded sub-block
                }
            }
        }
        if (!sig) continue;
        // greater1 / greater2 (9.3.4.2.6-7)
        int ctx_set = (i == 0 || cidx > 0) ? 0 : 2;
        if (any_sb && prev_c1 == 0) ++ctx_set;
        any_sb = true;
        int c1 = 1;
        uint32_t g1 = 0, g2 = 0;
        int first_sig = 31 - __builtin_clz(sig & -sig);  // lowest set bit
        int last_sig = 31 - __builtin_clz(sig);
        int num_g1 = 0, last_g1 = -1;
        for (uint32_t m = sig; m; ) {
            int nn = 31 - __builtin_clz(m);
            m &= ~(1u << nn);
            if (num_g1 >= 8) break;
            int ci = ctx_set * 4 + (c1 < 3 ? c1 : 3) + (cidx ? 16 : 0);
            int f = dec_bin(p, CTX_GT1 + ci);
            ++num_g1;
            if (f) {
                g1 |= 1u << nn;
                if (last_g1 < 0) last_g1 = nn;
            }
            if (c1 > 0) c1 = f ? 0 : c1 + 1;
        }
        prev_c1 = c1;
        bool sign_hidden = !p.cu_bypass && (last_sig - first_sig > 3);
        if (last_g1 >= 0 && dec_bin(p, CTX_GT2 + ctx_set + (cidx ? 4 : 0))) g2 = 1u << last_g1;
        bool hide = (p.flags & SP_SIGN_HIDING) && sign_hidden;
        int nsign = __builtin_popcount(sig) - (hide ? 1 : 0);
        uint32_t signs = dec_bypass_bits(p, nsign);
        signs = nsign ? signs << (32 - nsign) : 0u;  // first decoded sign in bit 31
        int num_sig = 0, sum_abs = 0;
        int c_last_abs = 0, c_last_rice = 0;
        bool first_rem = true;
        for (uint32_t m = sig; m; ) {
            int nn = 31 - __builtin_clz(m);
            m &= ~(1u << nn);
            int base = 1 + (int)((g1 >> nn) & 1) + (int)((g2 >> nn) & 1);
            int rem = 0;
            if (base == ((num_sig < 8) ? ((nn == last_g1) ? 3 : 2) : 1)) {
                int k;
                if (first_rem) {
                    k = 0;
                    first_rem = false;
                } else {
                    k = c_last_rice + (c_last_abs > 3 * (1 << c_last_rice) ? 1 : 0);
                    k = k < 4 ? k : 4;
                }
                uint32_t r = bin_coeff_abs_level_remaining([&]() { return dec_bypass(p); }, k);
                if (r == 0xffffffffu) {
                    p.status |= ST_SYNTAX;
                    r = 0;
                }
                rem = (int)r;
                c_last_abs = base + rem;
                c_last_rice = k;
            }
            int v = base + rem;
            bool neg;
            if (hide && nn == first_sig) {
                sum_abs += v;
                neg = (sum_abs & 1) != 0;
            } else {
                neg = (signs >> 31) != 0;
                signs <<= 1;
                if (hide) sum_abs += v;
            }
            if (neg) v = -v;
            const int pp = scan_pos(p, 2, scan, nn);
            const int xC = (xS << 2) + (pp & 15), yC = (yS << 2) + (pp >> 4);
            if (v > 32767) v = 32767;
            if (v < -32768) v = -32768;
            coef_put(p, ((uint32_t)(uint16_t)(int16_t)v << 16) | (uint32_t)(yC * n + xC));
            ++num_sig;
        }
    }
    coef_flush(p);
    ncoef = p.ncoef - coef_first;  // what was actually stored (capacity overflow drops a group)
}

// TU records are staged like coefficients: record k of the pending group in
// lane k of four staging VGPRs, one 16-byte store per lane at flush time.
HG_INLINE void tu_flush(Parser &p) {
#if !defined(HG_HOST_EMU)
    if (p.tstage_n) {
        const uint32_t n = p.tstage_n;
        const uint32_t cap = PCV(tu_cap) - 1;  // last slot = trash slot
        if (p.ntu + n <= cap) {
            const uint32_t idx = (uint32_t)p.lane < n ? p.ntu + p.lane : cap;
            HG_GLOBAL uint4 *d = (HG_GLOBAL uint4 *)(PCP(tu_out) + idx);
            *d = make_uint4(p.tstage[0], p.tstage[1], p.tstage[2], p.tstage[3]);
            p.ntu += n;
        } else {
            p.status |= ST_CAPACITY;
        }
        p.tstage_n = 0;
    }
#endif
}

HG_INLINE void tu_put(Parser &p, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
#if defined(HG_HOST_EMU)
    if (p.ntu < PCV(tu_cap)) {
        uint32_t *d = reinterpret_cast<uint32_t *>(PCP(tu_out) + p.ntu++);
        d[0] = w0;
        d[1] = w1;
        d[2] = w2;
        d[3] = w3;
    } else {
        p.status |= ST_CAPACITY;
    }
#else
    p.tstage[0] = (uint32_t)hg_writelane((int)w0, (int)p.tstage_n, (int)p.tstage[0]);
    p.tstage[1] = (uint32_t)hg_writelane((int)w1, (int)p.tstage_n, (int)p.tstage[1]);
    p.tstage[2] = (uint32_t)hg_writelane((int)w2, (int)p.tstage_n, (int)p.tstage[2]);
    p.tstage[3] = (uint32_t)hg_writelane((int)w3, (int)p.tstage_n, (int)p.tstage[3]);
    if (++p.tstage_n == 64) tu_flush(p);
#endif
}

// ---------------------------------------------------------------- TB emission
HG_INLINE void emit_tb(Parser &p, int cidx, int x, int y, int log2n, int mode, bool cbf) {
    bool ts = false;
    uint32_t first = p.ncoef, nc = 0;
    HG_PROF(uint64_t t_rc = prof_clock());
    if (cbf) residual_coding(p, log2n, cidx, mode, ts, first, nc);
    HG_PROF(p.prof[PF_RESID] += prof_clock() - t_rc);
    int qp;
    if (cidx == 0) {
        qp = p.qpy_cur + PCV(qpbdY);
    } else {
        int off = cidx == 1 ? PCV(cbOff) : PCV(crOff);
        int qpi = p.qpy_cur + off;
        qpi = qpi < -PCV(qpbdC) ? -PCV(qpbdC) : (qpi > 57 ? 57 : qpi);
        qp = chroma_qp_map(qpi, PCV(chroma)) + PCV(qpbdC);
    }
    uint8_t fl = (uint8_t)cidx;
    if (cbf) fl |= TU_CBF;
    if (ts) fl |= TU_TSKIP;
    if (p.cu_bypass) fl |= TU_BYPASS;
    if (cidx == 0 && log2n == 2) fl |= TU_DST;
    const uint32_t lo = (uint32_t)x | ((uint32_t)y << 16);
    const uint32_t mid = (uint32_t)log2n | ((uint32_t)fl << 8) | ((uint32_t)mode << 16) | ((uint32_t)(uint8_t)qp << 24);
    const uint32_t hi = (uint32_t)nc | ((uint32_t)p.rx << 16);
    tu_put(p, lo, mid, first, hi);
}

// 7.3.8.10 transform_unit
HG_INLINE void transform_unit(Parser &p, int x0, int y0, int xb, int yb, int log2n, int blk, bool cbf_l, bool cbf_cb,
                               bool cbf_cr, bool pcb, bool pcr) {
    const bool chroma4 = PCV(chroma) == 1 && log2n == 2;
    const bool cbf_c = PCV(chroma) == 0 ? false : (chroma4 ? (pcb || pcr) : (cbf_cb || cbf_cr));
    if ((cbf_l || cbf_c) && (p.flags & SP_CU_QP_DELTA) && !p.is_cu_qp_delta_coded) {
        int v = 0;
        while (v < 5 && dec_bin(p, CTX_CU_QP_DELTA + (v == 0 ? 0 : 1))) ++v;
        if (v == 5) {
            uint32_t s = bin_exp_golomb([&]() { return dec_bypass(p); }, 0);
            if (s == 0xffffffffu) {
                p.status |= ST_SYNTAX;
                s = 0;
            }
            v += (int)s;
        }
        if (v && dec_bypass(p)) v = -v;
        p.is_cu_qp_delta_coded = true;
        p.cu_qp_delta_val = v;
        update_qpy(p);
    }
    // edge / no-filter flags of every 4x4 luma block of this TB (MF_*)
    {
        const int nb = 1 << (log2n - 2);
        HG_LANE_LOOP(k, p.lane, nb * nb) {
            int bx = k % nb, by = k / nb;
            int gx = (x0 >> 2) + bx, gy = (y0 >> 2) + by;
            if (gx < PCV(w4) && gy < PCV(h4))
                PCP(gflags)[gy * PCV(w4) + gx] =
                    (uint8_t)((bx == 0 ? MF_EDGE_V : 0) | (by == 0 ? MF_EDGE_H : 0) | (p.cu_bypass ? MF_NOFILT : 0));
        }
    }
    const int lmode = unis(p.w->ipm[(y0 - p.ctby) >> 2][((x0 - p.ctbx) >> 2) + 1]);
    // luma TB, then (4:2:0) the Cb and Cr TBs — one emit_tb call site so it inlines once
    int ntb = 1;
    if (PCV(chroma) != 0 && (!chroma4 || blk == 3)) ntb = 3;
    for (int t = 0; t < ntb; ++t) {
        int x, y, l, m;
        bool cbf;
        if (t == 0) {
            x = x0, y = y0, l = log2n, m = lmode, cbf = cbf_l;
        } else if (!chroma4) {
            x = x0 >> 1, y = y0 >> 1, l = log2n - 1, m = p.cu_chroma_mode, cbf = t == 1 ? cbf_cb : cbf_cr;
        } else {
            x = xb >> 1, y = yb >> 1, l = 2, m = p.cu_chroma_mode, cbf = t == 1 ? pcb : pcr;
        }
        emit_tb(p, t, x, y, l, m, cbf);
    }
}

// 7.3.8.8 transform_tree, iterative (pre-order, children 0..3)
HG_INLINE void transform_tree(Parser &p, int x0, int y0, int log2cb) {
    auto pack = [](int x, int y, int xb, int yb, int l, int d, int blk, int pcb, int pcr) -> uint64_t {
        return (uint64_t)x | ((uint64_t)y << 13) | ((uint64_t)xb << 26) | ((uint64_t)yb << 39) |
               ((uint64_t)l << 52) | ((uint64_t)d << 55) | ((uint64_t)blk << 58) | ((uint64_t)pcb << 60) |
               ((uint64_t)pcr << 61);
    };
    uint64_t *st = p.w->tt;
    int sp = 0;
    st[0] = pack(x0, y0, x0, y0, log2cb, 0, 0, 0, 0);
    sp = 1;
    const int max_depth = PCV(maxDepthIntra) + p.cu_intra_split;
    while (sp > 0) {
        ensure_bytes(p);
        --sp;
        uint64_t e = st[sp];
        uint32_t lo = uni((uint32_t)e), hi = uni((uint32_t)(e >> 32));
        e = ((uint64_t)hi << 32) | lo;
        int x = (int)(e & 8191), y = (int)((e >> 13) & 8191), xb = (int)((e >> 26) & 8191), yb = (int)((e >> 39) & 8191);
        int l = (int)((e >> 52) & 7), d = (int)((e >> 55) & 7), blk = (int)((e >> 58) & 3);
        bool pcb = (e >> 60) & 1, pcr = (e >> 61) & 1;
        bool split;
        if (l <= PCV(maxTb) && l > PCV(minTb) && d < max_depth && !(p.cu_intra_split && d == 0))
            split = dec_bin(p, CTX_SPLIT_TF + 5 - l);
        else
            split = l > PCV(maxTb) || (p.cu_intra_split && d == 0);
        bool cbf_cb = false, cbf_cr = false;
        if (l > 2 && PCV(chroma) != 0) {
            if (d == 0 || pcb) cbf_cb = dec_bin(p, CTX_CBF_CHROMA + d);
            if (d == 0 || pcr) cbf_cr = dec_bin(p, CTX_CBF_CHROMA + d);
        }
        if (split) {
            int h = 1 << (l - 1);
            st[sp + 0] = pack(x + h, y + h, x, y, l - 1, d + 1, 3, cbf_cb, cbf_cr);
            st[sp + 1] = pack(x, y + h, x, y, l - 1, d + 1, 2, cbf_cb, cbf_cr);
            st[sp + 2] = pack(x + h, y, x, y, l - 1, d + 1, 1, cbf_cb, cbf_cr);
            st[sp + 3] = pack(x, y, x, y, l - 1, d + 1, 0, cbf_cb, cbf_cr);
            sp += 4;
            continue;
        }
        bool cbf_l = dec_bin(p, CTX_CBF_LUMA + (d == 0 ? 1 : 0));
        transform_unit(p, x, y, xb, yb, l, blk, cbf_l, cbf_cb, cbf_cr, pcb, pcr);
    }
}

// 8.4.2 luma intra prediction mode
HG_INLINE int derive_luma_mode(Parser &p, int xPb, int yPb, int prev, int mpm_idx, int rem) {
    int ca, cb;
    if (xPb <= 0) ca = 1;
    else ca = unis(p.w->ipm[(yPb - p.ctby) >> 2][((xPb - 1 - p.ctbx) >> 2) + 1]);
    if (yPb - 1 < p.ctby) cb = 1;  // above CTB (or picture edge) → DC
    else cb = unis(p.w->ipm[((yPb - 1 - p.ctby) >> 2)][((xPb - p.ctbx) >> 2) + 1]);
    int l0, l1, l2;
    if (ca == cb) {
        if (ca < 2) {
            l0 = 0;
            l1 = 1;
            l2 = 26;
        } else {
            l0 = ca;
            l1 = 2 + ((ca + 29) % 32);
            l2 = 2 + ((ca - 2 + 1) % 32);
        }
    } else {
        l0 = ca;
        l1 = cb;
        if (ca != 0 && cb != 0) l2 = 0;
        else if (ca != 1 && cb != 1) l2 = 1;
        else l2 = 26;
    }
    if (prev) return mpm_idx == 0 ? l0 : (mpm_idx == 1 ? l1 : l2);
    int t;
    if (l0 > l1) { t = l0; l0 = l1; l1 = t; }
    if (l0 > l2) { t = l0; l0 = l2; l2 = t; }
    if (l1 > l2) { t = l1; l1 = l2; l2 = t; }
    int m = rem;
    if (m >= l0) ++m;
    if (m >= l1) ++m;
    if (m >= l2) ++m;
    return m;
}

// 7.3.8.5 coding_unit (intra)
HG_INLINE void coding_unit(Parser &p, int x0, int y0, int log2cb, int depth) {
    const int n = 1 << log2cb;
    if (p.qg_new) {
        derive_qp_pred(p);
        p.qg_new = false;
    }
    update_qpy(p);
    p.cu_bypass = (p.flags & SP_TQ_BYPASS) ? dec_bin(p, CTX_TQ_BYPASS) : 0;
    int nxn = 0;
    if (log2cb == PCV(minCb)) nxn = !dec_bin(p, CTX_PART_MODE);
    if (!nxn && (p.flags & SP_PCM) && log2cb >= PCV(pcmMin) && log2cb <= PCV(pcmMax) && dec_term(p)) {
        // pcm_flag = 1: not supported on the GPU path (halfmoonbay has pcm_enabled_flag = 0)
        p.status |= ST_UNSUPPORTED;
        return;
    }
    // CtDepth of the CU
    {
        const int nd = n >> 3;
        const int dx = (x0 - p.ctbx) >> 3, dy = (y0 - p.ctby) >> 3;
        HG_LANE_LOOP(k, p.lane, nd * nd) p.w->depth[dy + k / nd][dx + k % nd + 1] = (uint8_t)depth;
    }
    const int np = nxn ? 4 : 1, pb = nxn ? n >> 1 : n;
    int prev[4] = {0, 0, 0, 0};
    for (int i = 0; i < np; ++i) prev[i] = dec_bin(p, CTX_PREV_INTRA);
    for (int i = 0; i < np; ++i) {
        int mpm = 0, rem = 0;
        if (prev[i]) mpm = dec_bypass(p) ? (dec_bypass(p) ? 2 : 1) : 0;
        else rem = (int)dec_bypass_bits(p, 5);
        const int xPb = x0 + (i & 1) * pb, yPb = y0 + (i >> 1) * pb;
        const int m = derive_luma_mode(p, xPb, yPb, prev[i], mpm, rem);
        const int nb = pb >> 2;
        const int bx = (xPb - p.ctbx) >> 2, by = (yPb - p.ctby) >> 2;
        HG_LANE_LOOP(k, p.lane, nb * nb) p.w->ipm[by + k / nb][bx + k % nb + 1] = (uint8_t)m;
    }
    if (PCV(chroma) != 0) {
        int icpm = dec_bin(p, CTX_CHROMA_MODE) ? (int)dec_bypass_bits(p, 2) : 4;
        int lm = unis(p.w->ipm[(y0 - p.ctby) >> 2][((x0 - p.ctbx) >> 2) + 1]);
        int cm;
        if (icpm == 4) {
            cm = lm;
        } else {
            cm = icpm == 0 ? 0 : (icpm == 1 ? 26 : (icpm == 2 ? 10 : 1));
            if (cm == lm) cm = 34;
        }
        p.cu_chroma_mode = cm;
    }
    p.cu_intra_split = nxn;
    transform_tree(p, x0, y0, log2cb);
    // QpY of the CU: local 8x8 map (for qPY_A/B) and global 4x4 map (deblocking)
    {
        const int nd = n >> 3;
        const int dx = (x0 - p.ctbx) >> 3, dy = (y0 - p.ctby) >> 3;
        HG_LANE_LOOP(k, p.lane, nd * nd) p.w->qpy[dy + k / nd][dx + k % nd] = (int8_t)p.qpy_cur;
        const int nb = n >> 2;
        HG_LANE_LOOP(k, p.lane, nb * nb) {
            int gx = (x0 >> 2) + k % nb, gy = (y0 >> 2) + k / nb;
            if (gx < PCV(w4) && gy < PCV(h4)) PCP(gqpy)[gy * PCV(w4) + gx] = (int8_t)p.qpy_cur;
        }
    }
    p.qp_prev_last = p.qpy_cur;
}

// 7.3.8.4 coding_quadtree, iterative
HG_INLINE void coding_quadtree(Parser &p) {
    uint32_t *st = p.w->cqt;
    st[0] = (uint32_t)p.ctbx | ((uint32_t)p.ctby << 13) | ((uint32_t)p.log2ctb << 26);
    int sp = 1;
    while (sp > 0 && !(p.status & ST_UNSUPPORTED)) {
        ensure_bytes(p);
        --sp;
        uint32_t e = uni(st[sp]);
        int x = (int)(e & 8191), y = (int)((e >> 13) & 8191), l = (int)((e >> 26) & 7), d = (int)(e >> 29);
        const int n = 1 << l;
        bool split;
        if (x + n <= PCV(W) && y + n <= PCV(H) && l > PCV(minCb)) {
            int cond = 0;
            const int dx = (x - p.ctbx) >> 3, dy = (y - p.ctby) >> 3;
            if (x > 0 && unis(p.w->depth[dy][dx]) > d) ++cond;  // column dx is x-8 (shifted by 1)
            if (y > 0) {
                int ad = (y - 1 < p.ctby) ? unis(p.depth_above[x >> 3]) : unis(p.w->depth[dy - 1][dx + 1]);
                if (ad > d) ++cond;
            }
            split = dec_bin(p, CTX_SPLIT_CU + cond);
        } else {
            split = l > PCV(minCb);
        }
        if (l >= PCV(log2qg)) {
            p.is_cu_qp_delta_coded = false;
            p.cu_qp_delta_val = 0;
            p.qg_new = true;
            p.qg_x = x;
            p.qg_y = y;
        }
        if (split) {
            const int h = n >> 1;
            auto pk = [&](int cx, int cy) {
                return (uint32_t)cx | ((uint32_t)cy << 13) | ((uint32_t)(l - 1) << 26) | ((uint32_t)(d + 1) << 29);
            };
            // push in reverse so child 0 is processed first
            if (x + h < PCV(W) && y + h < PCV(H)) {
                st[sp] = pk(x + h, y + h);
                ++sp;
            }
            if (y + h < PCV(H)) {
                st[sp] = pk(x, y + h);
                ++sp;
            }
            if (x + h < PCV(W)) {
                st[sp] = pk(x + h, y);
                ++sp;
            }
            st[sp] = pk(x, y);
            ++sp;
            continue;
        }
        coding_unit(p, x, y, l, d);
    }
}

}  // namespace

// ---------------------------------------------------------------- kernel
// Occupancy: 6 waves/SIMD (<= 80 VGPRs) so most pictures of a large batch are
// resident at once; the bin loop is latency-bound per wave, so more waves
// per SIMD is worth the few spills this costs.  HG_PARSE_WPE=0 disables.
#ifndef HG_PARSE_WPE
#define HG_PARSE_WPE 6
#endif
#if HG_PARSE_WPE > 0 && !defined(HG_HOST_EMU)
#define HG_PARSE_ATTR __attribute__((amdgpu_waves_per_eu(HG_PARSE_WPE, HG_PARSE_WPE)))
#else
#define HG_PARSE_ATTR
#endif
__global__ void __launch_bounds__(kParseWaves * 64) HG_PARSE_ATTR k_parse(BatchArgs a) {
#if defined(HG_HOST_EMU)
    unsigned char *smem = g_emu.smem;
#else
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
#endif
    // block = P pictures x G waves; wave (g, w) parses rows w, w+G, ... of picture
    // blockIdx.x * P + g.  G = 1 (the batch default) walks every WPP row of its
    // picture itself; G > 1 runs the rows of one picture concurrently.
    const int nwb = (int)HG_UNI(blockDim.x >> 6);
    const int G = a.parse_group;
    const int P = nwb / G;
    const int wave = (int)HG_UNI(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int gi = wave / G, wrow = wave - gi * G;
    const int pic_raw = a.pic0 + blockIdx.x * P + gi;
    const bool active = pic_raw < a.pic0 + a.n_pics;
    const int pic = active ? pic_raw : a.pic0;
    const PicDesc pd = a.pics[pic];
    const SeqParams sp = a.seqs[pd.seq];

    WaveLds *wl = reinterpret_cast<WaveLds *>(smem) + wave;
    const int dl_stride = ((a.max_width >> 3) + 15) & ~15;
    uint8_t *grp = smem + sizeof(WaveLds) * nwb + (size_t)gi * parse_group_bytes(a.max_width, a.max_wctb, G);
    uint32_t *progress = reinterpret_cast<uint32_t *>(grp);                      // [G]
    uint32_t *wpp_slot = progress + ((G + 3) & ~3);                              // [2][64] context words
    uint8_t *depth_line = reinterpret_cast<uint8_t *>(wpp_slot + 2 * 64);         // [2][dl_stride]
    SaoParams *sao_line = reinterpret_cast<SaoParams *>(depth_line + 2 * dl_stride);  // [2][max_wctb]

    Parser p;
    p.w = wl;
    p.w->pc.W = sp.width;
    p.w->pc.H = sp.height;
    p.log2ctb = sp.log2_ctb;
    p.ctb = 1 << sp.log2_ctb;
    p.w->pc.wctb = (PCV(W) + p.ctb - 1) >> p.log2ctb;
    p.w->pc.hctb = (PCV(H) + p.ctb - 1) >> p.log2ctb;
    p.w->pc.minCb = sp.log2_min_cb;
    p.w->pc.minTb = sp.log2_min_tb;
    p.w->pc.maxTb = sp.log2_max_tb;
    p.w->pc.maxDepthIntra = sp.max_th_depth_intra;
    p.w->pc.chroma = sp.chroma_format;
    p.w->pc.bdY = sp.bit_depth_y;
    p.w->pc.bdC = sp.bit_depth_c;
    p.w->pc.qpbdY = 6 * (PCV(bdY) - 8);
    p.w->pc.qpbdC = 6 * (PCV(bdC) - 8);
    p.flags = sp.flags;
    p.w->pc.pcmMin = sp.log2_min_pcm;
    p.w->pc.pcmMax = sp.log2_max_pcm;
    p.w->pc.log2qg = p.log2ctb - sp.diff_cu_qp_delta_depth;
    p.w->pc.cbOff = sp.cb_qp_offset + pd.cb_qp_off;
    p.w->pc.crOff = sp.cr_qp_offset + pd.cr_qp_off;
    p.w->pc.sliceQp = pd.slice_qp;
    p.w->pc.saoL = pd.sao_luma;
    p.w->pc.saoC = pd.sao_chroma;
    p.src = a.bits + pd.bits_off;
    p.nal_end = pd.bits_len;
    p.status = 0;
    p.lane = lane;
    p.cx.load_tables(lane);
#if !defined(HG_HOST_EMU)
    p.cstage = 0;
    p.cstage_n = 0;
    p.tstage[0] = p.tstage[1] = p.tstage[2] = p.tstage[3] = 0;
    p.tstage_n = 0;
    {
        const uint32_t e = kScanPos[3][0][lane];
        p.scanv = ((e & 7) | ((e >> 4) << 3)) | ((uint32_t)kScanInv[3][0][lane] << 8);
    }
#endif
    HG_PROF(for (int k = 0; k < PF_N; ++k) p.prof[k] = 0; const uint64_t t_start = prof_clock();)
    p.w->pc.w4 = (PCV(W) + 3) >> 2;
    p.w->pc.h4 = (PCV(H) + 3) >> 2;
    p.w->pc.gqpy = (HG_GLOBAL int8_t *)(a.maps + pd.map_off);
    p.w->pc.gflags = (HG_GLOBAL uint8_t *)(a.maps + pd.map_off + (size_t)PCV(w4) * PCV(h4));
    SaoParams *gsao = a.sao + pd.sao_off;
    const uint32_t *subs = a.subs + pd.sub_first;
    const bool wpp = (p.flags & SP_WPP) != 0;

    progress[wrow] = 0;
    __syncthreads();

    // rows: WPP → one substream per CTB row, wave w takes rows w, w+16, ...;
    // otherwise the picture is one substream and wave 0 walks every row.
    const int row_step = wpp ? G : 1;
    const int first_row = !active ? PCV(hctb) : (wpp ? wrow : (wrow == 0 ? 0 : PCV(hctb)));
    const uint32_t stride = (uint32_t)PCV(wctb) + 1;
    const int prev_wave = (wrow + G - 1) % G;
    bool stop = false;
    for (int r = first_row; r < PCV(hctb) && !stop; r += row_step) {
        p.ry = r;
        p.w->pc.tu_out = (HG_GLOBAL TuRec *)(a.tus + pd.tu_off + (uint64_t)r * pd.tu_cap_row);
        p.w->pc.coef_out = (HG_GLOBAL Coef *)(a.coefs + pd.coef_off + (uint64_t)r * pd.coef_cap_row);
        p.ntu = p.ncoef = 0;
        p.w->pc.tu_cap = pd.tu_cap_row;
        p.w->pc.coef_cap = pd.coef_cap_row;
        p.depth_above = depth_line + ((r + 1) & 1) * dl_stride;
        uint8_t *depth_cur_line = depth_line + (r & 1) * dl_stride;
        SaoParams *sao_above = sao_line + ((r + 1) & 1) * a.max_wctb;
        SaoParams *sao_cur_line = sao_line + (r & 1) * a.max_wctb;
        for (int c = 0; c < PCV(wctb); ++c) {
            p.rx = c;
            p.ctbx = c << p.log2ctb;
            p.ctby = r << p.log2ctb;
            if (wpp && r > 0) {
                // WPP lag: row r-1 must have finished CTU min(c+1, wctb-1)
                HG_PROF(uint64_t t_w = prof_clock());
                const uint32_t need = (uint32_t)(r - 1) * stride + (uint32_t)((c + 2) < PCV(wctb) ? (c + 2) : PCV(wctb));
                for (uint32_t spin = 0; uni(hg_atomic_load(&progress[prev_wave])) < need; ++spin) {
                    if (spin > (1u << 24)) {  // bounded: never hang the device
                        p.status |= ST_SUBSTREAM_END;
                        break;
                    }
                    HG_SLEEP();
                }
                HG_FENCE_ACQ();
                HG_PROF(p.prof[PF_SPIN] += prof_clock() - t_w);
            }
            if (c == 0 && (wpp || r == 0)) {
                // substream start: contexts (init or WPP sync, 9.3.1) + engine (9.3.2.5)
                if (r == 0 || PCV(wctb) < 2) ctx_init(p);
                else
                    p.cx.restore(wpp_slot + ((r + 1) & 1) * 64, lane);
                engine_init(p, subs[wpp ? r : 0]);
                if (r == 0) p.first_qg_in_slice = true;
            }
            // left-CTB columns of the per-wave maps
            if (c > 0) {
                const int nb4 = p.ctb >> 2, nb8 = p.ctb >> 3;
                HG_LANE_LOOP(k, lane, nb4) wl->ipm[k][0] = wl->ipm[k][nb4];
                HG_LANE_LOOP(k, lane, nb8) wl->depth[k][0] = wl->depth[k][nb8];
            }
            HG_PROF(uint64_t t_s = prof_clock());
            if (PCV(saoL) || PCV(saoC)) parse_sao(p, sao_above, gsao);
            HG_PROF(uint64_t t_q = prof_clock());
            coding_quadtree(p);
            HG_PROF(p.prof[PF_SAO] += t_q - t_s; p.prof[PF_CQT] += prof_clock() - t_q);
            if (p.status & ST_UNSUPPORTED) {
                stop = true;
            }
            if (wpp && c == 1)
                p.cx.save(wpp_slot + (r & 1) * 64, lane);
            // bottom row of this CTB for the row below: depths, SAO parameters
            {
                const int nb8 = p.ctb >> 3;
                HG_LANE_LOOP(k, lane, nb8) depth_cur_line[(p.ctbx >> 3) + k] = wl->depth[nb8 - 1][k + 1];
                sao_cur_line[c] = wl->sao_left;
            }
            // end_of_slice_segment_flag / end_of_subset_one_bit (slice.rs:214-227)
            const bool last_in_pic = (r == PCV(hctb) - 1) && (c == PCV(wctb) - 1);
            ensure_bytes(p);
            int eos = dec_term(p);
            if (eos != (last_in_pic ? 1 : 0)) p.status |= ST_SUBSTREAM_END;
            if (!last_in_pic && wpp && c == PCV(wctb) - 1) {
                if (!dec_term(p)) p.status |= ST_SUBSTREAM_END;
            }
            check_overrun(p);
            // publish progress (release: LDS lines, WPP slot, global maps)
            HG_FENCE_REL();
            hg_atomic_store(&progress[wrow], (uint32_t)r * stride + (uint32_t)(c + 1));
            if (stop) break;
        }
        tu_flush(p);
        a.row_counts[2 * (pd.row_off + r)] = p.ntu;
        a.row_counts[2 * (pd.row_off + r) + 1] = p.ncoef;
    }
    if (stop && wpp) {
        // let rows waiting on this wave drain
        hg_atomic_store(&progress[wrow], 0x7fffffffu);
    }
    if (p.status) atomicOr(&a.status[pic], p.status);  // uniform branch; idempotent OR
    HG_PROF(p.prof[PF_WAVE] = prof_clock() - t_start;
            if (lane == 0) for (int k = 0; k < PF_N; ++k) atomicAdd((unsigned long long *)&g_prof[k], (unsigned long long)p.prof[k]);)
}

ParseShape parse_shape(const BatchArgs &a) {
    // Many pictures: one wave per picture (no WPP wait, every wave busy);
    // few: the rows of a picture on G waves.  HEIFGPU_PARSE_GROUP overrides.
    static const int forced = [] {
        const char *e = std::getenv("HEIFGPU_PARSE_GROUP");
        return e ? std::atoi(e) : 0;
    }();
    const int rows = a.max_rows < 1 ? 1 : (a.max_rows > kParseWaves ? kParseWaves : a.max_rows);
    ParseShape sh;
    sh.group = forced > 0 ? (forced < rows ? forced : rows) : (a.n_pics >= kParseSerialMinPics ? 1 : rows);
    sh.pics_per_block = sh.group == 1 ? kParseSerialPicsPerBlock : 1;
    sh.blocks = (a.n_pics + sh.pics_per_block - 1) / sh.pics_per_block;
    const int nwb = sh.group * sh.pics_per_block;
    sh.threads = 64 * nwb;
    sh.lds = sizeof(WaveLds) * nwb + sh.pics_per_block * parse_group_bytes(a.max_width, a.max_wctb, sh.group);
    return sh;
}

#if defined(HG_HOST_EMU)
void emu_parse(const BatchArgs &a0) {
    if (parse_lanes_selected(a0)) return emu_parse_lanes(a0);
    BatchArgs a = a0;
    const ParseShape sh = parse_shape(a);
    a.parse_group = sh.group;
    emu_launch(k_parse, sh.blocks, 1, sh.threads / 64, a, false, sh.lds);
}
#else
hipError_t launch_parse(const BatchArgs &a0, hipStream_t s) {
    if (parse_lanes_selected(a0)) return launch_parse_lanes(a0, s);
    BatchArgs a = a0;
    const ParseShape sh = parse_shape(a);
    a.parse_group = sh.group;
    hipLaunchKernelGGL(k_parse, dim3(sh.blocks), dim3(sh.threads), sh.lds, s, a);
    return hipGetLastError();
}
#endif

}  // namespace hg

#if !defined(HG_HOST_EMU)
// Debug hook (include/heifgpu.h): copies the k_parse counters out and zeroes
// them.  Returns the number of counters, or 0 when the library was built
// without -DHG_PARSE_PROF (the product build).
extern "C" int heifgpu_debug_counters(uint64_t *out, int n) {
#if defined(HG_PARSE_PROF)
    uint64_t tmp[16] = {};
    if (hipMemcpyFromSymbol(tmp, HIP_SYMBOL(hg::g_prof), sizeof(tmp)) != hipSuccess) return -1;
    uint64_t zero[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(hg::g_prof), zero, sizeof(zero)) != hipSuccess) return -1;
    if (hg::parse_lanes_counters(tmp + 8) < 0) return -1;  // k_parse_lanes: slots 8..15
    for (int k = 0; k < n && k < 16; ++k) out[k] = tmp[k];
    return 16;
#else
    (void)out;
    (void)n;
    return 0;
#endif
}
#endif
