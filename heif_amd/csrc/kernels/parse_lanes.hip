// parse_lanes.hip — CABAC slice-data parser (pipeline stage 1), one
// substream per LANE.
//
// Replaces SliceSegmentReader::read_data / read_coding_tree_unit and the
// todo!() sao() / coding_quadtree() of src/hevc/slice.rs:206-256, with the
// engine of src/cabac/arithmetic.rs and the binarizations of
// src/cabac/decoder.rs, plus everything H.265 needs below them (7.3.8.3-14,
// 9.3.4.2 ctxInc, 8.4.2 MPM, 8.6.1 QP).  Outputs: TU records, coefficients,
// the QP / edge maps, SAO parameters and per-row counts (desc.hpp).
//
// Every lane of a wave runs its own substream: with WPP a lane is one CTB
// row of a picture and a picture's rows sit in consecutive lanes (R =
// min(rows, 64) lanes; a picture with more than 64 rows wraps round them, lane
// r taking rows r, r + R, r + 2R, ...); without WPP the slice is one
// substream and one lane walks all of its rows.  Each lane walks its substream as a sequence of
// syntax units (CTU start + SAO, coding-quadtree descent, coding-unit header,
// transform-tree descent + transform_unit, residual header, one 4x4
// sub-block, CTU end); one pass of the kernel loop runs one unit on every
// live lane, the lanes in the same kind of unit sharing its instructions, and
// the arithmetic decoder (context bytes in the lane's LDS block) runs inline
// inside the units.  So up to 64 substreams share each engine instruction,
// where k_parse spends a whole wave on one.
//
// WPP (9.3.1) inside the wave: row r+1 starts CTU c once row r has finished
// CTU c+1 (per-lane progress words in LDS, counting r * wctb + CTUs done so
// they stay monotone when a lane wraps to a later row); row r writes its
// contexts after CTU 1 straight into row r+1's lane block, or, when rows wrap
// (that lane may still be parsing an earlier row), into its staging block.  The CtDepth of a CTB's bottom
// 8x8 row and its SAO parameters reach the row below through global memory
// (maps arena / SAO array), read with L1-bypassing loads.
//
// Left / above neighbour state (IntraPredModeY, CtDepth, QpY) needs no CTB
// map: in z-order the last block written in a 4x4 (8x8) row of the CTB row is
// always the left neighbour of the next block in that row, and likewise for
// columns within a CTB, so a "last written" value per row and per column is
// enough (ipmL/ipmA, dL/dA, qL/qA).
#include "cabac.hpp"
#include "kernels.hpp"
#include "tables.hpp"

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#if defined(HG_HOST_EMU)
#include <cstdio>
#endif

#if !defined(HG_HOST_EMU)
// v_writelane_b32 (this clang exposes no builtin for it): lane `lane` of `old` := src
extern "C" __device__ int hg_writelane(int src, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
#endif

// HG_PARSE_TU (library build, Makefile): 1 compiles the lanes / rows kernels and
// launch_parse, 2 (kernels/parse_solo.hip) the solo / spread kernels, so each
// translation unit gets its own code-generation flags; unset, everything (the
// host emulation and the counter builds)
#if defined(HG_PARSE_TU) && HG_PARSE_TU != 1 && HG_PARSE_TU != 2
#error "HG_PARSE_TU is 1 or 2"
#endif
#if !defined(HG_PARSE_TU) || HG_PARSE_TU == 1
#define HG_PARSE_WANT_LANES 1
#else
#define HG_PARSE_WANT_LANES 0
#endif
#if !defined(HG_PARSE_TU) || HG_PARSE_TU == 2
#define HG_PARSE_WANT_SOLO 1
#else
#define HG_PARSE_WANT_SOLO 0
#endif

namespace hg {

namespace {
__constant__ uint8_t c_lps_l[256] = {HG_LPS_TABLE};
__constant__ uint8_t c_trans_l[64] = {HG_TRANS_LPS};
__constant__ uint8_t c_ctx_init_l[CTX_NUM] = {HG_CTX_INIT_VALUES};
}  // namespace
#if defined(HG_PARSE_PROF) && !defined(HG_HOST_EMU)
// s_memtime cycles per wave: [0] kernel, [1] passes, [2..6] unit kinds CTU, tree (CQT+CU+TT), TB, SB,
// CTU_END; [7] units run (lanes x unit executions) (tuning build only; heifgpu_debug_counters slots 8..15)
__device__ uint64_t g_prof_lanes[16];  // 8 used; 16 in the prof-sb build
// solo / spread: per CTU (index (global CTB row) * 128 + column) s_memrealtime of
// the first time its wave wanted to start it, the start of its U_CTU unit and
// the end of its U_CTU_END unit (heifgpu_debug_counters slots 8 on)
constexpr int kCtuTimeCap = 1 << 17;
__device__ uint64_t g_ctu_t[kCtuTimeCap][3];
// k_parse_lanes (one wave per workgroup): records kWaveRec.. of g_ctu_t hold
// each wave's own cycle breakdown, three records per wave (five in prof-sb)
constexpr int kWaveRec = 4096, kWaveRecCap = 4096;
#endif

namespace {

// engine row of pStateIdx st (Eng::tab): rangeTabLps[st][0..3], then the
// next context byte (pStateIdx << 1 | valMps) to XOR with valMps after an LPS
// (transIdxLps << 1, | 1 at pStateIdx 0 where valMps flips) and after an MPS
// (transIdxMps << 1)
HG_HD inline uint64_t state_row(int st) {
    uint64_t r = 0;
    for (int q = 0; q < 4; ++q) r |= (uint64_t)c_lps_l[(st << 2) | q] << (8 * q);
    const uint64_t lps_next = ((uint64_t)c_trans_l[st] << 1) | (st == 0 ? 1u : 0u);
    const uint64_t mps_next = (uint64_t)(st < 62 ? st + 1 : st) << 1;
    return r | (lps_next << 32) | (mps_next << 40);
}

// Vector engines (lanes): one row per context byte s = pStateIdx << 1 |
// valMps, valMps folded in: rangeTabLps[4], then the next context byte after
// an LPS (bits 32-38) and after an MPS (bits 40-46), each with the bin that
// path decodes to in its bit 7.  A decision indexes it by the byte itself and
// reads the new byte and the bin from one shift (no valMps extraction, XOR or
// row-index masking; r05 A/B at 128 images: 18,770 vs 18,590 Mpix/s); a
// register cache inserts the shifted byte under a 7-bit mask (v_bfi), so the
// bin bit costs no extra mask there (dec_t; r06 A/B: VALU 19.92 -> 19.60 G per
// launch, 23,056 -> 23,108 Mpix/s, profiles/r06/ab/ab_bfi.txt).
// (A/B r05: the decoded bin in bit 7 of the context byte itself, 256 rows:
// 19,020 vs 19,200 Mpix/s, rejected)
constexpr int kTabRows = 128;
HG_HD inline uint64_t state_row_ctx(int s) {
    const uint64_t r = state_row(s >> 1);
    const uint64_t mps = (uint64_t)(s & 1);
    return (r & 0xffffffffull) | (((((r >> 32) & 0xffu) ^ mps) | ((mps ^ 1u) << 7)) << 32) |
           (((((r >> 40) & 0xffu) ^ mps) | (mps << 7)) << 40);
}

constexpr uint32_t kProgDone = 0x7fffffffu;
// (parse waves at issue priority HG_PARSE_SETPRIO: wave.hpp)
// LanePic.flags bit above the SP_ flags: k_intra_stream reads this picture's TU
// and coefficient records while the parse writes them (agent-scope stores)
constexpr uint32_t PF_COHERENT = 1u << 31;

// per-lane LDS block (208 bytes: lanes l and l + 16 share a bank for one
// context byte; an odd 212-byte block, 64 banks, measured 76.8 vs 76.3 ms, r04)
struct alignas(16) LaneLds {
    uint8_t ctx[CTX_PAD];
    uint8_t ipmL[16], ipmA[16];  // IntraPredModeY (4x4 units): last written per row / per column
    uint8_t dL[8], dA[8];        // CtDepth (8x8 units)
    int8_t qL[8], qA[8];         // QpY (8x8 units)
};

// picture constants and output pointers (LDS, one per picture of the wave)
struct LanePic {
    int W, H, log2ctb, wctb, hctb, minCb, minTb, maxTb, maxDepthIntra, chroma;
    int log2qg, bdY, bdC, qpbdY, qpbdC, pcmMin, pcmMax, pcmBdY, pcmBdC, cbOff, crOff, sliceQp;
    int subx, suby;  // log2 SubWidthC, SubHeightC (Table 6-1)
    int w4, h4, w8, saoL, saoC;
    int R, lane0, ring;  // lanes of the picture, its first lane, rows wrap round the lanes (WPP rows > R)
    uint32_t flags, bits_off, bits_end, sub_first, row_off, tu_cap, coef_cap, pic;
    // global memory, said so in the type: a generic pointer loaded from LDS
    // would make every store through it a flat store, and flat stores count in
    // lgkmcnt, so each later LDS read of the wave would wait for them
    int8_t HG_GAS *gqpy;
    uint8_t HG_GAS *gflags;
    uint8_t HG_GAS *gdepth;
    SaoParams HG_GAS *gsao;
    TuRec HG_GAS *tu_base;
    Coef HG_GAS *coef_base;
};

// syntax units (Lane.st)
enum Unit : int {
    U_DONE = 0,
    U_CTU,      // WPP wait, substream start, sao()                      7.3.8.2-3
    U_CQT,      // coding_quadtree descent from the current node         7.3.8.4
    U_CU,       // coding_unit up to transform_tree                      7.3.8.5
    U_TT,       // transform_tree descent + transform_unit               7.3.8.8-10
    U_TB,       // next TB of the TU: record, or residual_coding header  7.3.8.11
    U_SB,       // one 4x4 sub-block of residual_coding                  7.3.8.11
    U_CTU_END,  // end_of_slice_segment_flag / end_of_subset_one_bit     7.3.8.1
};

// Lane.fl bits
enum : uint32_t {
    F_WPP = 1u << 0,
    F_FIRST_QG = 1u << 1,
    F_QG_NEW = 1u << 2,
    F_DQP_CODED = 1u << 3,
    F_BYPASS = 1u << 4,   // cu_transquant_bypass_flag
    F_NXN = 1u << 5,      // PART_NxN
    F_CBF_L = 1u << 6,
    F_CBF_CB = 1u << 7,
    F_CBF_CR = 1u << 8,
    F_TS = 1u << 9,       // transform_skip_flag of the current TB
    F_TB_CBF = 1u << 10,
    F_ANY_SB = 1u << 11,  // a sub-block of the TB had significant coefficients
    F_STOP = 1u << 12,
    F_PCM = 1u << 13,     // the TB being recorded is a PCM block
    F_REINIT = 1u << 14,  // solo modes: engine re-initialisation at byte L.reinit before the next unit
    // bits 16-31: the dependent segments started inside a row so far (kMsegOne
    // each; in fl, not a register of its own: the lanes parse sits at its VGPR floor)
};
constexpr uint32_t kMsegShift = 16, kMsegOne = 1u << kMsegShift;
// Lane.status bit, never reported (unit_ctu clears it): a dependent slice
// segment starts at the next CTU, inside the row (lanes_nmid).  Carried in
// status, which the CTU end's error branch writes anyway: set in fl there, the
// flag cost the lanes parse 16 VGPRs of allocation (160 -> 176)
constexpr uint32_t ST_SEGSW = 1u << 30;

struct Lane {
    // arithmetic decoder (9.3.4.3): ivlOffset carried with k look-ahead bits,
    // value = ivlOffset * 2^k + next k bits of the substream, so a renormalisation
    // only lowers k; a bit window tops value up 16 bits at a time
    uint32_t range, value;
    int k;
    uint64_t cur;     // next bits of the substream, MSB first (cn valid)
    int cn;
    // RBSP queue, dwords as loaded (little endian): a (ai consumed), then b (valid: bv), then f (in
    // flight: fp); lb = offset of the 16 bytes after the last loaded block.  f is issued at a pass
    // start and lands at the next one, after the pass's one memory wait, so refills inside a pass
    // never wait on memory (a wait for a load also waits for every older store)
    uint32_t a0, a1, a2, a3, b0, b1, b2, b3, f0, f1, f2, f3;
    int ai, bv, fp;
    uint32_t lb;
    int32_t budget;   // 8 * (bytes from the substream start to the picture's RBSP end) - bits moved into value
    uint32_t status;
    int st;
    uint32_t fl;
    int row, c, ctbx, ctby;
    // coding quadtree / transform tree node
    int qx, qy, ql, qd;
    int tx, ty, tl, td;
    uint32_t tcbf;  // cbf_cb | cbf_cr << 1 (| the 4:2:2 lower TBs' << 2, << 3) of the node at depth d, at bit 4d
    // quantization (8.6.1)
    int qp_prev_last, qp_pred, cu_qp_delta_val, qpy_cur, qg_x, qg_y;
    // coding unit: IntraPredModeY of PB k in byte k, IntraPredModeC
    int cu_modes, cu_chroma;
    // transform block
    int tb_t, tb_n, tb_cidx, tb_x, tb_y, tb_log2, tb_mode;
    uint32_t tb_coef0;
    // residual_coding state carried across sub-blocks
    int rc_scan, rc_last_sub, rc_last_pos, rc_i, rc_prev_c1;
    uint64_t rc_csbf;  // coded_sub_block_flag, bit yS * 8 + xS
    uint32_t ntu, ncoef;
    uint32_t nesc;              // escape levels of the row (stored down from the end of its coefficient space)
    uint32_t tu_row, coef_row;  // TuRec / Coef index of the current row's outputs
    // solo mode on the GPU: the context states, byte i of the LDS layout at
    // byte i & 3 of lane i >> 2 (35 lanes), read / written with v_readlane /
    // v_writelane; the one field whose lanes differ
    uint32_t cx;
    uint32_t reinit;  // F_REINIT: RBSP byte (absolute) where the engine restarts after PCM samples
#if defined(HG_PARSE_PROF_SB)
    // solo tuning build: s_memtime cycles of unit_sb's phases (header, sig loop,
    // greater1/2, signs + levels + coefficient stores) and sig bins / coefficients
    uint64_t psb[6];
#endif
};
#if defined(HG_PARSE_PROF_SB) && !defined(HG_HOST_EMU)
// (the lowest active lane accumulates: in the lanes kernel the lanes running
// the unit share one timeline, so the psb sums over lanes are the wave's time)
#define HG_SB_T(L, i, t0)                                                            \
    do {                                                                             \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                            \
        if ((int)__lane_id() == __builtin_ctzll(__ballot(1))) (L).psb[i] += t_ - (t0); \
        (t0) = t_;                                                                   \
    } while (0)
#else
#define HG_SB_T(L, i, t0) ((void)0)
#endif

// bytes of n lane blocks, rounded up so the LanePic after them stays 16-byte aligned
HG_HD inline size_t lane_blocks_bytes(int n) { return (sizeof(LaneLds) * (size_t)n + 15) & ~(size_t)15; }

// engine context of one lane (lanes mode: every lane its own substream; a
// picture's WPP rows are lanes of one wave, so no hand-off leaves the wave).
// (r05's row waves, k_parse_rows, were this engine with spread mode's
// hand-offs; removed in r06, their A/B record is DESIGN 5.4)
struct Eng {
    static constexpr bool kSolo = false;
    static constexpr bool kSpread = false;
    static constexpr bool kCtxReg = false;  // contexts in LDS (ctx)
    static constexpr bool kRowCtx = true;
    uint8_t *ctx;
    const uint64_t *tab;  // engine_row of every context byte (LDS)
    const uint64_t *seq;  // sig_seq(scan, pattern): slot of every scan position of a sub-block (LDS)
    const uint8_t *rbsp;  // BatchArgs::rbsp (emulation prevention removed by k_rbsp)
    uint32_t lim;         // no loads at or past this offset (the picture's RBSP end + 64)
    // the 8x8 up-right diagonal scan of 32x32 TBs' sub-blocks and its inverse in
    // LDS (null: the constant tables).  A lane-varying index into constant memory
    // is a vector load, and its wait would drain the wave's record stores too
    const uint8_t *sp8 = nullptr, *inv8 = nullptr;
    HG_HD uint64_t row(uint32_t st) const { return tab[st]; }
    HG_HD uint64_t seqw(int idx) const { return seq[idx]; }
    HG_HD int scan8(int scan, int i) const { return sp8 && scan == 0 ? sp8[i] : kScanPos[3][scan][i]; }
    HG_HD int scan8_inv(int scan, int r) const { return inv8 && scan == 0 ? inv8[r] : kScanInv[3][scan][r]; }
};

// Solo mode (k_parse_solo): one substream per WAVE, run by its lane 0 alone,
// so the engine state is wave-uniform.  The state rows live in two VGPRs
// across the lanes (lane s = pStateIdx s) and are read with v_readlane, and
// the RBSP comes from a 512-byte window in two VGPRs (dword d of the arena at
// lane d % 64 of register (d / 64) % 2), filled between units by whole-wave
// coalesced 256-byte loads through a staging VGPR: a chunk is loaded one
// chunk ahead of use and copied into the window (the copy is where the
// compiler waits for it) only when the reader enters the chunk before it, so
// a bin never waits on LDS for its state row and a refill almost never waits
// on memory.
#if defined(HG_HOST_EMU)
struct Win {
    const uint32_t *w;  // [2 * 64]
    uint32_t get(uint32_t d) const { return w[d & 127u]; }
};
#else
struct Win {
    uint32_t r0, r1;
    // both registers read and the result selected: a select of the register
    // (or of its address) becomes a dynamically indexed array in scratch
    __device__ __forceinline__ uint32_t get(uint32_t d) const {
        const int ln = __builtin_amdgcn_readfirstlane((int)(d & 63u));
        const uint32_t v0 = (uint32_t)__builtin_amdgcn_readlane((int)r0, ln);
        const uint32_t v1 = (uint32_t)__builtin_amdgcn_readlane((int)r1, ln);
        return (d & 64u) ? v1 : v0;
    }
};
#endif
template <bool Spread>
struct EngSoloT {
    static constexpr bool kSolo = true;
    static constexpr bool kRowCtx = false;  // rows per pStateIdx (tlo / thi)
    // one wave per workgroup: the rows of a picture on different CUs, their
    // WPP progress, context hand-off, SAO and depth lines in coherent global
    // memory.  Rule: hand-off data goes out only through store_agent, so the
    // progress word needs vmcnt(0) only, not an L2 write-back (unit_ctu_end)
    static constexpr bool kSpread = Spread;
#if defined(HG_HOST_EMU)
    static constexpr bool kCtxReg = false;  // one lane per wave: contexts stay in the LDS block
#else
    static constexpr bool kCtxReg = true;   // contexts in Lane::cx
#endif
    uint8_t *ctx;
    uint32_t tlo, thi;    // lane s: state_row(s) (GPU); unused under emulation
    const uint64_t *seq;  // (emulation; the GPU reads sqlo / sqhi)
    const uint8_t *rbsp;
    uint32_t lim;
    Win win;
    // lane i < 15: sig_seq(i).  Read from LDS (`seq`) by default: the
    // v_readlane form (HG_SOLO_SEQ_VGPR) measured 26.7 against 25.7 ms for
    // one image (r05 same-box A/B, profiles/r05/ab/b1_engine_variants.txt);
    // the two builds differ mostly in where the register allocator put its
    // SGPR spills (89 here against 138)
    uint32_t sqlo, sqhi;
    // lane i: kScanPos[3][0][i] | kScanInv[3][0][i] << 8 (a byte of constant memory
    // is a vector load even at a uniform index: v_readlane instead)
    uint32_t scan8v;
#if defined(HG_HOST_EMU)
    int scan8(int scan, int i) const { return kScanPos[3][scan][i]; }
    int scan8_inv(int scan, int r) const { return kScanInv[3][scan][r]; }
#else
    __device__ __forceinline__ int scan8(int scan, int i) const {
#if defined(HG_NO_SCAN8)  // A/B only: the constant tables
        return kScanPos[3][scan][i];
#endif
        if (scan != 0) return kScanPos[3][scan][i];
        return __builtin_amdgcn_readlane((int)scan8v, __builtin_amdgcn_readfirstlane(i)) & 0xff;
    }
    __device__ __forceinline__ int scan8_inv(int scan, int r) const {
#if defined(HG_NO_SCAN8)
        return kScanInv[3][scan][r];
#endif
        if (scan != 0) return kScanInv[3][scan][r];
        return (__builtin_amdgcn_readlane((int)scan8v, __builtin_amdgcn_readfirstlane(r)) >> 8) & 0xff;
    }
#endif
#if defined(HG_HOST_EMU)
    uint64_t row(uint32_t st) const { return state_row((int)st); }
    uint64_t seqw(int idx) const { return seq[idx]; }
#else
    __device__ __forceinline__ uint64_t seqw(int idx) const {
#if !defined(HG_SOLO_SEQ_VGPR)
        return seq[idx];
#endif
        const int i = __builtin_amdgcn_readfirstlane(idx);
        return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)sqlo, i) |
               ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)sqhi, i) << 32);
    }
    __device__ __forceinline__ uint64_t row(uint32_t st) const {
        const int s = __builtin_amdgcn_readfirstlane((int)st);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)tlo, s);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)thi, s);
        return (uint64_t)lo | ((uint64_t)hi << 32);
    }
#endif
};
using EngSolo = EngSoloT<false>;
using EngSpread = EngSoloT<true>;

#if !defined(HG_HOST_EMU)
// Solo mode: the wave's substream state is equal in every lane; say so to the
// compiler (v_readfirstlane), so the units keep it in SGPRs and branch on it
// with s_cbranch instead of exec masks.
__device__ __forceinline__ uint32_t uni32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int uni32(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    return (uint64_t)uni32((uint32_t)v) | ((uint64_t)uni32((uint32_t)(v >> 32)) << 32);
}
[[maybe_unused]] __device__ __forceinline__ void uni_state(Lane &L) {
#define HG_U(f) L.f = uni32(L.f)
#if defined(HG_SOLO_UNI_ALL)  // A/B only: r04's list, every field (134 SGPRs spilled into VGPR lanes)
    HG_U(range); HG_U(value); HG_U(k); HG_U(cn); HG_U(lb); HG_U(budget); HG_U(status); HG_U(st); HG_U(fl);
    HG_U(row); HG_U(c); HG_U(ctbx); HG_U(ctby); HG_U(qx); HG_U(qy); HG_U(ql); HG_U(qd); HG_U(tx); HG_U(ty);
    HG_U(tl); HG_U(td); HG_U(tcbf); HG_U(qp_prev_last); HG_U(qp_pred); HG_U(cu_qp_delta_val); HG_U(qpy_cur);
    HG_U(qg_x); HG_U(qg_y); HG_U(cu_modes); HG_U(cu_chroma); HG_U(tb_t); HG_U(tb_n); HG_U(tb_cidx); HG_U(tb_x);
    HG_U(tb_y); HG_U(tb_log2); HG_U(tb_mode); HG_U(tb_coef0); HG_U(rc_scan); HG_U(rc_last_sub); HG_U(rc_last_pos);
    HG_U(rc_i); HG_U(rc_prev_c1); HG_U(ntu); HG_U(ncoef); HG_U(nesc); HG_U(tu_row); HG_U(coef_row);
#elif defined(HG_SOLO_UNI_TB)  // A/B: the default set and the TB unit's fields
    HG_U(range); HG_U(value); HG_U(k); HG_U(cn); HG_U(lb); HG_U(budget); HG_U(st); HG_U(fl);
    HG_U(qx); HG_U(qy); HG_U(ql); HG_U(qd); HG_U(tx); HG_U(ty); HG_U(tl); HG_U(td); HG_U(tcbf);
    HG_U(ctbx); HG_U(ctby); HG_U(tb_log2); HG_U(tb_cidx); HG_U(rc_i); HG_U(rc_scan); HG_U(rc_last_sub);
    HG_U(rc_last_pos); HG_U(rc_prev_c1); HG_U(tb_t); HG_U(tb_n); HG_U(tb_mode); HG_U(tb_x); HG_U(tb_y);
#elif defined(HG_SOLO_UNI_LEAN)  // A/B: the default set without the tree positions
    HG_U(range); HG_U(value); HG_U(k); HG_U(cn); HG_U(lb); HG_U(budget); HG_U(st); HG_U(fl);
    HG_U(ql); HG_U(qd); HG_U(tl); HG_U(td); HG_U(tcbf);
    HG_U(tb_log2); HG_U(tb_cidx); HG_U(rc_i); HG_U(rc_scan); HG_U(rc_last_sub); HG_U(rc_last_pos); HG_U(rc_prev_c1);
#else
    // the engine and the tree / residual state the units branch on; the other
    // fields stay in VGPRs (all 64 lanes alike) and are read where used.  r05
    // A/B, one image, same box: 27.2 ms against 28.1 with every field scalar
    // (r04; that list left 134 SGPRs spilled into VGPR lanes, reloaded at
    // every unit) and 29.5 with the engine alone (profiles/r05/ab/b1_engine_select_uni.txt)
    HG_U(range); HG_U(value); HG_U(k); HG_U(cn); HG_U(lb); HG_U(budget); HG_U(st); HG_U(fl);
    HG_U(qx); HG_U(qy); HG_U(ql); HG_U(qd); HG_U(tx); HG_U(ty); HG_U(tl); HG_U(td); HG_U(tcbf);
    HG_U(ctbx); HG_U(ctby); HG_U(tb_log2); HG_U(tb_cidx); HG_U(rc_i); HG_U(rc_scan); HG_U(rc_last_sub);
    HG_U(rc_last_pos); HG_U(rc_prev_c1);
#endif
#undef HG_U
    L.cur = uni64(L.cur);
    L.rc_csbf = uni64(L.rc_csbf);
}
#endif

#if !defined(HG_SOLO_SLEEP)
#define HG_SOLO_SLEEP 1
#endif

// driver side of a solo wave's RBSP window: chunks (64 dwords, 256 bytes) c
// and c + 1 of the reader in the window, c + 2 staged (in flight)
struct SoloWin {
#if defined(HG_HOST_EMU)
    uint32_t *w, *f;  // [128], [64]
    void load(const uint8_t *rbsp, uint32_t chunk, uint32_t lim, int) {
        for (int l = 0; l < 64; ++l) {  // big-endian words (as the GPU window holds them)
            const uint32_t o = std::min((chunk * 64u + (uint32_t)l) * 4u, lim);
            f[l] = ((uint32_t)rbsp[o] << 24) | ((uint32_t)rbsp[o + 1] << 16) | ((uint32_t)rbsp[o + 2] << 8) |
                   (uint32_t)rbsp[o + 3];
        }
    }
    void commit(uint32_t chunk) {
        for (int l = 0; l < 64; ++l) w[(chunk & 1u) * 64u + (uint32_t)l] = f[l];
    }
    Win view() const { return Win{w}; }
#else
    uint32_t r0, r1, f;
    // every lane loads its dword of the chunk (one coalesced 256-byte load)
    __device__ __forceinline__ void load(const uint8_t *rbsp, uint32_t chunk, uint32_t lim, int lane) {
        const uint32_t o = (chunk * 64u + (uint32_t)lane) * 4u;
        f = *reinterpret_cast<const uint32_t *>(rbsp + (o < lim ? o : lim));
    }
    // the copy is the first use of the staged load: the compiler waits for it
    // here.  The window holds big-endian words (byte-swapped once per dword, by
    // the lanes in parallel), so the engine's bit refill is scalar shifts only
    __device__ __forceinline__ void commit(uint32_t chunk) {
        const bool odd = (chunk & 1u) != 0;  // both written: no address select
        const uint32_t be = __builtin_bswap32(f);
        r1 = odd ? be : r1;
        r0 = odd ? r0 : be;
    }
    __device__ __forceinline__ Win view() const { return Win{r0, r1}; }
#endif
    uint32_t ck;  // the staged chunk
    // a substream (re)starts at byte `start`
    HG_HD void restart(const uint8_t *rbsp, uint32_t start, uint32_t lim, int lane) {
        const uint32_t c0 = start >> 8;
        load(rbsp, c0, lim, lane);
        commit(c0);
        load(rbsp, c0 + 1, lim, lane);
        commit(c0 + 1);
        load(rbsp, c0 + 2, lim, lane);
        ck = c0 + 2;
    }
    // before a unit, the reader at dword rd: keep its chunk and the next in the window
    HG_HD void advance(const uint8_t *rbsp, uint32_t rd, uint32_t lim, int lane) {
        const uint32_t cc = rd >> 6;
        if (cc + 1 < ck) return;
        if (cc >= ck) {  // a unit ran past the window (corrupt stream): reload
            restart(rbsp, cc << 8, lim, lane);
            return;
        }
        commit(ck);
        load(rbsp, ck + 1, lim, lane);
        ++ck;
    }
};

// ------------------------------------------------------------------ memory helpers
#if defined(HG_HOST_EMU)
inline uint32_t prog_load(const uint32_t *p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline void prog_store(uint32_t *p, uint32_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
inline uint32_t load_word_coherent(const uint32_t *p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline void release_fence() { std::atomic_thread_fence(std::memory_order_release); }
inline void store_tu(TuRec *d, uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
    uint32_t *p = reinterpret_cast<uint32_t *>(d);
    p[0] = x;
    p[1] = y;
    p[2] = z;
    p[3] = w;
}
inline void store_tu_agent(TuRec *d, uint32_t x, uint32_t y, uint32_t z, uint32_t w) { store_tu(d, x, y, z, w); }
inline void store_word_agent(uint32_t *p, uint32_t v) { *p = v; }
#else
__device__ __forceinline__ uint32_t prog_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
__device__ __forceinline__ void prog_store(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
// 4-byte load that bypasses the L1: the word was written by another lane of
// this wave (same CU, so the L2 of this XCD has it)
__device__ __forceinline__ uint32_t load_word_coherent(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// drain this wave's global stores (SAO parameters, depth line) before the
// progress word that lets the lane below read them
__device__ __forceinline__ void release_fence() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); }
__device__ __forceinline__ void store_tu(TuRec *d, uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
    *reinterpret_cast<uint4 *>(d) = make_uint4(x, y, z, w);
}
// the same as agent-scope (sc1) stores: coherent across the XCDs' L2s once
// complete, so the spread parse publishes them with a wait, not an L2 write-back
__device__ __forceinline__ void store_tu_agent(TuRec *d, uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
    uint64_t *q = reinterpret_cast<uint64_t *>(d);
    __hip_atomic_store(q, (uint64_t)x | ((uint64_t)y << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, (uint64_t)z | ((uint64_t)w << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_word_agent(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#endif

// n bytes of v at p (v's 8-byte pattern repeats for n > 8: a 64x64 CU's
// 16-byte QpY row): one store when n is 2, 4 or 8 and p is n-aligned
HG_HD inline void store_bytes(uint8_t *p, int n, uint64_t v) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    if (n == 8 && !(a & 7)) {
        *reinterpret_cast<uint64_t *>(p) = v;
    } else if (n == 4 && !(a & 3)) {
        *reinterpret_cast<uint32_t *>(p) = (uint32_t)v;
    } else if (n == 2 && !(a & 1)) {
        *reinterpret_cast<uint16_t *>(p) = (uint16_t)v;
    } else {
        for (int i = 0; i < n; ++i) p[i] = (uint8_t)(v >> (8 * (i & 7)));
    }
}

// Spread mode: words another CU reads (agent-scope atomics: sc1 accesses,
// coherent across the XCDs' L2s without whole-cache write-backs), and the
// wait that makes this wave's earlier such stores visible before a progress word
#if defined(HG_HOST_EMU)
template <class T>
inline void store_agent(T *p, T v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
inline uint32_t load_agent(const uint32_t *p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline void stores_done() { std::atomic_thread_fence(std::memory_order_release); }
#else
template <class T>
__device__ __forceinline__ void store_agent(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t load_agent(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// s_waitcnt vmcnt(0): every store of this wave has completed
__device__ __forceinline__ void stores_done() { __builtin_amdgcn_s_waitcnt(0x0f70); }
#endif

HG_HD inline uint8_t load_byte_coherent(const uint8_t *p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t w = load_word_coherent(reinterpret_cast<const uint32_t *>(a & ~uintptr_t(3)));
    return (uint8_t)(w >> ((a & 3) * 8));
}

// ------------------------------------------------------------------ bytes
// Each lane reads its substream straight from the RBSP arena, which k_rbsp
// (rbsp.hip) filled with emulation prevention removed (rbsp_reader.rs:11-39).
// The bit window refills from a per-lane queue of up to 8 dwords in registers;
// 16 more bytes are loaded at each pass start and used from the next pass on,
// after the pass's single s_waitcnt, so no refill inside a pass waits on
// memory (a wait for a load also drains every older store of the wave: with a
// one-dword prefetch it cost ~5 % of the parse).  Loads stop 64 bytes past
// the picture's end (arena padding); an overrun of a corrupt stream shows as
// budget + k < 0 at the CTU end (ST_OVERRUN).
// 16 bytes at `off` (dword aligned), clamped to `lim` (inside the arena's padding)
#if defined(HG_HOST_EMU)
inline void load_x4(const uint8_t *p, uint32_t off, uint32_t lim, uint32_t &x, uint32_t &y, uint32_t &z, uint32_t &w) {
    uint32_t v[4];
    for (int i = 0; i < 4; ++i) {
        const uint32_t o = std::min(off + 4u * (uint32_t)i, lim);
        v[i] = (uint32_t)p[o] | ((uint32_t)p[o + 1] << 8) | ((uint32_t)p[o + 2] << 16) | ((uint32_t)p[o + 3] << 24);
    }
    x = v[0], y = v[1], z = v[2], w = v[3];
}
// the pass start's one memory wait (host emulation: nothing in flight)
inline void pass_wait() {}
#else
__device__ __forceinline__ void load_x4(const uint8_t *p, uint32_t off, uint32_t lim, uint32_t &x, uint32_t &y,
                                        uint32_t &z, uint32_t &w) {
    const uint4 v = *reinterpret_cast<const uint4 *>(p + (off < lim ? off : lim));
    x = v.x, y = v.y, z = v.z, w = v.w;
}
// s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15): every global access of this wave so far
__device__ __forceinline__ void pass_wait() { __builtin_amdgcn_s_waitcnt(0x0f70); }
#endif
HG_HD inline uint32_t bswap32(uint32_t w) {
    return (w >> 24) | ((w >> 8) & 0xff00u) | ((w << 8) & 0xff0000u) | (w << 24);
}

// next RBSP dword of the queue.  Normally a or b; a lane that drained both
// inside one pass takes f (waiting for it) or loads synchronously.  Solo
// mode: dword L.lb of the register window (filled between units), already
// big-endian (be_pop).
template <class EG>
HG_HD inline uint32_t q_pop(Lane &L, const EG &G) {
    if constexpr (EG::kSolo) return G.win.get(L.lb++);
#if !defined(HG_HOST_EMU) && defined(__HIP_DEVICE_COMPILE__)
    // the dword at index ai as three v_cndmask.  Written in C++ the selection
    // compiles to nested exec-mask branches (a dozen SALU instructions at every
    // refill site), and as bit tests into a dynamically indexed scratch array;
    // r05 A/B at 128 images: 19,490 against 19,200 (branches) and 17,520
    // (scratch) Mpix/s; 17 % fewer static instructions in k_parse_lanes
    uint32_t w;
    asm("v_cmp_eq_u32 vcc, 1, %1\n\t"
        "v_cndmask_b32 %0, %2, %3, vcc\n\t"
        "v_cmp_eq_u32 vcc, 2, %1\n\t"
        "v_cndmask_b32 %0, %0, %4, vcc\n\t"
        "v_cmp_eq_u32 vcc, 3, %1\n\t"
        "v_cndmask_b32 %0, %0, %5, vcc"
        : "=&v"(w)
        : "v"(L.ai), "v"(L.a0), "v"(L.a1), "v"(L.a2), "v"(L.a3)
        : "vcc");
#else
    const uint32_t w = L.ai == 0 ? L.a0 : (L.ai == 1 ? L.a1 : (L.ai == 2 ? L.a2 : L.a3));
#endif
    if (++L.ai == 4) {
        L.ai = 0;
        if (L.bv) {
            L.a0 = L.b0, L.a1 = L.b1, L.a2 = L.b2, L.a3 = L.b3;
            L.bv = 0;
        } else if (L.fp) {
            L.a0 = L.f0, L.a1 = L.f1, L.a2 = L.f2, L.a3 = L.f3;
            L.fp = 0;
        } else {
            load_x4(G.rbsp, L.lb, G.lim, L.a0, L.a1, L.a2, L.a3);
            L.lb += 16;
        }
    }
    return w;
}

// the next 32 bits of the substream, MSB first
template <class EG>
HG_HD inline uint32_t be_pop(Lane &L, const EG &G) {
    if constexpr (EG::kSolo) return q_pop(L, G);
    return bswap32(q_pop(L, G));
}

// pass start (after pass_wait): land f, issue the next block
template <class EG>
HG_HD inline void q_refill(Lane &L, const EG &G) {
    if (L.fp && !L.bv) {
        L.b0 = L.f0, L.b1 = L.f1, L.b2 = L.f2, L.b3 = L.f3;
        L.bv = 1;
        L.fp = 0;
    }
    if (!L.fp && L.lb) {
        load_x4(G.rbsp, L.lb, G.lim, L.f0, L.f1, L.f2, L.f3);
        L.lb += 16;
        L.fp = 1;
    }
#if !defined(HG_NO_TOPUP)
    // top the bit window up to more than 32 bits once per pass, so that inside
    // the pass vfill's pop (the queue select and its reload branches, run by
    // the whole wave whenever one lane needs it) is rarely reached
    if (L.cn <= 32) {
        L.cur |= (uint64_t)be_pop(L, G) << (32 - L.cn);
        L.cn += 32;
    }
#endif
}

// value += 16 more look-ahead bits (k < 8 on entry, so k <= 23 and value < 2^32 after).
// (A/B r03: comparisons as sign masks with k <= 22 and v_bfi selects instead
// of compares into VCC: parse 94 vs 91 ms at 128 images, 37.9 vs 36.1 ms for
// one image in spread mode — the compares stay.)
template <class EG>
HG_HD inline void vfill(Lane &L, const EG &G) {
    if (L.cn < 16) {
        L.cur |= (uint64_t)be_pop(L, G) << (32 - L.cn);
        L.cn += 32;
    }
#if !defined(HG_HOST_EMU) && defined(__HIP_DEVICE_COMPILE__)
    if constexpr (EG::kSolo) {
        // scalar: the compiler turns this into a funnel shift, which only the VALU has
        const uint32_t top = (uint32_t)(L.cur >> 48);
        uint32_t nv;
        asm("s_lshl_b32 %0, %1, 16\n\ts_or_b32 %0, %0, %2" : "=&s"(nv) : "s"(uni32(L.value)), "s"(uni32(top)) : "scc");
        L.value = nv;
    } else
#endif
    {
        L.value = (L.value << 16) | (uint32_t)(L.cur >> 48);
    }
    L.cur <<= 16;
    L.cn -= 16;
    L.k += 16;
    L.budget -= 16;
}

// 9.3.2.5: engine initialisation at RBSP offset `start` (absolute), picture RBSP end `end`
// (solo mode: the driver has filled the window from `start` on)
template <class EG>
HG_HD inline void engine_init(Lane &L, const EG &G, uint32_t start, uint32_t end) {
    const uint32_t a0 = start & ~3u, sh = (start & 3u) * 8u;
    if constexpr (EG::kSolo) {
        L.lb = a0 >> 2;
    } else {
        load_x4(G.rbsp, a0, G.lim, L.a0, L.a1, L.a2, L.a3);
        load_x4(G.rbsp, a0 + 16, G.lim, L.b0, L.b1, L.b2, L.b3);
        L.ai = 0;
        L.bv = 1;
        L.fp = 0;
        L.lb = a0 + 32;
    }
    L.cur = (uint64_t)be_pop(L, G) << (32 + sh);
    L.cn = 32 - (int)sh;
    L.budget = 8 * (int32_t)(end - start);
    L.value = 0;
    L.k = -9;  // the first 9 bits are ivlOffset itself
    vfill(L, G);
    vfill(L, G);
    L.range = 510;
    if ((L.value >> L.k) >= 510) {
        // ivlOffset 510 / 511 (9.3.2.5 forbids it): flagged, and clamped so that
        // value < range << k holds and every later bin stays in range (a bypass
        // run of n bins < 2^n, so no syntax element leaves its domain)
        L.status |= ST_CABAC_INIT;
        L.value = (509u << L.k) | ((1u << L.k) - 1u);
    }
}

// ------------------------------------------------------------------ engine (9.3.4.3)
// DecodeDecision (arithmetic.rs:97-144), branch-free: one row per pStateIdx
// gives rangeTabLps and both transitions; the renormalisation of either path
// is a shift by clz and lowers k.
// (a & m) | (b & ~m) as one v_bfi_b32: written as C the compiler re-masks the
// inserted value first (a bit-field extract of the row, then the OR)
HG_HD inline uint32_t bfi32(uint32_t m, uint32_t a, uint32_t b) {
#if !defined(HG_HOST_EMU) && defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
#else
    return (a & m) | (b & ~m);
#endif
}

// (vector engines, state_row_ctx) a decision on context byte s; t receives
// the new byte in bits 0-6 and the bin in bit 7, bits above are not cleared
template <class EG>
HG_HD inline int dec_t(Lane &L, const EG &G, uint32_t s, uint32_t &t) {
    const uint64_t row = G.row(s);
    const uint32_t lps = ((uint32_t)row >> ((L.range >> 3) & 24u)) & 0xffu;
    const uint32_t rm = L.range - lps;
    const uint32_t sr = rm << L.k;
    const bool isl = L.value >= sr;
    L.value -= isl ? sr : 0u;
    const uint32_t rn = isl ? lps : rm;
    const int nb = __builtin_clz(rn) - 23;
    L.range = rn << nb;
    L.k -= nb;
    t = (uint32_t)(row >> (isl ? 32 : 40));
    if (L.k < 8) vfill(L, G);
    return (int)((t >> 7) & 1u);
}

template <class EG>
HG_HD inline int dec_s(Lane &L, const EG &G, uint32_t &s) {
    if constexpr (EG::kRowCtx) {
        uint32_t t;
        const int bin = dec_t(L, G, s, t);
        s = t & 0x7fu;
        return bin;
    }
    const uint32_t st = s >> 1, mps = s & 1u;
    const uint64_t row = G.row(st);
    const uint32_t hi = (uint32_t)(row >> 32);  // next byte after an LPS | after an MPS << 8
    const uint32_t lps = ((uint32_t)row >> ((L.range >> 3) & 24u)) & 0xffu;
    const uint32_t rm = L.range - lps;
    const uint32_t sr = rm << L.k;
#if !defined(HG_HOST_EMU) && defined(__HIP_DEVICE_COMPILE__)
    if constexpr (EG::kSolo) {
        // scalar engine: the LPS test as an integer straight from SCC (as a
        // boolean the compiler carries a lane mask and rebuilds the bin
        // through a VALU select and v_readfirstlane), then mask arithmetic.
        // (uni32: the lanes are identical, but where the compiler cannot
        // prove it, e.g. at engine start, the operands must be made scalar)
#if defined(HG_SOLO_OLD_SELECT)  // A/B only: the r04 form (the bin from SCC, then mask arithmetic)
        uint32_t lp;
        asm("s_cmp_ge_u32 %1, %2\n\ts_cselect_b32 %0, 1, 0" : "=s"(lp) : "s"(uni32(L.value)), "s"(uni32(sr)) : "scc");
        const uint32_t m = 0u - lp;
        s = ((hi >> (8u & ~m)) & 0xffu) ^ mps;
        L.value -= sr & m;
        const uint32_t rn = (lps & m) | (rm & ~m);
        const int nb = __builtin_clz(rn) - 23;
#else
        // one compare, every choice an s_cselect on its SCC: the bin, the new
        // range, what leaves the offset and the shift that picks the next state
        uint32_t lp, rn, d, sh;
        asm("s_cmp_ge_u32 %4, %5\n\t"
            "s_cselect_b32 %0, 1, 0\n\t"
            "s_cselect_b32 %1, %6, %7\n\t"
            "s_cselect_b32 %2, %5, 0\n\t"
            "s_cselect_b32 %3, 0, 8"
            : "=&s"(lp), "=&s"(rn), "=&s"(d), "=&s"(sh)
            : "s"(uni32(L.value)), "s"(uni32(sr)), "s"(uni32(lps)), "s"(uni32(rm))
            : "scc");
        s = ((hi >> sh) & 0xffu) ^ mps;
        L.value -= d;
        const int nb = __builtin_clz(rn) - 23;
#endif
        L.range = rn << nb;
        L.k -= nb;
        if (L.k < 8) vfill(L, G);
        return (int)(mps ^ lp);
    }
#endif
    const bool isl = L.value >= sr;
    L.value -= isl ? sr : 0u;
    const uint32_t rn = isl ? lps : rm;
    const int nb = __builtin_clz(rn) - 23;
    L.range = rn << nb;
    L.k -= nb;
    s = ((hi >> (isl ? 0 : 8)) & 0xffu) ^ mps;
    if (L.k < 8) vfill(L, G);
    return (int)(mps ^ (isl ? 1u : 0u));
}

// context state ci: a byte of the LDS block, or (solo on the GPU) of Lane::cx
template <class EG>
HG_HD inline uint32_t ctx_ld(const Lane &L, const EG &G, int ci) {
#if !defined(HG_HOST_EMU)
    if constexpr (EG::kCtxReg) {
        const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)L.cx, ci >> 2);
        return (w >> ((ci & 3) * 8)) & 0xffu;
    }
#endif
    return G.ctx[ci];
}
template <class EG>
HG_HD inline void ctx_st(Lane &L, const EG &G, int ci, uint32_t v) {
#if !defined(HG_HOST_EMU)
    if constexpr (EG::kCtxReg) {
        const int sh = (ci & 3) * 8;
        const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)L.cx, ci >> 2);
        L.cx = (uint32_t)hg_writelane((int)((w & ~(0xffu << sh)) | (v << sh)), ci >> 2, (int)L.cx);
        return;
    }
#endif
    G.ctx[ci] = (uint8_t)v;
}

// the same on context ci
template <class EG>
HG_HD inline int dec(Lane &L, const EG &G, int ci) {
#if !defined(HG_HOST_EMU)
    if constexpr (EG::kCtxReg) {  // one v_readlane serves the read and the write back
        const int sh = (ci & 3) * 8;
        const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)L.cx, ci >> 2);
        uint32_t s = (w >> sh) & 0xffu;
        const int bin = dec_s(L, G, s);
        L.cx = (uint32_t)hg_writelane((int)((w & ~(0xffu << sh)) | (s << sh)), ci >> 2, (int)L.cx);
        return bin;
    }
#endif
    uint32_t s = G.ctx[ci];
    const int bin = dec_s(L, G, s);
    G.ctx[ci] = (uint8_t)s;
    return bin;
}

// A/B switch (HG_SB_GENERIC): the 9-slot sig_coeff_flag loop for every TB size
[[maybe_unused]] HG_HD constexpr bool sb_generic_loop() {
#if defined(HG_SB_GENERIC)
    return true;
#else
    return false;
#endif
}

// byte `slot` (0..11) of a 3-word register cache of context states
HG_HD inline uint32_t cache_get(uint32_t c0, uint32_t c1, uint32_t c2, int slot) {
    const uint32_t w = slot < 4 ? c0 : (slot < 8 ? c1 : c2);
    return (w >> ((slot & 3) * 8)) & 0xffu;
}
HG_HD inline void cache_put(uint32_t &c0, uint32_t &c1, uint32_t &c2, int slot, uint32_t s) {
    const int sh = (slot & 3) * 8;
    const uint32_t w = slot < 4 ? c0 : (slot < 8 ? c1 : c2);
    const uint32_t nw = (w & ~(0xffu << sh)) | (s << sh);
    c0 = slot < 4 ? nw : c0;
    c1 = (slot >> 2) == 1 ? nw : c1;
    c2 = slot >= 8 ? nw : c2;
}

// DecodeBypass (arithmetic.rs:146-157)
template <class EG>
HG_HD inline int byp(Lane &L, const EG &G) {
    L.k -= 1;
    const uint32_t sr = L.range << L.k;
    const bool one = L.value >= sr;
    L.value -= one ? sr : 0u;
    if (L.k < 8) vfill(L, G);
    return one ? 1 : 0;
}

// floor(top / r) for top < 2^24 and 256 <= r <= 510: f32 reciprocal estimate, then one correction
HG_HD inline uint32_t div_range(uint32_t top, uint32_t r) {
#if defined(HG_HOST_EMU)
    return top / r;
#else
    const uint32_t q = (uint32_t)((float)top * __builtin_amdgcn_rcpf((float)r));
    const int32_t rem = (int32_t)top - (int32_t)(q * r);
    // the correction as sign bits (|rem| < 2r): compares and selects here become
    // a lane-mask boolean that the scalar engine rebuilds through the VALU
    return q + ((uint32_t)((int32_t)r - 1 - rem) >> 31) - ((uint32_t)rem >> 31);
#endif
}

// n (0..8) bypass bins in one step.  n successive DecodeBypass steps are the
// long division of ivlOffset * 2^n + (the next n bits) by ivlCurrRange: the
// quotient is the n bins, the remainder the new ivlOffset.
template <class EG>
HG_HD inline uint32_t byp_n(Lane &L, const EG &G, int n) {
    L.k -= n;  // k >= 8 >= n on entry
    const uint32_t q = div_range(L.value >> L.k, L.range);
    L.value -= (q * L.range) << L.k;
    if (L.k < 8) vfill(L, G);
    return q;
}

template <class EG>
HG_HD inline uint32_t byp_bits(Lane &L, const EG &G, int n) {
    uint32_t v = 0;
    while (n > 0) {
        const int c = n < 8 ? n : 8;
        v = (v << c) | byp_n(L, G, c);
        n -= c;
    }
    return v;
}

// coeff_abs_level_remaining's non-escape part (decoder.rs:230-261: prefix
// TR(cMax 4 << k, k), i.e. up to 4 one-bins, a 0, then k suffix bins) in ONE
// division: the next 8 bins are divided out without consuming them, the
// prefix p is their leading ones (at most 4), and when p < 4 the whole code
// (p + 1 + k <= 8 bins) is a prefix of those 8, consumed at once (a prefix of
// a long-division quotient is the quotient of the shorter division).  Returns
// the value, or -1 after consuming the 4 ones of an escape.
template <class EG>
HG_HD inline int byp_rem(Lane &L, const EG &G, int k) {
    const uint32_t q8 = div_range(L.value >> (L.k - 8), L.range);  // k >= 8 on entry
    const int p = __builtin_clz(((~q8) << 24) | (1u << 27));        // leading ones, at most 4
    const int used = p < 4 ? p + 1 + k : 4;
    const uint32_t q = q8 >> (8 - used);
    L.k -= used;
    L.value -= (q * L.range) << L.k;
    if (L.k < 8) vfill(L, G);
    return p < 4 ? (p << k) + (int)(q & ((1u << k) - 1u)) : -1;
}

// a unary bypass prefix of at most m (1..8) bins: the number p of 1-bins
// before the first 0, consuming min(p + 1, m) bins
template <class EG>
HG_HD inline int byp_unary(Lane &L, const EG &G, int m) {
    const uint32_t q = div_range(L.value >> (L.k - m), L.range);
    const int p = __builtin_clz(((~q) << (32 - m)) | (1u << (31 - m)));
    const int used = p < m ? p + 1 : m;
    L.k -= used;
    L.value -= ((q >> (m - used)) * L.range) << L.k;
    if (L.k < 8) vfill(L, G);
    return p;
}

// DecodeTerminate (arithmetic.rs:159-169)
template <class EG>
HG_HD inline int term(Lane &L, const EG &G) {
    L.range -= 2;
    const uint32_t sr = L.range << L.k;
    if (L.value >= sr) {
        // 1 ends the engine's run (end of a segment / subset, pcm_flag: a new
        // initialisation follows).  A corrupt stream may read on: keep
        // value < range << k, so later bins stay in their domains
        L.value = sr - 1u;
        return 1;
    }
    if (L.range < 256) {
        L.range <<= 1;
        L.k -= 1;
        if (L.k < 8) vfill(L, G);
    }
    return 0;
}

// ------------------------------------------------------------------ derivations
// Table 8-3: IntraPredModeC of 4:2:2 from the 4:2:0-style derivation, 35 modes
// packed four per word as bytes
HG_HD inline int mode422(int m) {
    constexpr uint32_t t[9] = {0x02020100u, 0x05030202u, 0x0b0a0807u, 0x12100f0du, 0x16151413u,
                               0x18181717u, 0x1b1a1919u, 0x1d1c1c1bu, 0x001f1e1du};
    return (int)((t[m >> 2] >> (8 * (m & 3))) & 0xffu);
}

HG_HD inline int chroma_qp_map(int qpi, int chroma) {
    if (chroma != 1) return qpi < 51 ? qpi : 51;
    if (qpi < 30) return qpi;
    if (qpi > 43) return qpi - 6;
    // Table 8-10 for qPi 30..43 (29 30 31 32 33 33 34 34 35 35 36 36 37 37), without a private array
    return qpi < 34 ? qpi - 1 : 33 + ((qpi - 34) >> 1);
}

HG_HD inline void update_qpy(Lane &L, const LanePic &P) {
    L.qpy_cur = ((L.qp_pred + L.cu_qp_delta_val + 52 + 2 * P.qpbdY) % (52 + P.qpbdY)) - P.qpbdY;
}

// 8.6.1 qPY_PRED of the current quantization group
HG_HD inline void derive_qp_pred(Lane &L, const LaneLds &ld, const LanePic &P) {
    int prev;
    const bool first_in_ctb = L.qg_x == L.ctbx && L.qg_y == L.ctby;
    if (L.fl & F_FIRST_QG) {
        prev = P.sliceQp;
        L.fl &= ~F_FIRST_QG;
    } else if ((L.fl & F_WPP) && first_in_ctb && L.c == 0) {
        prev = P.sliceQp;
    } else {
        prev = L.qp_prev_last;
    }
    const int mask = (1 << P.log2ctb) - 1;
    const int qa = (L.qg_x & mask) ? ld.qL[(L.qg_y - L.ctby) >> 3] : prev;
    const int qb = (L.qg_y & mask) ? ld.qA[(L.qg_x - L.ctbx) >> 3] : prev;
    L.qp_pred = (qa + qb + 1) >> 1;
}

// 8.4.2 luma intra prediction mode of the PB at (xPb, yPb)
HG_HD inline int derive_luma_mode(const Lane &L, const LaneLds &ld, int xPb, int yPb, int prev, int mpm_idx,
                                  int rem) {
    const int ca = xPb <= 0 ? 1 : ld.ipmL[(yPb - L.ctby) >> 2];
    const int cb = (yPb - 1 < L.ctby) ? 1 : ld.ipmA[(xPb - L.ctbx) >> 2];  // above CTB (or picture edge) → DC
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

// 6.5.3-6.5.5 scans.  Packed 4-bit 2x2 / 4x4 scans (entry x | (y << 2)) are
// selected, not indexed, so they stay immediates; the 8x8 sub-block scan of
// 32x32 TBs comes from the table.  scan_pos returns x | (y << 4).
HG_HD inline uint64_t scan4_word(int scan) { return scan == 0 ? kScan4Pos[0] : (scan == 1 ? kScan4Pos[1] : kScan4Pos[2]); }
template <class EG>
HG_HD inline int scan_pos(const EG &G, int l, int scan, int i) {
    if (l == 3) return G.scan8(scan, i);
    if (l == 0) return 0;
    const uint64_t t = l == 2 ? scan4_word(scan) : (scan == 0 ? kScan2Pos[0] : (scan == 1 ? kScan2Pos[1] : kScan2Pos[2]));
    const uint32_t e = (uint32_t)(t >> (4 * i)) & 15u;
    return (int)((e & 3) | ((e >> 2) << 4));
}
template <class EG>
HG_HD inline int scan_inv(const EG &G, int l, int scan, int raster) {
    if (l == 3) return G.scan8_inv(scan, raster);
    if (l == 0) return 0;
    const uint64_t t = l == 2 ? (scan == 0 ? kScan4Inv[0] : (scan == 1 ? kScan4Inv[1] : kScan4Inv[2]))
                              : (scan == 0 ? kScan2Inv[0] : (scan == 1 ? kScan2Inv[1] : kScan2Inv[2]));
    return (int)((uint32_t)(t >> (4 * raster)) & 15u);
}

// sig_coeff_flag ctxInc patterns (9.3.4.2.5) per prevCsbf, as one nibble per raster position
// e = x | (y << 2), each + 1 (slot of the sub-block's context cache)
constexpr uint64_t sig_pat_nib(int pc) {
    uint64_t w = 0;
    for (int e = 0; e < 16; ++e) {
        const int x = e & 3, y = e >> 2;
        const int v = pc == 0 ? (x + y == 0 ? 2 : (x + y < 3 ? 1 : 0))
                    : pc == 1 ? (y == 0 ? 2 : (y == 1 ? 1 : 0))
                    : pc == 2 ? (x == 0 ? 2 : (x == 1 ? 1 : 0)) : 2;
        w |= (uint64_t)(v + 1) << (4 * e);
    }
    return w;
}
HG_HD inline uint64_t sig_slots(int pcs) {
    return pcs == 0 ? sig_pat_nib(0) : pcs == 1 ? sig_pat_nib(1) : pcs == 2 ? sig_pat_nib(2) : sig_pat_nib(3);
}
HG_HD inline int msb32(uint32_t m) { return 31 - __builtin_clz(m); }

// context slot of sig_coeff_flag per scan position n of a 4x4 sub-block
// (nibble n), for scanIdx 0..2 and slot pattern 0..3 (prevCsbf, sizes > 4x4)
// or 4 (ctxIdxMap, 4x4 TBs): 15 words, computed into LDS at kernel start
HG_HD inline uint64_t sig_seq(int idx) {
    const int scan = idx / 5, pat = idx % 5;
    const uint64_t slots = pat == 4 ? kSigCtxMap4 : sig_slots(pat);
    const uint64_t sw = scan4_word(scan);
    uint64_t q = 0;
    for (int n = 0; n < 16; ++n) {
        const int e = (int)((sw >> (4 * n)) & 15u);
        q |= ((slots >> (4 * e)) & 15u) << (4 * n);
    }
    return q;
}

// the 8x8 diagonal scan of 32x32 TBs (kScanPos[3][0]) and its inverse into LDS, one entry per lane
HG_HD inline void scan8_tables(uint8_t *t, int lane) {
    t[lane] = kScanPos[3][0][lane];
    t[64 + lane] = kScanInv[3][0][lane];
}

struct Env {
    const BatchArgs *a;
    LaneLds *lds;    // the wave's 64 lane blocks
    uint32_t *prog;  // [64] row * wctb + CTUs finished in the lane's current row
    uint8_t *wctx;   // [64][CTX_PAD] WPP context staging of wrapping pictures (null when none wraps)
    int lane;
};

// WPP context staging block read at the start of substream `row` (written
// after CTU 1 of row - 1): per picture with job lanes (one block is enough:
// row r + 1 writes it only after its own start, and row r + 2 cannot start
// before that), else per row slot (lane / wave / spread row)
HG_HD inline uint8_t *wpp_stage(const Env &E, const LanePic &P, int row) {
    return E.wctx + (size_t)(P.lane0 + row % P.R) * CTX_PAD;
}
// progress word of substream `row` (monotone row * wctb + CTUs done, so a
// slot shared by rows r and r + R never runs backwards)
HG_HD inline uint32_t *prog_word(const Env &E, const LanePic &P, int row) { return &E.prog[P.lane0 + row % P.R]; }

// WPP, for parsing: a row's first CTU needs the contexts stored after CTU 1
// of the row above (9.3.1), so two CTUs of it done; CTU c > 0 only reads the
// CTU above it (split_cu_flag's CtDepth, sao_merge_up_flag; intra modes and
// QP prediction stay inside the CTB row), so one CTU ahead is enough.  The
// 2-CTU lag of the reconstruction (above-right neighbours) is k_intra's.
template <class EG>
HG_HD inline bool wpp_ready(const Lane &L, const LanePic &P, const Env &E) {
    if (!(L.fl & F_WPP) || L.row == 0) return true;
    const int ahead = L.c == 0 ? 2 : L.c + 1;
    const uint32_t need = (uint32_t)(L.row - 1) * (uint32_t)P.wctb + (uint32_t)(ahead < P.wctb ? ahead : P.wctb);
    const uint32_t *pw = prog_word(E, P, L.row - 1);
    return (EG::kSpread ? load_agent(pw) : prog_load(pw)) >= need;
}

// RBSP offset (absolute) at which a lane about to run U_CTU starts its
// substream (engine and context initialisation, unit_ctu), or ~0u
// dependent slice segments starting inside a CTB row of picture P (PicDesc.flags)
HG_HD inline uint32_t lanes_nmid(const LanePic &P) { return (P.flags >> PD_NMID_SHIFT) & PD_NMID_MAX; }

// (Mid: the lanes engine, which takes dependent segments starting inside a
// row; the scalar engines do not, parse_mode_for gives such batches the lanes parse)
template <bool Mid>
HG_HD inline uint32_t substream_start(const Lane &L, const LanePic &P, const BatchArgs &a) {
    if (L.c != 0) {
        if constexpr (Mid) {
            if (L.status & ST_SEGSW) {
                // a dependent segment starting inside the row (the picture's row
                // entries, the end entry, then these); past the picture's
                // list (a corrupt stream, flagged by unit_ctu): the RBSP end
                const uint32_t m = L.fl >> kMsegShift;
                return P.bits_off +
                       (a.rsubs[P.sub_first + (uint32_t)P.hctb + (m < lanes_nmid(P) ? 1u + m : 0u)] & SUB_OFFSET);
            }
        }
        return ~0u;
    }
    if ((L.fl & F_WPP) || L.row == 0)
        return P.bits_off + (a.rsubs[P.sub_first + ((L.fl & F_WPP) ? L.row : 0)] & SUB_OFFSET);
    if (P.flags & SP_ROW_SEGMENTS) {  // no WPP: a dependent slice segment may start at this row
        const uint32_t e = a.rsubs[P.sub_first + L.row];
        if (!(e & SUB_CONTINUE)) return P.bits_off + (e & SUB_OFFSET);
    }
    return ~0u;
}

HG_HD inline void row_outputs(Lane &L, const LanePic &P) {
    L.tu_row = (uint32_t)L.row * P.tu_cap;
    L.coef_row = (uint32_t)L.row * P.coef_cap;
    L.ntu = L.ncoef = L.nesc = 0;
}

// one coefficient, one 4-byte store.  (Grouping four into a 16-byte store
// through registers measured 5 % slower: the selects run on every lane of
// every coefficient step, the saved stores were cheap.)
HG_HD inline void coef_push(Lane &L, const LanePic &P, uint32_t w) {
    if (P.flags & PF_COHERENT) store_word_agent((uint32_t *)(P.coef_base + L.coef_row + L.ncoef++), w);
    else P.coef_base[L.coef_row + L.ncoef++] = w;
}

// ------------------------------------------------------------------ units
// U_CTU: CTU start (7.3.8.2) and sao() (7.3.8.3).  Returns without a state
// change while the row above is less than two CTUs ahead (WPP).
template <class EG>
HG_HD inline void unit_ctu(Lane &L, LaneLds &ld, LanePic &P, const Env &E, const EG &G) {
    if (!wpp_ready<EG>(L, P, E)) return;
    L.ctbx = L.c << P.log2ctb;
    L.ctby = L.row << P.log2ctb;
    const uint32_t start = substream_start<!EG::kSolo>(L, P, *E.a);
    if (start != ~0u) {
        // substream start: contexts (init; the WPP copy already in ld.ctx; or, a
        // dependent slice segment without WPP, the previous segment's final
        // state, which the lane still holds: 9.3.2.4) + engine.  A dependent
        // segment starting inside a row (ST_SEGSW) keeps the contexts and qPY_PREV
        const bool segsw = !EG::kSolo && (L.status & ST_SEGSW) != 0;
        const bool init = !segsw && (L.row == 0 || ((L.fl & F_WPP) && P.wctb < 2));
        const bool wpp_copy = !init && (L.fl & F_WPP);
        if constexpr (EG::kCtxReg) {
#if !defined(HG_HOST_EMU)
            // every lane its dword of the contexts: initialised, or the row above's copy
            const int ln = (int)__lane_id();
            uint32_t w = L.cx;
            if (init) {
                w = 0;
                for (int b = 0; b < 4; ++b) {
                    const int i = 4 * ln + b;
                    if (i < CTX_NUM) w |= (uint32_t)ctx_init_state(c_ctx_init_l[i], P.sliceQp) << (8 * b);
                }
            } else if (wpp_copy) {
                w = 0;
                if (ln < CTX_PAD / 4) {
                    const uint8_t *src = (EG::kSpread || P.ring) ? wpp_stage(E, P, L.row) : ld.ctx;
                    const uint32_t *sw = reinterpret_cast<const uint32_t *>(src) + ln;
                    w = EG::kSpread ? load_agent(sw) : *sw;
                }
            }
            L.cx = w;
#endif
        } else if (init) {
#pragma nounroll
            for (int i = 0; i < CTX_NUM; ++i) ld.ctx[i] = ctx_init_state(c_ctx_init_l[i], P.sliceQp);
        } else if (wpp_copy && (EG::kSpread || P.ring)) {
            const uint32_t *src = reinterpret_cast<const uint32_t *>(wpp_stage(E, P, L.row));
            uint32_t *dst = reinterpret_cast<uint32_t *>(ld.ctx);
#pragma nounroll
            for (int k = 0; k < CTX_PAD / 4; ++k) dst[k] = EG::kSpread ? load_agent(src + k) : src[k];
        }
        engine_init(L, G, start, P.bits_end);
        if (segsw) {
            L.status &= ~ST_SEGSW;
            if ((L.fl >> kMsegShift) >= lanes_nmid(P)) L.status |= ST_SUBSTREAM_END;  // no such segment
            L.fl += kMsegOne;
        } else {
            if (L.row == 0) L.fl |= F_FIRST_QG;
            if constexpr (!EG::kSolo) {
                // WPP: this row's lane counts the segments started inside rows from
                // those of earlier rows (batch.cpp: after the picture's mid list)
                const uint32_t nm = lanes_nmid(P);
                if ((L.fl & F_WPP) && nm)
                    L.fl = (L.fl & (kMsegOne - 1)) |
                           (E.a->subs[P.sub_first + (uint32_t)P.hctb + 1u + nm + L.row] << kMsegShift);
            }
        }
    }
    if (P.saoL || P.saoC) {
        int ml = 0, mu = 0;
        if (L.c > 0) ml = dec(L, G, CTX_SAO_MERGE);
        if (L.row > 0 && !ml) mu = dec(L, G, CTX_SAO_MERGE);
        // the CTB's SaoParams as 8 words (desc.hpp layout), built in registers:
        // no per-lane LDS copy (merge-left re-reads the left CTB's entry, which
        // this lane stored one CTU earlier)
        uint32_t *dst = reinterpret_cast<uint32_t *>(P.gsao + (size_t)L.row * P.wctb + L.c);
        uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0, w4 = 0, w5 = 0, w6 = 0, w7 = 0;
        if (ml || mu) {
            const uint32_t *src = ml ? dst - 8 : reinterpret_cast<const uint32_t *>(P.gsao + (size_t)(L.row - 1) * P.wctb + L.c);
            w0 = load_word_coherent(src + 0);
            w1 = load_word_coherent(src + 1);
            w2 = load_word_coherent(src + 2);
            w3 = load_word_coherent(src + 3);
            w4 = load_word_coherent(src + 4);
            w5 = load_word_coherent(src + 5);
            w6 = load_word_coherent(src + 6);
            w7 = load_word_coherent(src + 7);
        } else {
            // byte b of the 32-byte record (every offset below is a constant after unrolling)
            auto put8 = [&](int b, uint32_t v) {
                const uint32_t m = (v & 0xffu) << (8 * (b & 3));
                switch (b >> 2) {
                case 0: w0 |= m; break;
                case 1: w1 |= m; break;
                case 2: w2 |= m; break;
                case 3: w3 |= m; break;
                case 4: w4 |= m; break;
                case 5: w5 |= m; break;
                case 6: w6 |= m; break;
                default: w7 |= m; break;
                }
            };
            auto put16 = [&](int b, int v) {
                put8(b, (uint32_t)v);
                put8(b + 1, (uint32_t)v >> 8);
            };
            const int ncomp = P.chroma ? 3 : 1;
            int type1 = 0, eo1 = 0;
#pragma unroll
            for (int cc = 0; cc < 3; ++cc) {
                if (cc >= ncomp) break;
                if (!((P.saoL && cc == 0) || (P.saoC && cc > 0))) continue;
                const int type = cc < 2 ? (dec(L, G, CTX_SAO_TYPE) ? (byp(L, G) ? 2 : 1) : 0) : type1;
                if (cc == 1) type1 = type;
                put8(cc, (uint32_t)type);
                if (!type) continue;
                const int bd = cc ? P.bdC : P.bdY;
                const int cmax = (1 << ((bd < 10 ? bd : 10) - 5)) - 1;
                int o[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {  // TR(cMax), bypass
                    int v = 0;
                    while (v < cmax && byp(L, G)) ++v;
                    o[i] = v;
                }
                int band_eo;
                if (type == 1) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (o[i] && byp(L, G)) o[i] = -o[i];
                    band_eo = (int)byp_bits(L, G, 5);
                } else {
                    band_eo = cc < 2 ? (int)byp_bits(L, G, 2) : eo1;
                    if (cc == 1) eo1 = band_eo;
                    o[2] = -o[2];
                    o[3] = -o[3];
                }
                put8(3 + cc, (uint32_t)band_eo);
#pragma unroll
                for (int i = 0; i < 4; ++i) put16(6 + 8 * cc + 2 * i, o[i]);
            }
        }
        const uint32_t w[8] = {w0, w1, w2, w3, w4, w5, w6, w7};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if constexpr (EG::kSpread) store_agent(dst + k, w[k]);
            else dst[k] = w[k];
        }
    }
    L.qx = L.ctbx, L.qy = L.ctby, L.ql = P.log2ctb, L.qd = 0;
    L.st = U_CQT;
}

// U_CQT: split_cu_flag descent (7.3.8.4) from the current node to a CU
template <class EG>
HG_HD inline void unit_cqt(Lane &L, LaneLds &ld, LanePic &P, const EG &G) {
    for (;;) {
        const int n = 1 << L.ql;
        bool split;
        if (L.qx + n <= P.W && L.qy + n <= P.H && L.ql > P.minCb) {
            int cond = 0;  // 9.3.4.2.2 ctxInc of split_cu_flag
            if (L.qx > 0 && ld.dL[(L.qy - L.ctby) >> 3] > L.qd) ++cond;
            if (L.qy > 0) {
                const int ad = (L.qy - 1 < L.ctby)
                                   ? load_byte_coherent(P.gdepth + (size_t)(L.row - 1) * P.w8 + (L.qx >> 3))
                                   : ld.dA[(L.qx - L.ctbx) >> 3];
                if (ad > L.qd) ++cond;
            }
            split = dec(L, G, CTX_SPLIT_CU + cond) != 0;
        } else {
            split = L.ql > P.minCb;
        }
        if (L.ql >= P.log2qg) {
            L.fl = (L.fl & ~F_DQP_CODED) | F_QG_NEW;
            L.cu_qp_delta_val = 0;
            L.qg_x = L.qx;
            L.qg_y = L.qy;
        }
        if (!split) break;
        --L.ql;  // child 0 (always inside the picture)
        ++L.qd;
    }
    L.st = U_CU;
}

HG_HD inline void cu_done(Lane &L, LaneLds &ld, LanePic &P);
HG_HD inline void tu_emit(Lane &L, const LanePic &P);

// pcm_flag = 1 (7.3.8.7 pcm_sample(); the reference parses the SPS PCM fields,
// parameter_set_reader.rs:107-125): the decoder has consumed through the
// codeword's final 1 bit, the samples start at the next byte boundary
// (pcm_alignment_zero_bits).  They are recorded as bypass TBs (TU_PCM) whose
// "coefficients" are the samples << (BitDepth - PcmBitDepth) in raster order:
// k_transform copies them and k_intra adds them to a zero prediction.  The
// engine restarts at the byte after them (9.3.2.5).  The CU counts as
// INTRA_DC for later MPM derivations (8.4.2) and is one deblocking block,
// unfiltered with pcm_loop_filter_disabled_flag.
template <class EG>
HG_HD inline void pcm_cu(Lane &L, LaneLds &ld, LanePic &P, const EG &G) {
    const int n = 1 << L.ql;
    {
        const int nb = n >> 2, by = (L.qy - L.ctby) >> 2, bx = (L.qx - L.ctbx) >> 2;
        for (int k = 0; k < nb; ++k) {
            ld.ipmL[by + k] = 1;
            ld.ipmA[bx + k] = 1;
        }
    }
    // bits consumed so far: 8 * end - budget - k (absolute RBSP bit position)
    uint32_t bit = (uint32_t)(8 * (int32_t)P.bits_end - L.budget - L.k + 7) & ~7u;
    L.fl = (L.fl | F_PCM | F_TB_CBF) & ~F_TS;
    // luma, then Cb and Cr; a 4:2:2 chroma block (raster, m wide, 2m tall) is
    // two stacked square TBs
    const int ntb = P.chroma == 0 ? 1 : (P.chroma == 2 ? 5 : 3), nh = P.chroma == 2 ? 2 : 1;
    for (int t = 0; t < ntb; ++t) {
        const int c = t == 0 ? 0 : 1 + (t - 1) / nh, h = t == 0 ? 0 : (t - 1) % nh;
        const int l2 = (c && P.chroma != 3) ? L.ql - 1 : L.ql, m = 1 << l2;
        const int pbd = c ? P.pcmBdC : P.pcmBdY, sh = (c ? P.bdC : P.bdY) - pbd;
        L.tb_cidx = c;
        L.tb_x = c ? L.qx >> P.subx : L.qx;
        L.tb_y = c ? (L.qy >> P.suby) + (h << l2) : L.qy;
        L.tb_log2 = l2;
        L.tb_mode = 1;
        L.tb_coef0 = L.ncoef;
#pragma nounroll
        for (int i = 0; i < m * m; ++i) {
            // clamped to the substream's padded end: a truncated stream reads padding
            // (and reports ST_OVERRUN below), never past the arena
            const uint32_t b = (bit >> 3) < G.lim ? bit >> 3 : G.lim;
            const uint32_t w = ((uint32_t)G.rbsp[b] << 16) | ((uint32_t)G.rbsp[b + 1] << 8) | (uint32_t)G.rbsp[b + 2];
            const uint32_t v = (w >> (24u - (bit & 7u) - (uint32_t)pbd)) & ((1u << pbd) - 1u);
            bit += (uint32_t)pbd;
            if (L.ncoef + L.nesc < P.coef_cap) coef_push(L, P, ((v << sh) << 16) | (uint32_t)i);
            else L.status |= ST_CAPACITY;
        }
        tu_emit(L, P);
    }
    L.fl &= ~(F_PCM | F_TB_CBF);
    {  // the CU's 4x4 blocks: one block for the deblocking edges
        const int nb = n >> 2, gx0 = L.qx >> 2, gy0 = L.qy >> 2;
        const int wx = gx0 + nb <= P.w4 ? nb : P.w4 - gx0, hy = gy0 + nb <= P.h4 ? nb : P.h4 - gy0;
        const uint64_t nf = ((L.fl & F_BYPASS) || (P.flags & SP_PCM_LOOP_FILTER_DISABLED)) ? MF_NOFILT : 0;
        const uint64_t rep = 0x0101010101010101ull;
        for (int y = 0; y < hy; ++y) {
            uint8_t *row = P.gflags + (size_t)(gy0 + y) * P.w4 + gx0;
            const uint64_t h = (y == 0 ? (uint64_t)MF_EDGE_H : 0u) | nf;
            store_bytes(row, wx, (rep * h) | (uint64_t)MF_EDGE_V);
        }
    }
    const uint32_t next = bit >> 3;  // the samples end on a byte boundary
    if (next > P.bits_end) L.status |= ST_OVERRUN;
    if constexpr (EG::kSolo) {  // the driver moves the window first (run_unit re-initialises)
        L.reinit = next;
        L.lb = next >> 2;
        L.fl |= F_REINIT;
    } else {
        engine_init(L, G, next, P.bits_end);
    }
    cu_done(L, ld, P);
}

// U_CU: coding_unit (7.3.8.5) up to its transform_tree
template <class EG>
HG_HD inline void unit_cu(Lane &L, LaneLds &ld, LanePic &P, const EG &G) {
    if (L.fl & F_QG_NEW) {
        derive_qp_pred(L, ld, P);
        L.fl &= ~F_QG_NEW;
    }
    update_qpy(L, P);
    L.fl &= ~(F_BYPASS | F_NXN);
    if ((P.flags & SP_TQ_BYPASS) && dec(L, G, CTX_TQ_BYPASS)) L.fl |= F_BYPASS;
    if (L.ql == P.minCb && !dec(L, G, CTX_PART_MODE)) L.fl |= F_NXN;
    const bool nxn = (L.fl & F_NXN) != 0;
    const bool pcm = !nxn && (P.flags & SP_PCM) && L.ql >= P.pcmMin && L.ql <= P.pcmMax && term(L, G);
    {  // CtDepth of the CU
        const int nd = 1 << (L.ql - 3);
        const int dy = (L.qy - L.ctby) >> 3, dx = (L.qx - L.ctbx) >> 3;
        for (int k = 0; k < nd; ++k) {
            ld.dL[dy + k] = (uint8_t)L.qd;
            ld.dA[dx + k] = (uint8_t)L.qd;
        }
    }
    if (pcm) {
        pcm_cu(L, ld, P, G);
        return;
    }
    const int np = nxn ? 4 : 1;
    const int pb = nxn ? 1 << (L.ql - 1) : 1 << L.ql;
    int prev = 0;
    for (int i = 0; i < np; ++i) prev |= dec(L, G, CTX_PREV_INTRA) << i;
    int modes = 0;
    for (int i = 0; i < np; ++i) {
        const int p = (prev >> i) & 1;
        int mpm = 0, rem = 0;
        if (p) mpm = byp(L, G) ? (byp(L, G) ? 2 : 1) : 0;
        else rem = (int)byp_bits(L, G, 5);
        const int xPb = L.qx + (i & 1) * pb, yPb = L.qy + (i >> 1) * pb;
        const int m = derive_luma_mode(L, ld, xPb, yPb, p, mpm, rem);
        modes |= m << (8 * i);
        const int nb = pb >> 2, by = (yPb - L.ctby) >> 2, bx = (xPb - L.ctbx) >> 2;
        for (int k = 0; k < nb; ++k) {
            ld.ipmL[by + k] = (uint8_t)m;
            ld.ipmA[bx + k] = (uint8_t)m;
        }
    }
    L.cu_modes = modes;
    if (P.chroma) {  // intra_chroma_pred_mode: per PB with 4:4:4, else per CU; 8.4.3
        const int nc = P.chroma == 3 ? np : 1;
        int cms = 0;
        for (int i = 0; i < nc; ++i) {
            const int icpm = dec(L, G, CTX_CHROMA_MODE) ? (int)byp_bits(L, G, 2) : 4;
            const int lm = (modes >> (8 * i)) & 0xff;
            int cm;
            if (icpm == 4) {
                cm = lm;
            } else {
                cm = icpm == 0 ? 0 : (icpm == 1 ? 26 : (icpm == 2 ? 10 : 1));
                if (cm == lm) cm = 34;
            }
            if (P.chroma == 2) cm = mode422(cm);
            cms |= cm << (8 * i);
        }
        L.cu_chroma = nc == 1 ? (int)((uint32_t)cms * 0x01010101u) : cms;  // byte k: PB k
    }
    L.tx = L.qx, L.ty = L.qy, L.tl = L.ql, L.td = 0, L.tcbf = 0;
    L.st = U_TT;
}

// U_TT: transform_tree descent (7.3.8.8) from the current node to a leaf,
// then transform_unit (7.3.8.10) up to its first TB
template <class EG>
HG_HD inline void unit_tt(Lane &L, LaneLds &ld, LanePic &P, const EG &G) {
    const bool nxn = (L.fl & F_NXN) != 0;
    const int max_depth = P.maxDepthIntra + (nxn ? 1 : 0);
    for (;;) {
        bool split;
        if (L.tl <= P.maxTb && L.tl > P.minTb && L.td < max_depth && !(nxn && L.td == 0))
            split = dec(L, G, CTX_SPLIT_TF + 5 - L.tl) != 0;
        else
            split = L.tl > P.maxTb || (nxn && L.td == 0);
        uint32_t cbf = 0;  // cbf_cb | cbf_cr << 1, 4:2:2 lower TBs << 2 / << 3 (7.3.8.8)
        if ((L.tl > 2 && P.chroma) || P.chroma == 3) {
            const uint32_t pc = L.td == 0 ? 3u : (L.tcbf >> (4 * (L.td - 1))) & 3u;
            const bool two = P.chroma == 2 && (!split || L.tl == 3);
            if (pc & 1) {
                cbf |= (uint32_t)dec(L, G, CTX_CBF_CHROMA + L.td);
                if (two) cbf |= (uint32_t)dec(L, G, CTX_CBF_CHROMA + L.td) << 2;
            }
            if (pc & 2) {
                cbf |= (uint32_t)dec(L, G, CTX_CBF_CHROMA + L.td) << 1;
                if (two) cbf |= (uint32_t)dec(L, G, CTX_CBF_CHROMA + L.td) << 3;
            }
        }
        L.tcbf = (L.tcbf & ~(15u << (4 * L.td))) | (cbf << (4 * L.td));
        if (!split) break;
        --L.tl;  // child 0
        ++L.td;
    }
    const uint32_t cbf = (L.tcbf >> (4 * L.td)) & 15u;
    L.fl &= ~F_CBF_L;
    if (dec(L, G, CTX_CBF_LUMA + (L.td == 0 ? 1 : 0))) L.fl |= F_CBF_L;
    // transform_unit
    const bool chroma4 = (P.chroma == 1 || P.chroma == 2) && L.tl == 2;
    const uint32_t pc = L.td > 0 ? (L.tcbf >> (4 * (L.td - 1))) & 15u : 0u;  // the parent's chroma cbfs
    const bool cbf_c = P.chroma == 0 ? false : (chroma4 ? pc != 0 : cbf != 0);
    if (((L.fl & F_CBF_L) || cbf_c) && (P.flags & SP_CU_QP_DELTA) && !(L.fl & F_DQP_CODED)) {
        int v = 0;  // cu_qp_delta_abs: TR prefix (cMax 5), EG0 suffix
        while (v < 5 && dec(L, G, CTX_CU_QP_DELTA + (v == 0 ? 0 : 1))) ++v;
        if (v == 5) {
            int ones = 0;
            bool bad = false;
            while (byp(L, G)) {
                if (++ones > 31) {
                    bad = true;
                    break;
                }
            }
            if (bad) L.status |= ST_SYNTAX;
            else v += (int)(((1u << ones) - 1u) + byp_bits(L, G, ones));
        }
        if (v && byp(L, G)) v = -v;
        // 7.4.9.14: CuQpDeltaVal in [-(26 + QpBdOffsetY / 2), 25 + QpBdOffsetY / 2]
        // (outside it, QpY and the scaling shift would leave their ranges)
        const int vlo = -(26 + P.qpbdY / 2), vhi = 25 + P.qpbdY / 2;
        if (v < vlo || v > vhi) {
            L.status |= ST_SYNTAX;
            v = v < vlo ? vlo : vhi;
        }
        L.fl |= F_DQP_CODED;
        L.cu_qp_delta_val = v;
        update_qpy(L, P);
    }
    {  // edge / no-filter flags of every 4x4 luma block of the TB (MF_*)
        const int nb = 1 << (L.tl - 2), gx0 = L.tx >> 2, gy0 = L.ty >> 2;
        const int wx = gx0 + nb <= P.w4 ? nb : P.w4 - gx0, hy = gy0 + nb <= P.h4 ? nb : P.h4 - gy0;
        const uint64_t nf = (L.fl & F_BYPASS) ? MF_NOFILT : 0;
        const uint64_t rep = 0x0101010101010101ull;
        for (int y = 0; y < hy; ++y) {
            uint8_t *row = P.gflags + (size_t)(gy0 + y) * P.w4 + gx0;
            const uint64_t h = (y == 0 ? (uint64_t)MF_EDGE_H : 0u) | nf;
            store_bytes(row, wx, (rep * h) | (uint64_t)MF_EDGE_V);
        }
    }
    const int blk = L.td == 0 ? 0 : (((L.tx >> L.tl) & 1) | (((L.ty >> L.tl) & 1) << 1));
    // luma, then Cb and Cr (two each with 4:2:2: upper, lower)
    L.tb_n = (P.chroma != 0 && (!chroma4 || blk == 3)) ? (P.chroma == 2 ? 5 : 3) : 1;
    L.tb_t = 0;
    L.st = U_TB;
}

// record of the current TB (TuRec, desc.hpp)
HG_HD inline void tu_emit(Lane &L, const LanePic &P) {
    int qp;
    if (L.tb_cidx == 0) {
        qp = L.qpy_cur + P.qpbdY;
    } else {
        const int off = L.tb_cidx == 1 ? P.cbOff : P.crOff;
        int qpi = L.qpy_cur + off;
        qpi = qpi < -P.qpbdC ? -P.qpbdC : (qpi > 57 ? 57 : qpi);
        qp = chroma_qp_map(qpi, P.chroma) + P.qpbdC;
    }
    uint32_t f = (uint32_t)L.tb_cidx;
    if (L.fl & F_TB_CBF) f |= TU_CBF;
    if (L.fl & F_TS) f |= TU_TSKIP;
    if (L.fl & F_BYPASS) f |= TU_BYPASS;
    if (L.fl & F_PCM) f |= TU_PCM | TU_BYPASS;
    if (L.tb_cidx == 0 && L.tb_log2 == 2) f |= TU_DST;
    if (L.ntu < P.tu_cap) {
        const uint32_t w0 = (uint32_t)L.tb_x | ((uint32_t)L.tb_y << 16);
        const uint32_t w1 = (uint32_t)L.tb_log2 | (f << 8) | ((uint32_t)L.tb_mode << 16) | ((uint32_t)(uint8_t)qp << 24);
        const uint32_t w3 = (L.ncoef - L.tb_coef0) | ((uint32_t)L.c << 16);
        if (P.flags & PF_COHERENT) store_tu_agent(P.tu_base + L.tu_row + L.ntu, w0, w1, L.tb_coef0, w3);
        else store_tu(P.tu_base + L.tu_row + L.ntu, w0, w1, L.tb_coef0, w3);
        ++L.ntu;
    } else {
        L.status |= ST_CAPACITY;
    }
}

HG_HD inline void cu_done(Lane &L, LaneLds &ld, LanePic &P);

// After a TB: its record, then the next TB of the TU, the next transform-tree
// node, or (tree done) the CU's QpY and the next coding-quadtree node / CTU end.
HG_HD inline void tb_done(Lane &L, LaneLds &ld, LanePic &P) {
    tu_emit(L, P);
    if (++L.tb_t < L.tb_n) {
        L.st = U_TB;
        return;
    }
    // next transform-tree node in z-order (nodes are aligned to their size)
    while (L.td > 0) {
        const int s = 1 << L.tl;
        const int b = ((L.tx >> L.tl) & 1) | (((L.ty >> L.tl) & 1) << 1);
        if (b < 3) {
            const int px = L.tx & ~(2 * s - 1), py = L.ty & ~(2 * s - 1);
            L.tx = px + ((b + 1) & 1) * s;
            L.ty = py + ((b + 1) >> 1) * s;
            L.st = U_TT;
            return;
        }
        L.tx &= ~(2 * s - 1);
        L.ty &= ~(2 * s - 1);
        ++L.tl;
        --L.td;
    }
    cu_done(L, ld, P);
}

// end of a CU: QpY for qPY_A/B and the 4x4 map (deblocking), then the next
// coding-quadtree node in z-order (skipping children outside the picture) or
// the CTU end
HG_HD inline void cu_done(Lane &L, LaneLds &ld, LanePic &P) {
    {
        const int n = 1 << L.ql, nd = n >> 3;
        const int dy = (L.qy - L.ctby) >> 3, dx = (L.qx - L.ctbx) >> 3;
        for (int k = 0; k < nd; ++k) {
            ld.qL[dy + k] = (int8_t)L.qpy_cur;
            ld.qA[dx + k] = (int8_t)L.qpy_cur;
        }
        const int nb = n >> 2, gx0 = L.qx >> 2, gy0 = L.qy >> 2;
        const int wx = gx0 + nb <= P.w4 ? nb : P.w4 - gx0, hy = gy0 + nb <= P.h4 ? nb : P.h4 - gy0;
        for (int y = 0; y < hy; ++y) {
            int8_t *row = P.gqpy + (size_t)(gy0 + y) * P.w4 + gx0;
            store_bytes(reinterpret_cast<uint8_t *>(row), wx, 0x0101010101010101ull * (uint8_t)L.qpy_cur);
        }
        L.qp_prev_last = L.qpy_cur;
    }
    // next coding-quadtree node in z-order, skipping children outside the picture
    while (L.qd > 0) {
        const int s = 1 << L.ql;
        const int px = L.qx & ~(2 * s - 1), py = L.qy & ~(2 * s - 1);
        for (int b = (((L.qx >> L.ql) & 1) | (((L.qy >> L.ql) & 1) << 1)) + 1; b < 4; ++b) {
            const int cx = px + (b & 1) * s, cy = py + (b >> 1) * s;
            if (cx < P.W && cy < P.H) {
                L.qx = cx;
                L.qy = cy;
                L.st = U_CQT;
                return;
            }
        }
        L.qx = px;
        L.qy = py;
        ++L.ql;
        --L.qd;
    }
    L.st = U_CTU_END;
}

// U_TB: TB tb_t of the TU; without coefficients it is done here, otherwise
// residual_coding's header (transform_skip_flag, last position) is parsed
template <class EG>
HG_HD inline void unit_tb(Lane &L, LaneLds &ld, LanePic &P, const EG &G) {
    const int t = L.tb_t;
    const bool chroma4 = (P.chroma == 1 || P.chroma == 2) && L.tl == 2;
    // component and (4:2:2) upper / lower half of TB t: luma, Cb (, Cb lower), Cr (, Cr lower)
    const bool c422 = P.chroma == 2;
    const int comp = t == 0 ? 0 : (c422 ? 1 + ((t - 1) >> 1) : t), half = (c422 && t > 0) ? (t - 1) & 1 : 0;
    bool cbf;
    L.tb_cidx = comp;
    if (t == 0) {
        L.tb_x = L.tx;
        L.tb_y = L.ty;
        L.tb_log2 = L.tl;
        int k = 0;  // IntraPredModeY of the PB the TB lies in
        if (L.fl & F_NXN) {
            const int half = 1 << (L.ql - 1);
            k = ((L.ty - L.qy) >= half ? 2 : 0) + ((L.tx - L.qx) >= half ? 1 : 0);
        }
        L.tb_mode = (L.cu_modes >> (8 * k)) & 0xff;
        cbf = (L.fl & F_CBF_L) != 0;
    } else if (!chroma4) {
        L.tb_log2 = P.chroma == 3 ? L.tl : L.tl - 1;  // log2TrafoSizeC
        L.tb_x = L.tx >> P.subx;
        L.tb_y = (L.ty >> P.suby) + (half << L.tb_log2);
        int k = 0;  // IntraPredModeC of the PB (4:4:4 NxN: four)
        if (P.chroma == 3 && (L.fl & F_NXN)) {
            const int hp = 1 << (L.ql - 1);
            k = ((L.ty - L.qy) >= hp ? 2 : 0) + ((L.tx - L.qx) >= hp ? 1 : 0);
        }
        L.tb_mode = (L.cu_chroma >> (8 * k)) & 0xff;
        cbf = ((L.tcbf >> (4 * L.td + (comp - 1) + 2 * half)) & 1u) != 0;
    } else {  // 4:2:0 / 4:2:2, 4x4 luma TBs: the chroma TBs of the 8x8 parent, after its 4th luma TB
        const int s = 1 << (L.tl + 1);
        L.tb_x = (L.tx & ~(s - 1)) >> 1;
        L.tb_y = ((L.ty & ~(s - 1)) >> P.suby) + 4 * half;
        L.tb_log2 = 2;
        L.tb_mode = L.cu_chroma & 0xff;
        cbf = ((L.tcbf >> (4 * (L.td - 1) + (comp - 1) + 2 * half)) & 1u) != 0;
    }
    L.fl = (L.fl & ~(F_TS | F_TB_CBF)) | (cbf ? F_TB_CBF : 0u);
    L.tb_coef0 = L.ncoef;
    if (!cbf) {
        tb_done(L, ld, P);
        return;
    }
    // residual_coding header (7.3.8.11)
    const int l2 = L.tb_log2, n = 1 << l2, cidx = comp;
    if ((P.flags & SP_TRANSFORM_SKIP) && !(L.fl & F_BYPASS) && l2 == 2 && dec(L, G, CTX_TS_FLAG + (cidx ? 1 : 0)))
        L.fl |= F_TS;
    // last_sig_coeff_{x,y}_prefix (decoder.rs:109-130), suffixes
    const int cmax = (l2 << 1) - 1;
    const int off = cidx == 0 ? 3 * (l2 - 2) + ((l2 - 1) >> 2) : 15;
    const int shift = cidx == 0 ? (l2 + 1) >> 2 : l2 - 2;
    int px = 0, py = 0;
    while (px < cmax && dec(L, G, CTX_LAST_X + off + (px >> shift))) ++px;
    while (py < cmax && dec(L, G, CTX_LAST_Y + off + (py >> shift))) ++py;
    int lx = px, ly = py;
    if (px > 3) {
        const int k = (px >> 1) - 1;
        lx = (1 << k) * (2 + (px & 1)) + (int)byp_bits(L, G, k);
    }
    if (py > 3) {
        const int k = (py >> 1) - 1;
        ly = (1 << k) * (2 + (py & 1)) + (int)byp_bits(L, G, k);
    }
    int scan = 0;  // 7.4.9.11 scanIdx
    if (l2 == 2 || (l2 == 3 && (cidx == 0 || P.chroma == 3))) {
        if (L.tb_mode >= 6 && L.tb_mode <= 14) scan = 2;
        else if (L.tb_mode >= 22 && L.tb_mode <= 30) scan = 1;
    }
    if (scan == 2) {
        const int tt = lx;
        lx = ly;
        ly = tt;
    }
    if (lx >= n || ly >= n) {
        L.status |= ST_SYNTAX;
        lx &= n - 1;
        ly &= n - 1;
    }
    const int sbl = l2 - 2, sbw = 1 << sbl;
    L.rc_scan = scan;
    L.rc_last_sub = scan_inv(G, sbl, scan, (ly >> 2) * sbw + (lx >> 2));
    L.rc_last_pos = scan_inv(G, 2, scan, (ly & 3) * 4 + (lx & 3));
    L.rc_csbf = 0;
    L.rc_prev_c1 = 1;
    L.fl &= ~F_ANY_SB;
    L.rc_i = L.rc_last_sub;
    L.st = U_SB;
}

// bit n of a 16-bit mask to bit 4n (a nibble per scan position).  Scalar
// engine: two s_bitreplicate_b64_b32 (each bit doubled) and a mask, three
// SALU ops instead of the twelve of the shift-and-mask ladder
template <bool Scalar = false>
HG_HD inline uint64_t spread16_nib(uint32_t m) {
#if !defined(HG_HOST_EMU) && defined(__HIP_DEVICE_COMPILE__) && !defined(HG_NO_BITREPLICATE)
    if constexpr (Scalar) {
        uint64_t x2, x4;
        asm("s_bitreplicate_b64_b32 %0, %1" : "=s"(x2) : "s"(uni32(m & 0xffffu)));
        asm("s_bitreplicate_b64_b32 %0, %1" : "=s"(x4) : "s"((uint32_t)x2));
        return x4 & 0x1111111111111111ull;
    }
#endif
    uint64_t x = m & 0xffffu;
    x = (x | (x << 24)) & 0x000000ff000000ffull;
    x = (x | (x << 12)) & 0x000f000f000f000full;
    x = (x | (x << 6)) & 0x0303030303030303ull;
    x = (x | (x << 3)) & 0x1111111111111111ull;
    return x;
}

// the sub-block's record (SbRec): one 16-byte store (4 coefficient words); the
// first escape of the record is the escape slot at L.nesc when it started
template <class L_, class P_>
HG_HD inline void sb_store(L_ &L, const P_ &P, uint32_t sig, uint32_t signs, uint64_t nib, int xS, int yS, bool hide) {
    const uint32_t nesc_sb = (uint32_t)__builtin_popcountll(nib & (nib >> 1) & (nib >> 2) & (nib >> 3) & 0x1111111111111111ull);
    const uint32_t esc0 = P.coef_cap - 1 - (L.nesc - nesc_sb);  // row-relative index of its first escape
    const uint32_t w0 = (sig & 0xffffu) | (signs & 0xffff0000u);
    const uint32_t w3 = (uint32_t)xS | ((uint32_t)yS << 3) | ((uint32_t)L.rc_scan << 6) | (hide ? 1u << 8 : 0u) |
                        (esc0 << 9);
    if (L.ncoef + L.nesc + 4 <= P.coef_cap) {
        TuRec *d = (TuRec *)(P.coef_base + L.coef_row + L.ncoef);
        if (P.flags & PF_COHERENT) store_tu_agent(d, w0, (uint32_t)nib, (uint32_t)(nib >> 32), w3);
        else store_tu(d, w0, (uint32_t)nib, (uint32_t)(nib >> 32), w3);
        L.ncoef += 4;
    } else {
        L.status |= ST_CAPACITY;
    }
}

// U_SB: sub-block rc_i of residual_coding (7.3.8.11, 9.3.4.2.5-7)
template <class EG>
HG_HD inline void unit_sb(Lane &L, LaneLds &ld, LanePic &P, const EG &G) {
#if defined(HG_PARSE_PROF_SB) && !defined(HG_HOST_EMU)
    uint64_t tsb = __builtin_amdgcn_s_memtime();
#endif
    const int l2 = L.tb_log2, cidx = L.tb_cidx, i = L.rc_i;
    const int sbl = l2 - 2, sbw = 1 << sbl;
    const int sp = scan_pos(G, sbl, L.rc_scan, i);
    const int xS = sp & 15, yS = sp >> 4;
    int pcs = 0;  // prevCsbf
    if (xS < sbw - 1) pcs |= (int)((L.rc_csbf >> (yS * 8 + xS + 1)) & 1);
    if (yS < sbw - 1) pcs |= (int)((L.rc_csbf >> ((yS + 1) * 8 + xS)) & 1) << 1;
    bool coded = true, infer_dc = false;
    if (i < L.rc_last_sub && i > 0) {
        coded = dec(L, G, CTX_CSBF + ((pcs & 1) | (pcs >> 1)) + (cidx ? 2 : 0)) != 0;
        infer_dc = true;
    }
    uint32_t sig = 0;
    if (coded) {
        L.rc_csbf |= 1ull << (yS * 8 + xS);
        int nstart = 15;
        if (i == L.rc_last_sub) {
            sig = 1u << L.rc_last_pos;
            nstart = L.rc_last_pos - 1;
        }
        // sig_coeff_flag contexts of the sub-block (9.3.4.2.5) in a register
        // cache: a 4x4 TB uses sigCtx 0..8 (ctxIdxMap, slots 0..8); larger TBs
        // use sigCtx 0 at the TB's DC (slot 0) and off + 0..2 (slots 1..3)
        const int cbase = CTX_SIG + (cidx ? 27 : 0);
        auto cb = [&](int i) { return ctx_ld(L, G, cbase + i); };
        uint64_t seq = G.seqw(L.rc_scan * 5 + (l2 == 2 ? 4 : pcs));  // slot per scan position
        uint32_t c0 = 0, c1 = 0, c2 = 0;
        // vector engines: the sub-block's (up to 9) context states as 7-bit fields
        // of one 64-bit word, slot k at bit 7k (a state byte is below 128:
        // pStateIdx << 1 | valMps), so a slot is one 64-bit shift and mask each way.
        // The 3-word byte cache the scalar engine keeps took two compares, two
        // selects and a bit-field extract to read a slot and three selects to
        // write it back.  r06 A/B (profiles/r06/ab/ab_cc7.txt): 22,805 -> 23,052
        // Mpix/s at 128 images; in the scalar engine's 4x4 loop the same fields
        // cost one image 24.88 -> 25.2 ms, so it keeps its byte word and slot 8
        constexpr bool kCc7 = !EG::kSolo;
        uint64_t cc = 0;
        int off = 0;
        if (l2 == 2) {
            if constexpr (kCc7) {
                for (int k = 0; k < 9; ++k) cc |= (uint64_t)cb(k) << (7 * k);
            } else {
                c0 = cb(0) | (cb(1) << 8) | (cb(2) << 16) | (cb(3) << 24);
                c1 = cb(4) | (cb(5) << 8) | (cb(6) << 16) | (cb(7) << 24);
                c2 = cb(8);
            }
        } else {
            off = cidx == 0 ? ((xS | yS) ? 3 : 0) + (l2 == 3 ? (L.rc_scan == 0 ? 9 : 15) : 21) : (l2 == 3 ? 9 : 12);
            if ((xS | yS) == 0) seq &= ~0xfull;  // DC of the TB (scan position 0 of sub-block 0): sigCtx 0
            if constexpr (kCc7)
                cc = (uint64_t)cb(0) | ((uint64_t)cb(off) << 7) | ((uint64_t)cb(off + 1) << 14) |
                     ((uint64_t)cb(off + 2) << 21);
            else
                c0 = cb(0) | (cb(off) << 8) | (cb(off + 1) << 16) | (cb(off + 2) << 24);
        }
        HG_SB_T(L, 0, tsb);
        if constexpr (EG::kSolo) {
          if (l2 > 2 && !sb_generic_loop()) {
            // scalar engine, TBs above 4x4: the four slots in one 32-bit word
            // (a byte shift reads or writes a slot), no slot 8 to select
            auto dec_slot4 = [&](uint32_t slot) -> uint32_t {
                const uint32_t sh = slot * 8u;
                uint32_t cs = (c0 >> sh) & 0xffu;
                const uint32_t bin = (uint32_t)dec_s(L, G, cs);
                c0 = (c0 & ~(0xffu << sh)) | (cs << sh);
                return bin;
            };
            uint32_t sg = sig;
            for (int nn = nstart; nn > 0; --nn) sg |= dec_slot4((uint32_t)(seq >> (4 * nn)) & 3u) << nn;
            if (nstart >= 0) sg |= (infer_dc && sg == 0) ? 1u : dec_slot4((uint32_t)seq & 3u);
            sig = sg;
          } else {
            // scalar engine: slots 0..7 as one 64-bit word (a shift reads or
            // writes a slot), slot 8 apart; every select branch-free, the bin
            // an integer, so an iteration is one scalar chain
            uint64_t cc = (uint64_t)c0 | ((uint64_t)c1 << 32);
            auto dec_slot = [&](uint32_t slot) -> uint32_t {
                const uint32_t sh = (slot & 7u) * 8u;
                const bool hi = slot >= 8u;
                uint32_t cs = hi ? c2 : (uint32_t)(cc >> sh) & 0xffu;
                const uint32_t bin = (uint32_t)dec_s(L, G, cs);
                const uint64_t ncc = (cc & ~(0xffull << sh)) | ((uint64_t)cs << sh);
                cc = hi ? cc : ncc;
                c2 = hi ? cs : c2;
                return bin;
            };
            // positions nstart .. 1 are always decoded; only position 0 of a
            // coded sub-block with no other significant coefficient is inferred
            uint32_t sg = sig;
            for (int nn = nstart; nn > 0; --nn) sg |= dec_slot((uint32_t)(seq >> (4 * nn)) & 15u) << nn;
            if (nstart >= 0) sg |= (infer_dc && sg == 0) ? 1u : dec_slot((uint32_t)seq & 15u);
            sig = sg;
            c0 = (uint32_t)cc;
            c1 = (uint32_t)(cc >> 32);
          }
        } else {
            // positions nstart .. 1 without a per-position branch (the bin is or-ed
            // in), position 0 apart: inferred in a coded sub-block with no other
            // significant coefficient (r05 A/B against the r04 loop, which tested
            // for the inferred DC at every position: parse alone 63.1 -> 59.9 ms,
            // 18,770 -> 19,260 Mpix/s at 128 images)
            auto dec_slot = [&](int slot) -> uint32_t {
                if constexpr (kCc7) {
                    // the new byte goes in under the field's mask (v_bfi), which
                    // also drops dec_t's bin bit
                    const uint32_t sh = (uint32_t)slot * 7u;
                    const uint64_t m = 0x7full << sh;
                    uint32_t t;
                    const uint32_t bin = (uint32_t)dec_t(L, G, (uint32_t)(cc >> sh) & 0x7fu, t);
                    const uint64_t tv = (uint64_t)t << sh;
                    cc = (uint64_t)bfi32((uint32_t)m, (uint32_t)tv, (uint32_t)cc) |
                         ((uint64_t)bfi32((uint32_t)(m >> 32), (uint32_t)(tv >> 32), (uint32_t)(cc >> 32)) << 32);
                    return bin;
                } else {
                    uint32_t cs = cache_get(c0, c1, c2, slot);
                    const uint32_t bin = (uint32_t)dec_s(L, G, cs);
                    cache_put(c0, c1, c2, slot, cs);
                    return bin;
                }
            };
            if constexpr (kCc7) {
                // the slot of position nn taken from the top nibble of a copy of
                // seq shifted left one nibble per position (no per-lane shift count)
                uint64_t sq = nstart > 0 ? seq << (4 * (15 - nstart)) : 0ull;
                for (int nn = nstart; nn > 0; --nn) {
                    sig |= dec_slot((int)(uint32_t)(sq >> 60)) << nn;
                    sq <<= 4;
                }
            } else {
                for (int nn = nstart; nn > 0; --nn) sig |= dec_slot((int)((seq >> (4 * nn)) & 15u)) << nn;
            }
            if (nstart >= 0) {
                if (infer_dc && sig == 0) sig |= 1u;
                else sig |= dec_slot((int)(seq & 15u));
            }
        }
        auto cw = [&](int i, uint32_t v) { ctx_st(L, G, cbase + i, v & 0xffu); };
        if constexpr (kCc7) {
            if (l2 == 2) {
                for (int k = 0; k < 9; ++k) cw(k, (uint32_t)(cc >> (7 * k)) & 0x7fu);
            } else {
                cw(0, (uint32_t)cc & 0x7fu);
                cw(off, (uint32_t)(cc >> 7) & 0x7fu);
                cw(off + 1, (uint32_t)(cc >> 14) & 0x7fu);
                cw(off + 2, (uint32_t)(cc >> 21) & 0x7fu);
            }
        } else if (l2 == 2) {
            for (int k = 0; k < 4; ++k) cw(k, c0 >> (8 * k));
            for (int k = 0; k < 4; ++k) cw(4 + k, c1 >> (8 * k));
            cw(8, c2);
        } else {
            cw(0, c0);
            cw(off, c0 >> 8);
            cw(off + 1, c0 >> 16);
            cw(off + 2, c0 >> 24);
        }
#if defined(HG_PARSE_PROF_SB) && !defined(HG_HOST_EMU)
        L.psb[4] += (uint64_t)(nstart + 1);
#endif
        HG_SB_T(L, 1, tsb);
    }
    if (sig) {
        // greater1 / greater2 (9.3.4.2.6-7)
        int ctx_set = (i == 0 || cidx > 0) ? 0 : 2;
        if ((L.fl & F_ANY_SB) && L.rc_prev_c1 == 0) ++ctx_set;
        L.fl |= F_ANY_SB;
        int c1 = 1;
        uint32_t g1 = 0, g2 = 0;
        // the ctxSet's four greater1 contexts (9.3.4.2.6) in one register
        const int gbase = CTX_GT1 + ctx_set * 4 + (cidx ? 16 : 0);
        uint32_t gc = ctx_ld(L, G, gbase) | (ctx_ld(L, G, gbase + 1) << 8) | (ctx_ld(L, G, gbase + 2) << 16) |
                      (ctx_ld(L, G, gbase + 3) << 24);
        const int first_sig = 31 - __builtin_clz(sig & (0u - sig));
        const int last_sig = msb32(sig);
        int num_g1 = 0, last_g1 = -1;
        uint32_t beyond8 = sig;  // after the greater1 loop: the significant positions past the first eight
        if constexpr (EG::kSolo) {
            // scalar engine: the first 8 significant positions, every update a
            // select on integers (no boolean carried across the engine's refill branch)
            uint32_t &m = beyond8;
            for (int j = 0; j < 8 && m; ++j) {
                const int nn = msb32(m);
                m ^= 1u << nn;
                const uint32_t gs = (uint32_t)(c1 < 3 ? c1 : 3) * 8u;
                uint32_t cs = (gc >> gs) & 0xffu;
                const uint32_t f = (uint32_t)dec_s(L, G, cs);
                gc = (gc & ~(0xffu << gs)) | (cs << gs);
                g1 |= f << nn;
                c1 = (c1 > 0 && !f) ? c1 + 1 : 0;
            }
            // the first greater1 flag set in decoding order: positions decode from the highest down
            last_g1 = g1 ? msb32(g1) : -1;
        } else {
            for (uint32_t &m = beyond8; m && num_g1 < 8;) {
                const int nn = msb32(m);
                m &= ~(1u << nn);
                const int gs = (c1 < 3 ? c1 : 3) * 8;
                const uint32_t gm = 0x7fu << gs;  // (bit 7 of every byte of gc stays 0)
                uint32_t t;
                const int f = dec_t(L, G, (gc >> gs) & 0xffu, t);
                gc = bfi32(gm, t << gs, gc);
                ++num_g1;
                g1 |= (uint32_t)f << nn;
                if (c1 > 0) c1 = f ? 0 : c1 + 1;
            }
            last_g1 = g1 ? msb32(g1) : -1;  // the first set in decoding order (positions decode downwards)
        }
        L.rc_prev_c1 = c1;
        for (int k = 0; k < 4; ++k) ctx_st(L, G, gbase + k, (gc >> (8 * k)) & 0xffu);
        if (last_g1 >= 0 && dec(L, G, CTX_GT2 + ctx_set + (cidx ? 4 : 0))) g2 = 1u << last_g1;
        HG_SB_T(L, 2, tsb);
        const bool sign_hidden = !(L.fl & F_BYPASS) && (last_sig - first_sig > 3);
        const bool hide = (P.flags & SP_SIGN_HIDING) && sign_hidden;
        const int nsign = __builtin_popcount(sig) - (hide ? 1 : 0);
        uint32_t signs = byp_bits(L, G, nsign);
        signs = nsign ? signs << (32 - nsign) : 0u;  // first decoded sign in bit 31
        // The sub-block leaves as one 16-byte record (SbRec, desc.hpp): the
        // significance map, the signs in decoding order, and abs - 1 of every
        // scan position as a nibble (15: the level is in the row's escape list,
        // which grows down from the end of the row's coefficient space).  abs - 1
        // is greater1 + greater2 (bit masks spread to nibbles) plus
        // coeff_abs_level_remaining where one is coded, so only those levels
        // are visited, one at a time (their Rice parameters chain); the r03
        // layout stored every coefficient with its own 4-byte store.
#if defined(HG_R05_BASE)
        uint64_t nib = spread16_nib(g1) + spread16_nib(g2);
#else
        uint64_t nib = spread16_nib<EG::kSolo>(g1) + (g2 ? 1ull << (4 * last_g1) : 0ull);  // (g2: at most the one bit)
#endif
        {
            // the levels with a coded remainder: greater1 set but not the one with a
            // greater2 flag, greater2 set, and every position past the first eight
            const uint32_t lastb = last_g1 >= 0 ? 1u << last_g1 : 0u;
#if defined(HG_R05_BASE)  // A/B only: the first-eight mask recomputed (as before)
            uint32_t m8 = sig;
            for (int j = 0; j < 8 && m8; ++j) m8 &= ~(1u << msb32(m8));
            m8 = sig & ~m8;
            uint32_t need = (g1 & ~lastb) | g2 | (sig & ~m8);
#else
            uint32_t need = (g1 & ~lastb) | g2 | beyond8;
#endif
            int last_abs = 0, last_rice = 0;
            bool first_rem = true;
            while (need) {
                const int nn = msb32(need);
                need ^= 1u << nn;
                const int base = 1 + (int)((g1 >> nn) & 1) + (int)((g2 >> nn) & 1);
                int k;
                if (first_rem) {
                    k = 0;
                    first_rem = false;
                } else {
                    k = last_rice + (last_abs > 3 * (1 << last_rice) ? 1 : 0);
                    k = k < 4 ? k : 4;
                }
                // coeff_abs_level_remaining (decoder.rs:230-261): TR(4 << k, k) prefix, EG(k + 1) escape
                int rem = byp_rem(L, G, k);
                if (rem < 0) {
                    // EG(k + 1) prefix: unary ones, up to 8 per division, at most 31 - (k + 1)
                    const int lim = 31 - (k + 1);
                    int ones = 0;
                    for (;;) {
                        const int mm = lim + 1 - ones < 8 ? lim + 1 - ones : 8;
                        const int pz = byp_unary(L, G, mm);
                        ones += pz;
                        if (pz < mm || ones > lim) break;  // the terminating 0 read, or too many ones
                    }
                    if (ones > lim) {
                        L.status |= ST_SYNTAX;
                        rem = 0;
                    } else {
                        rem = (int)((4u << k) + (((1u << ones) - 1u) << (k + 1)) + byp_bits(L, G, ones + k + 1));
                    }
                }
                last_abs = base + rem;
                last_rice = k;
                const int am1 = base - 1 + rem;  // abs - 1
                nib = (nib & ~(0xfull << (4 * nn))) | ((uint64_t)(am1 < 15 ? am1 : 15) << (4 * nn));
                if (am1 >= 15) {  // escape: the whole level, in descending scan order from the row's end
                    if (L.ncoef + L.nesc + 4 < P.coef_cap) {
                        Coef HG_GAS *e = P.coef_base + L.coef_row + P.coef_cap - 1 - L.nesc;
                        if (P.flags & PF_COHERENT) store_word_agent((uint32_t *)e, (uint32_t)last_abs);
                        else *e = (uint32_t)last_abs;
                    } else {
                        L.status |= ST_CAPACITY;
                    }
                    ++L.nesc;
                }
            }
        }
        HG_SB_T(L, 3, tsb);
        sb_store(L, P, sig, signs, nib, xS, yS, hide);
    }
    if (--L.rc_i < 0) tb_done(L, ld, P);
}

// U_CTU_END: WPP context storage, the depth line, end_of_slice_segment_flag /
// end_of_subset_one_bit (slice.rs:214-227), progress, next CTU / row
template <class EG>
HG_HD inline void unit_ctu_end(Lane &L, LaneLds &ld, LanePic &P, const Env &E, const EG &G) {
    if ((L.fl & F_WPP) && L.c == 1 && L.row + 1 < P.hctb) {
        // 9.3.2.4 storage for the next row's substream: into its lane's block, or
        // its staging block when that lane may still be parsing an earlier row
        uint32_t *dst = reinterpret_cast<uint32_t *>((EG::kSpread || P.ring) ? wpp_stage(E, P, L.row + 1)
                                                                              : E.lds[P.lane0 + (L.row + 1) % P.R].ctx);
        if constexpr (EG::kCtxReg) {
#if !defined(HG_HOST_EMU)
            const int ln = (int)__lane_id();  // every lane stores its dword
            if (ln < CTX_PAD / 4) {
                if constexpr (EG::kSpread) store_agent(dst + ln, L.cx);
                else dst[ln] = L.cx;
            }
#endif
        } else {
            const uint32_t *src = reinterpret_cast<const uint32_t *>(ld.ctx);
#pragma nounroll
            for (int k = 0; k < CTX_PAD / 4; ++k) {
                if constexpr (EG::kSpread) store_agent(dst + k, src[k]);
                else dst[k] = src[k];
            }
        }
    }
    {  // bottom CtDepth of this CTB for the row below
        const int nb8 = 1 << (P.log2ctb - 3), col0 = L.ctbx >> 3;
        uint8_t *line = P.gdepth + (size_t)L.row * P.w8;
        for (int k = 0; k < nb8 && col0 + k < P.w8; ++k) {
            if constexpr (EG::kSpread) store_agent(line + col0 + k, ld.dA[k]);
            else line[col0 + k] = ld.dA[k];
        }
    }
    const bool last_in_pic = L.row == P.hctb - 1 && L.c == P.wctb - 1;
    // end_of_slice_segment_flag = 1 at the picture's last CTU (unless a tile's
    // substream goes on: SP_SUBSET_END) and at the end of a row that ends a slice segment
    const bool seg_end = !last_in_pic && L.c == P.wctb - 1 && (P.flags & SP_ROW_SEGMENTS) &&
                         (E.a->rsubs[P.sub_first + L.row] & SUB_SEG_END);
    const bool eos = (last_in_pic && !(P.flags & SP_SUBSET_END)) || seg_end;
    // inside a row of a picture with dependent segments starting inside rows,
    // end_of_slice_segment_flag = 1 ends one: the next starts at the next CTU
    if (term(L, G) != (eos ? 1 : 0)) {
        // end_of_slice_segment_flag = 1 inside a row: a dependent segment starts
        // at the next CTU (unit_ctu checks that the picture has one)
        if constexpr (EG::kSolo) L.status |= ST_SUBSTREAM_END;
        else L.status |= (!eos && L.c < P.wctb - 1) ? ST_SEGSW : (uint32_t)ST_SUBSTREAM_END;
    }
    if (!eos && (last_in_pic || ((L.fl & F_WPP) && L.c == P.wctb - 1)) && !term(L, G)) L.status |= ST_SUBSTREAM_END;
    if (L.budget + L.k < 0) L.status |= ST_OVERRUN;  // read past the NAL unit
    ++L.c;
    const uint32_t pv = (L.fl & F_STOP) ? kProgDone : (uint32_t)L.row * (uint32_t)P.wctb + (uint32_t)L.c;
    if constexpr (EG::kSpread) {
        if (E.a->xntu) {  // k_intra's streaming mode reads this row's records as they appear
            // the records (agent-scope stores: PF_COHERENT) before the count: an
            // agent release, which k_intra_stream's acquire after its poll pairs with
            HG_REL_AGENT();
            store_agent(E.a->xntu + P.row_off + L.row, L.ntu);
        }
        // The rule that makes vmcnt(0) enough here: every word the row below
        // reads after this progress word (the context hand-off, SAO parameters,
        // the depth line) went out above as an agent-scope store (store_agent,
        // coherent at L2 across XCDs), so completing them orders them.  A plain
        // store into hand-off data would need HG_REL_AGENT() (L2 write-back) here.
        stores_done();
        store_agent(prog_word(E, P, L.row), pv);
    } else {
        release_fence();
        prog_store(prog_word(E, P, L.row), pv);
    }
    if (!(L.fl & F_STOP) && L.c < P.wctb) {
        L.st = U_CTU;
        return;
    }
    uint32_t *rc = E.a->row_counts + 2 * (size_t)(P.row_off + L.row);
    rc[0] = L.ntu;
    rc[1] = L.ncoef;
    const int step = (L.fl & F_WPP) ? P.R : 1;  // one substream (no WPP): walk on to the next row
    if (!(L.fl & F_STOP) && L.row + step < P.hctb) {
        L.row += step;
        L.c = 0;
        row_outputs(L, P);
        L.st = U_CTU;
        return;
    }
    // (ST_SEGSW: never reported; the scalar engines never set it)
    const uint32_t st_rep = EG::kSolo ? L.status : (L.status & ~ST_SEGSW);
    if (st_rep) atomicOr(&E.a->status[P.pic], st_rep);
    L.st = U_DONE;
}

// Runs unit `kind` on this lane (the caller passes a wave-uniform kind and
// only lanes in that unit).  One unit kind per pass keeps the dispatch a
// uniform branch: a divergent switch over the units would linearise them, and
// every L field a unit updates would then need a register per unit.
template <class EG>
HG_HD inline void run_unit(int kind, Lane &L, LaneLds &ld, LanePic &P, const Env &E, const EG &G) {
    if constexpr (EG::kSolo) {
        if (L.fl & F_REINIT) {  // after PCM samples: the driver has moved the window to L.reinit
            engine_init(L, G, L.reinit, P.bits_end);
            L.fl &= ~F_REINIT;
        }
    }
    switch (kind) {
    case U_SB: unit_sb(L, ld, P, G); break;
    case U_TB: unit_tb(L, ld, P, G); break;
    case U_TT: unit_tt(L, ld, P, G); break;
    case U_CU: unit_cu(L, ld, P, G); break;
    case U_CQT: unit_cqt(L, ld, P, G); break;
    case U_CTU: unit_ctu(L, ld, P, E, G); break;
    case U_CTU_END: unit_ctu_end(L, ld, P, E, G); break;
    default: break;
    }
}

// a lane in U_CTU can start its CTU (WPP: the row above is two CTUs ahead)
template <class EG = Eng>
HG_HD inline bool ctu_ready(const Lane &L, const LanePic &P, const Env &E) { return wpp_ready<EG>(L, P, E); }

// lane setup: picture constants, outputs, first state.  Returns false for an idle lane.
// `cap` lanes (waves, solo mode) at most per picture.
// (Mid: the lanes engine, which keeps the picture's count of segment starts
// inside rows in P.flags; the scalar engines do not take such pictures)
template <bool Mid = true>
HG_HD inline bool pic_init(LanePic &P, const BatchArgs &a, int pic, int lane0, int cap) {
    const PicDesc &pd = a.pics[pic];
    if (pd.flags & PD_ASSEMBLY) return false;  // no coded data of its own
    const SeqParams &sp = a.seqs[pd.seq];
    const int log2ctb = sp.log2_ctb, ctb = 1 << log2ctb;
    const int hctb = (sp.height + ctb - 1) >> log2ctb;
    const bool wpp = (sp.flags & SP_WPP) != 0;
    const int R = wpp ? (hctb < cap ? hctb : cap) : 1;
    P.R = R;
    P.lane0 = lane0;
    P.ring = wpp && hctb > R;
    P.W = sp.width;
    P.H = sp.height;
    P.log2ctb = log2ctb;
    P.wctb = (sp.width + ctb - 1) >> log2ctb;
    P.hctb = hctb;
    P.minCb = sp.log2_min_cb;
    P.minTb = sp.log2_min_tb;
    P.maxTb = sp.log2_max_tb;
    P.maxDepthIntra = sp.max_th_depth_intra;
    P.chroma = sp.chroma_format;
    P.subx = (sp.chroma_format == 1 || sp.chroma_format == 2) ? 1 : 0;
    P.suby = sp.chroma_format == 1 ? 1 : 0;
    P.log2qg = log2ctb - sp.diff_cu_qp_delta_depth;
    P.bdY = sp.bit_depth_y;
    P.bdC = sp.bit_depth_c;
    P.qpbdY = 6 * (sp.bit_depth_y - 8);
    P.qpbdC = 6 * (sp.bit_depth_c - 8);
    P.pcmMin = sp.log2_min_pcm;
    P.pcmMax = sp.log2_max_pcm;
    P.pcmBdY = sp.pcm_bd_y;
    P.pcmBdC = sp.pcm_bd_c;
    P.cbOff = sp.cb_qp_offset + pd.cb_qp_off;
    P.crOff = sp.cr_qp_offset + pd.cr_qp_off;
    P.sliceQp = pd.slice_qp;
    P.w4 = (sp.width + 3) >> 2;
    P.h4 = (sp.height + 3) >> 2;
    P.w8 = (sp.width + 7) >> 3;
    P.saoL = pd.sao_luma;
    P.saoC = pd.sao_chroma;
    // (bits 16-30: the picture's segment starts inside rows, PicDesc.flags; lanes_nmid)
    P.flags = sp.flags | (a.xntu ? PF_COHERENT : 0u) | (Mid ? pd.flags & (PD_NMID_MAX << PD_NMID_SHIFT) : 0u);
    P.bits_off = (uint32_t)pd.bits_off;
    P.bits_end = (uint32_t)pd.bits_off + a.rsubs[pd.sub_first + pd.n_sub];  // RBSP end (k_rbsp)
    P.sub_first = pd.sub_first;
    P.row_off = pd.row_off;
    P.tu_cap = pd.tu_cap_row;
    P.coef_cap = pd.coef_cap_row;
    P.pic = (uint32_t)pic;
    P.gqpy = (int8_t HG_GAS *)(a.maps + pd.map_off);
    P.gflags = (uint8_t HG_GAS *)(a.maps + pd.map_off + (size_t)P.w4 * P.h4);
    P.gdepth = (uint8_t HG_GAS *)(a.maps + pd.map_off + 2 * (size_t)P.w4 * P.h4);
    P.gsao = (SaoParams HG_GAS *)(a.sao + pd.sao_off);
    P.tu_base = (TuRec HG_GAS *)(a.tus + pd.tu_off);
    P.coef_base = (Coef HG_GAS *)(a.coefs + pd.coef_off);
    return true;
}

// lane state at the start of substream `row` of picture P
HG_HD inline void lane_start(Lane &L, const LanePic &P, LaneLds &ld, int row) {
    L.status = 0;
    L.cn = 0;
    L.k = 8;
    L.ai = L.bv = L.fp = 0;
    L.lb = 0;
    L.fl = (P.flags & SP_WPP) ? F_WPP : 0u;  // (no segment started inside a row yet: bits 16-31)
    L.row = row;
    L.c = 0;
    L.qp_prev_last = P.sliceQp;
    row_outputs(L, P);
    L.st = U_CTU;
}

template <bool Mid = true>
HG_HD inline bool lane_init(Lane &L, LanePic &P, LaneLds &ld, const BatchArgs &a, int pic, int row, int lane0,
                            int cap) {
    if (!pic_init<Mid>(P, a, pic, lane0, cap) || row >= P.R) return false;
    lane_start(L, P, ld, row);
    return true;
}

// pictures per wave: a picture's lanes (BatchArgs::lane_rows) are consecutive.
// A wave's time is its pictures' WPP chains times the cost of a pass, and a
// pass costs more with more pictures' lanes in it (more unit kinds and longer
// divergent loops), so a batch that cannot fill every SIMD takes the fewest
// pictures per wave that still fit one wave per SIMD (single 4032x3024
// image on MI355X: parse 85 -> 66 ms at 1 picture per wave instead of 4);
// a full batch packs 64 lanes (config 4: 1536 waves).  HEIFGPU_LANES_PPW
// forces a value (tuning); HEIFGPU_PARSE_ADAPT=0 always packs.
inline int lanes_simds() {
    static const int simds = [] {
        const char *e = std::getenv("HEIFGPU_PARSE_SIMDS");
        if (e) return std::atoi(e);
#if !defined(HG_HOST_EMU)
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
            return 4 * cus;
#endif
        return 1024;
    }();
    return simds;
}
inline int lanes_pics_per_wave(int lane_rows, int n_pics) {
    static const int forced = [] {
        const char *e = std::getenv("HEIFGPU_LANES_PPW");
        return e ? std::atoi(e) : 0;
    }();
    static const bool adapt = [] {
        const char *e = std::getenv("HEIFGPU_PARSE_ADAPT");
        return !e || std::atoi(e) != 0;
    }();
    const int full = 64 / (lane_rows < 1 ? 1 : (lane_rows > 64 ? 64 : lane_rows));
    if (forced > 0) return forced < full ? forced : full;
    if (adapt && n_pics > 0) {
        const long S = lanes_simds();
        for (int p = 1; p < full; ++p)
            if ((n_pics + p - 1) / p <= S) return p;
        // No packing fits one wave per SIMD: the fewest pictures per wave that
        // fit two per SIMD (k_parse_lanes' VGPRs allow two), so no SIMD holds
        // two waves while others hold one.  Config 4 (6144 pictures): 3 per
        // wave, 2048 waves; r04 A/B: parse alone 70.3 -> 64.6 ms, beside the
        // reconstruction 78.4 -> 73.4, step 85.9 -> 85.4 ms.
        for (int p = 1; p < full; ++p)
            if ((n_pics + p - 1) / p <= 2 * S) return p;
    }
    return full;
}

}  // namespace

#if HG_PARSE_WANT_LANES  // (the host-side choices live in the lanes translation unit)
// Wave slot -> picture.  A wave runs until its heaviest picture is parsed,
// and every extra busy picture in it adds divergent units to each pass, so
// the critical path is the wave holding the most work.  Pictures are sorted
// by payload size and dealt snake-wise (wave w of W gets ranks w, 2W-1-w,
// 2W+w, 4W-1-w, ...): heavy beside light.  Empty slots are ~0u.
// HEIFGPU_PARSE_ORDER=0: batch order (kept for the emulation test of an
// unsorted dealing).  (r06 A/B, DESIGN 5.13: dealing by WPP critical path, or
// the lightest pictures beside each wave's heaviest, won only where a wave's
// companions repeat one bitstream, on the permuted halfmoonbay shard; on
// distinct tiles both were neutral or worse, so snake dealing stays.  The
// dispatcher puts waves w and w + W/2 on one SIMD; pairing the heaviest wave
// with the lightest moved nothing, and the heaviest pictures two per wave (the
// rest four) lost 7.7 %: a wave's time is its heaviest picture's chain.)
int lanes_parse_order(const PicDesc *pics, int n, int lane_rows, int ppw_force, std::vector<uint32_t> &order) {
    static const int on = [] {
        const char *e = std::getenv("HEIFGPU_PARSE_ORDER");
        return e ? std::atoi(e) : 1;
    }();
    const int full = 64 / (lane_rows < 1 ? 1 : (lane_rows > 64 ? 64 : lane_rows));
    const int ppw = ppw_force > 0 ? std::min(ppw_force, full) : lanes_pics_per_wave(lane_rows, n);
    if (!on || n <= 0) {
        order.resize((size_t)n);
        for (int i = 0; i < n; ++i) order[(size_t)i] = (uint32_t)i;
        order.resize((size_t)((n + ppw - 1) / ppw) * ppw, ~0u);
        return ppw;
    }
    std::vector<uint32_t> by_size;  // assembly pictures have nothing to parse: no slot
    for (int i = 0; i < n; ++i)
        if (!(pics[i].flags & PD_ASSEMBLY)) by_size.push_back((uint32_t)i);
    n = (int)by_size.size();
    std::stable_sort(by_size.begin(), by_size.end(),
                     [&](uint32_t x, uint32_t y) { return pics[x].bits_len > pics[y].bits_len; });
    const int W = (n + ppw - 1) / ppw;
    order.assign((size_t)W * ppw, ~0u);
    for (int r = 0; r < n; ++r) {
        const int band = r / W, pos = r % W;
        const int w = (band & 1) ? W - 1 - pos : pos;
        order[(size_t)w * ppw + band] = by_size[(size_t)r];
    }
    return ppw;
}

// Parse mode of a batch.  Spread mode parses each substream on a wave of its
// own (every lane alike, so one syntax unit at a time with nothing else in
// the pass), one workgroup per substream so a picture's rows spread over CUs:
// far faster per substream than a lane of a packed wave, but 64 lanes do one
// substream's work, so it is the latency path of small and middle batches,
// where packed waves cannot fill the SIMDs anyway.  MI355X, halfmoonbay
// permutations, row-major spread against lanes (profiles/r06/ab/ab_mid.txt,
// Mpix/s): 4 images 1,677 / 910, 16 4,711 / 2,864, 32 6,787 / 6,174, 64 7,819
// / 11,135; distinct tiles at 32 images 7,683 / 7,768.  So batches up to 1536
// pictures (32 such images) take spread mode.  HEIFGPU_PARSE=lanes|solo|spread
// forces a mode for every batch, HEIFGPU_SOLO_MAX_PICS moves the switch-over.
int parse_mode_for(int requested, int n_pics, const PicDesc *pics) {
    if (pics)
        for (int i = 0; i < n_pics; ++i)
            if (pics[i].flags >> PD_NMID_SHIFT) return PARSE_LANES;
    static const int env = [] {
        const char *e = std::getenv("HEIFGPU_PARSE");
        if (!e) return PARSE_AUTO;
        const std::string v(e);
        return v == "solo"     ? PARSE_SOLO
               : v == "spread" ? PARSE_SPREAD
               : v == "lanes"  ? PARSE_LANES
                               : PARSE_AUTO;
    }();
    static const int max_pics = [] {
        const char *e = std::getenv("HEIFGPU_SOLO_MAX_PICS");
        return e ? std::atoi(e) : 1536;
    }();
    if (env != PARSE_AUTO) return env;
    if (requested == PARSE_LANES || requested == PARSE_SOLO || requested == PARSE_SPREAD)
        return requested;
    return n_pics <= max_pics ? PARSE_SPREAD : PARSE_LANES;
}

// waves per solo workgroup: one per WPP row of the tallest picture, at most 16
// (1024 threads); taller pictures wrap their rows round the waves
int solo_waves_for(int lane_rows) { return lane_rows < 1 ? 1 : (lane_rows > kSoloMaxWaves ? kSoloMaxWaves : lane_rows); }

// spread mode: one wave slot per substream, entry row << 20 | picture, in
// row-major order: row r of every picture (heaviest picture first) before row
// r + 1 of any.  A row's wave holds its slot (and its SIMD residency) from the
// dequeue until the row is parsed; picture-major order (a picture's rows in
// consecutive slots) filled the resident waves with rows waiting on the WPP
// ramp of their own picture, row-major order finds the row above long started.
// r06 A/B: 16 images 3,474 -> 4,711 Mpix/s, 32 images 3,847 ->
// 6,787 (distinct tiles: 3,709 -> 6,651 and 3,994 -> 7,683), one image equal.
// A row's predecessor keeps a lower slot, held by a running wave
// (k_parse_solo<true> takes its slot from the job counter).
int spread_parse_order(const PicDesc *pics, int n, std::vector<uint32_t> &order) {
    std::vector<uint32_t> by_size((size_t)n);
    for (int i = 0; i < n; ++i) by_size[(size_t)i] = (uint32_t)i;
    std::stable_sort(by_size.begin(), by_size.end(),
                     [&](uint32_t x, uint32_t y) { return pics[x].bits_len > pics[y].bits_len; });
    order.clear();
    uint32_t max_sub = 0;
    for (uint32_t p : by_size) {
        if (p >= (1u << 20) || pics[p].n_sub >= (1u << 12)) return -1;
        max_sub = std::max(max_sub, pics[p].n_sub);
    }
    for (uint32_t r = 0; r < max_sub; ++r)
        for (uint32_t p : by_size)
            if (r < pics[p].n_sub) order.push_back(p | (r << 20));
    return 1;
}

#endif  // HG_PARSE_WANT_LANES

#if defined(HG_HOST_EMU)
// one wave at a time, one unit per live lane per pass, lanes in order
void emu_parse_lanes(const BatchArgs &a) {
    const int ppw = a.parse_order && a.parse_group > 0 ? a.parse_group : lanes_pics_per_wave(a.lane_rows, a.n_pics);
    const int n_slots = a.parse_order ? a.n_slots : a.n_pics;
    const int waves = (n_slots + ppw - 1) / ppw;
    uint64_t tab[kTabRows], seq[15];
    uint8_t scan8[128];
    for (int i = 0; i < 64; ++i) scan8_tables(scan8, i);
    for (int i = 0; i < kTabRows; ++i) tab[i] = state_row_ctx(i);
    for (int i = 0; i < 15; ++i) seq[i] = sig_seq(i);
    std::vector<LaneLds> lds(64);
    std::vector<LanePic> pics(64);
    std::vector<Lane> lanes(64);
    std::vector<uint8_t> wctx(a.wpp_ring ? 64 * CTX_PAD : 0);
    uint32_t prog[64];
    static const bool stats = std::getenv("HEIFGPU_LANES_STATS") != nullptr;
    // modelling knob (emulation only): the unit kinds of one pass, in order, as
    // digits (default "1234567": U_CTU .. U_CTU_END once)
    static const std::string order = [] {
        const char *e = std::getenv("HEIFGPU_EMU_PASS_ORDER");
        return std::string(e && *e ? e : "1234567");
    }();
    for (int w = 0; w < waves; ++w) {
        for (int l = 0; l < 64; ++l) {
            prog[l] = 0;
            const int pl = l / a.lane_rows, row = l % a.lane_rows;
            const int slot = w * ppw + pl;
            const bool in = pl < ppw && slot < n_slots && (!a.parse_order || a.parse_order[slot] != ~0u);
            const int pic = a.pic0 + (in && a.parse_order ? (int)a.parse_order[slot] : slot);
            const bool live = in && lane_init(lanes[l], pics[pl], lds[l], a, pic, row, pl * a.lane_rows, a.lane_rows);
            if (!live) lanes[l].st = U_DONE;
        }
        Env E{&a, lds.data(), prog, a.wpp_ring ? wctx.data() : nullptr, 0};
        long passes = 0, units = 0, kruns = 0, kr[8] = {}, ku[8] = {};
        for (;; ++passes) {
            bool any = false, progressed = false;
            for (int l = 0; l < 64; ++l) any |= lanes[l].st != U_DONE;
            if (!any) break;
            for (int l = 0; l < 64; ++l)
                if (lanes[l].st != U_DONE) {
                    const LanePic &P = pics[l / a.lane_rows];
                    const Eng G{lds[l].ctx, tab, seq, a.rbsp, (P.bits_end + 64u) & ~3u, scan8, scan8 + 64};
                    q_refill(lanes[l], G);
                }
            // the kernel's pass: every unit kind in syntax order, each on the lanes in it
            for (const char ch : order) {
                const int kind = ch - '0';
                bool mine[64], anym = false;
                int cnt = 0;
                for (int l = 0; l < 64; ++l) {
                    E.lane = l;
                    mine[l] = lanes[l].st == kind && (kind != U_CTU || ctu_ready(lanes[l], pics[l / a.lane_rows], E));
                    anym |= mine[l];
                    cnt += mine[l] ? 1 : 0;
                }
                if (!anym) continue;
                ++kruns;
                ++kr[kind];
                ku[kind] += cnt;
                for (int l = 0; l < 64; ++l) {
                    Lane &L = lanes[l];
                    E.lane = l;
                    LanePic &P = pics[l / a.lane_rows];
                    if (!mine[l]) continue;
                    progressed = true;
                    ++units;
                    const Eng G{lds[l].ctx, tab, seq, a.rbsp, (P.bits_end + 64u) & ~3u, scan8, scan8 + 64};
                    run_unit(kind, L, lds[l], P, E, G);
                }
            }
            if (!progressed) {  // every live lane waits: cannot happen (the top row never waits)
                for (int l = 0; l < 64; ++l)
                    if (lanes[l].st != U_DONE) {
                        lanes[l].status |= ST_SUBSTREAM_END;
                        atomicOr(&a.status[pics[l / a.lane_rows].pic], lanes[l].status & ~ST_SEGSW);
                        lanes[l].st = U_DONE;
                    }
                break;
            }
        }
        if (stats) {
            printf("wave %d: %ld passes, %.1f units per pass, %ld kind runs, %.2f units per kind run\n", w, passes,
                   (double)units / passes, kruns, (double)units / kruns);
            printf("  runs");
            for (int k = U_CTU; k <= U_CTU_END; ++k) printf(" %ld", kr[k]);
            printf("\n  units");
            for (int k = U_CTU; k <= U_CTU_END; ++k) printf(" %ld", ku[k]);
            printf("\n");
        }
    }
}

// solo mode: each picture's rows (waves) round-robin, one unit per ready wave
// per round, with the GPU driver's window logic (SoloWin) per wave
template <bool Spread>
void emu_parse_solo(const BatchArgs &a) {
    using EG = EngSoloT<Spread>;
    const int NW = Spread ? a.max_rows : a.solo_waves;  // spread: every row of a picture its own wave
    const int n_slots = a.parse_order ? a.n_slots : a.n_pics;
    uint64_t seq[15];
    for (int i = 0; i < 15; ++i) seq[i] = sig_seq(i);
    std::vector<LaneLds> lds((size_t)NW);
    std::vector<Lane> lanes((size_t)NW);
    std::vector<uint8_t> wctx((size_t)NW * CTX_PAD);
    std::vector<uint32_t> wbuf((size_t)NW * 192);
    std::vector<SoloWin> wins((size_t)NW);
    LanePic P;
    uint32_t prog[64];
    for (int slot = 0; slot < n_slots; ++slot) {
        const bool in = !a.parse_order || a.parse_order[slot] != ~0u;
        if (!in) continue;
        // spread: one entry per row (row << 20 | picture); the picture's row-0 entry runs all its rows here
        const uint32_t ent = a.parse_order ? a.parse_order[slot] : (uint32_t)slot;
        if (Spread && (ent >> 20) != 0) continue;
        const int pic = a.pic0 + (int)(Spread ? (ent & 0xfffffu) : ent);
        for (int w = 0; w < NW; ++w) {
            prog[w] = 0;
            if (!lane_init<false>(lanes[(size_t)w], P, lds[(size_t)w], a, pic, w, 0, Spread ? (1 << 20) : NW))
                lanes[(size_t)w].st = U_DONE;
            wins[(size_t)w].w = &wbuf[(size_t)w * 192];
            wins[(size_t)w].f = &wbuf[(size_t)w * 192 + 128];
        }
        const uint32_t lim = (P.bits_end + 64u) & ~3u;
        if (Spread)
            for (int w = 0; w < P.R; ++w) a.xprog[P.row_off + (uint32_t)w] = 0;  // this picture's words only
        Env E = Spread ? Env{&a, lds.data(), a.xprog + P.row_off, a.xctx + (size_t)P.row_off * CTX_PAD, 0}
                       : Env{&a, lds.data(), prog, wctx.data(), 0};
        for (;;) {
            bool any = false, progressed = false;
            for (int w = 0; w < NW; ++w) {
                Lane &L = lanes[(size_t)w];
                if (L.st == U_DONE) continue;
                any = true;
                E.lane = w;
                if (L.st == U_CTU && !ctu_ready<EG>(L, P, E)) continue;
                progressed = true;
                SoloWin &sw = wins[(size_t)w];
                const uint32_t start = L.st == U_CTU ? substream_start<false>(L, P, a) : ~0u;
                if (start != ~0u) sw.restart(a.rbsp, start, lim, 0);
                else sw.advance(a.rbsp, L.lb, lim, 0);
                const EG G{lds[(size_t)w].ctx, 0u, 0u, seq, a.rbsp, lim, sw.view(), 0u, 0u, 0u};
                run_unit(L.st, L, lds[(size_t)w], P, E, G);
            }
            if (!any) break;
            if (!progressed) {
                for (int w = 0; w < NW; ++w)
                    if (lanes[(size_t)w].st != U_DONE) {
                        lanes[(size_t)w].status |= ST_SUBSTREAM_END;
                        atomicOr(&a.status[P.pic], lanes[(size_t)w].status);
                        lanes[(size_t)w].st = U_DONE;
                    }
                break;
            }
        }
    }
}

void emu_parse(const BatchArgs &a) {
    if (a.parse_mode == PARSE_SOLO) emu_parse_solo<false>(a);
    else if (a.parse_mode == PARSE_SPREAD) emu_parse_solo<true>(a);
    else emu_parse_lanes(a);
}
#else
// LDS of one wave: LaneLds per used lane, LanePic per picture, progress words,
// engine tables, and the WPP context staging when rows wrap
// kTabRows + 16 engine-table words, then the 8x8 scan and its inverse (128 bytes)
constexpr size_t kLaneTablesBytes = (kTabRows + 16) * sizeof(uint64_t) + 128;
inline size_t lanes_lds_bytes(int ppw, int lane_rows, bool ring) {
    return lane_blocks_bytes(ppw * lane_rows) + sizeof(LanePic) * (size_t)ppw + 64 * sizeof(uint32_t) +
           kLaneTablesBytes + (ring ? 64 * (size_t)CTX_PAD : 0);
}

// the job counter: lane 0 takes the next number, the wave shares it
__device__ __forceinline__ uint32_t dequeue_job(uint32_t *ctr) {
    uint32_t j = 0;
    if (__lane_id() == 0) j = atomicAdd(ctr, 1u);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)j);
}

#if HG_PARSE_WANT_LANES
// a register budget of 256 (2 waves per SIMD, the occupancy the VGPR floor
// below fixes anyway); 0 leaves it to the compiler
#if !defined(HG_PARSE_WPE)
#define HG_PARSE_WPE 2
#endif
#if HG_PARSE_WPE > 0
#define HG_PARSE_ATTR __attribute__((amdgpu_waves_per_eu(HG_PARSE_WPE)))
#else
#define HG_PARSE_ATTR
#endif
__global__ void __launch_bounds__(64) HG_PARSE_ATTR k_parse_lanes(BatchArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int ppw = a.parse_group;  // pictures per wave (launch_parse)
    const int nl = ppw * a.lane_rows;
    LaneLds *s_lds = reinterpret_cast<LaneLds *>(smem);
    LanePic *s_pic = reinterpret_cast<LanePic *>(smem + lane_blocks_bytes(nl));
    uint32_t *s_prog = reinterpret_cast<uint32_t *>(s_pic + ppw);
    uint64_t *s_tab = reinterpret_cast<uint64_t *>(s_prog + 64);
    uint64_t *s_seq = s_tab + kTabRows;
    uint8_t *s_scan = reinterpret_cast<uint8_t *>(s_seq + 16);
    uint8_t *s_wctx = a.wpp_ring ? s_scan + 128 : nullptr;
    const int lane = threadIdx.x;
#if HG_PARSE_SETPRIO > 0
    // the parse is the latency-critical stream: win issue arbitration against
    // the reconstruction kernels of the previous decode sharing the SIMD
    __builtin_amdgcn_s_setprio(HG_PARSE_SETPRIO);
#endif
#if !defined(HG_PARSE_NO_VGPR_FLOOR)
    // at least 176 VGPRs, so at most 2 parse waves per SIMD whatever the allocator
    // needs: at <= 168 a SIMD takes 3, the reconstruction kernels beside them find no
    // room and the step loses 7 % (A/B in DESIGN 5.11)
    asm volatile("" ::: "v175");
#endif
    for (int i = lane; i < kTabRows; i += 64) s_tab[i] = state_row_ctx(i);
    if (lane < 15) s_seq[lane] = sig_seq(lane);
    scan8_tables(s_scan, lane);
    const int pl = lane / a.lane_rows, row = lane % a.lane_rows;
    const int slot = (int)blockIdx.x * ppw + pl;
    const int n_slots = a.parse_order ? a.n_slots : a.n_pics;
    const bool in = pl < ppw && slot < n_slots && (!a.parse_order || a.parse_order[slot] != ~0u);
    const int pic = a.pic0 + (in && a.parse_order ? (int)a.parse_order[slot] : slot);
    Lane L;
    LaneLds &ld = s_lds[lane < nl ? lane : 0];
    LanePic &P = s_pic[pl < ppw ? pl : 0];
    s_prog[lane] = 0;
    const bool live = in && lane_init(L, P, ld, a, pic, row, pl * a.lane_rows, a.lane_rows);
    if (!live) L.st = U_DONE;
#if defined(HG_PARSE_PROF_SB)
    for (int k = 0; k < 6; ++k) L.psb[k] = 0;
#endif
    __syncthreads();
    const Env E{&a, s_lds, s_prog, s_wctx, lane};
#if defined(HG_NO_SCAN8)
    const Eng G{ld.ctx, s_tab, s_seq, a.rbsp, live ? (P.bits_end + 64u) & ~3u : 0u};
#else
    const Eng G{ld.ctx, s_tab, s_seq, a.rbsp, live ? (P.bits_end + 64u) & ~3u : 0u, s_scan, s_scan + 64};
#endif
#if defined(HG_PARSE_PROF)
    uint64_t pf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint64_t t_start = __builtin_amdgcn_s_memtime();
    const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();
#endif
#if defined(HG_PARSE_PROF)
    uint64_t pw = 0;                                // the passes' start (pass_wait, q_refill)
    uint32_t kc[U_CTU_END] = {0, 0, 0, 0, 0, 0, 0};  // passes that ran each unit kind
#endif
    for (uint32_t pass = 0;; ++pass) {
        if (!__any(L.st != U_DONE)) break;
#if defined(HG_PARSE_PROF)
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
        pass_wait();
        if (live) q_refill(L, G);
#if defined(HG_PARSE_PROF)
        pw += __builtin_amdgcn_s_memtime() - t0;
#endif
        // one pass: every unit kind in syntax order, each run by the lanes in it
        // (a uniform loop: the units are never linearised into one divergent region)
        bool progressed = false;
#pragma unroll
        for (int kind = U_CTU; kind <= U_CTU_END; ++kind) {
            const bool mine = L.st == kind && (kind != U_CTU || ctu_ready(L, P, E));
            if (!__any(mine)) continue;
            progressed = true;
#if defined(HG_PARSE_PROF)
            ++kc[kind - 1];
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            pf[7] += (uint64_t)__popcll(__ballot(mine));  // lanes running a unit
#endif
            if (mine) run_unit(kind, L, ld, P, E, G);
#if defined(HG_PARSE_PROF)
            const uint64_t t2 = __builtin_amdgcn_s_memtime();
            pf[kind <= U_CTU ? 2 : kind <= U_TT ? 3 : kind - 1] += t2 - t1;
#endif
        }
#if defined(HG_PARSE_PROF)
        ++pf[1];
#endif
        if (!progressed || pass > (1u << 30)) {  // every live lane waits: cannot happen (the top row never waits)
            if (L.st != U_DONE) {
                L.status |= ST_SUBSTREAM_END;
                atomicOr(&a.status[P.pic], L.status & ~ST_SEGSW);
            }
            break;
        }
    }
#if defined(HG_PARSE_PROF)
    pf[0] = __builtin_amdgcn_s_memtime() - t_start;
    if (lane == 0)
        for (int k = 0; k < 8; ++k) atomicAdd((unsigned long long *)&g_prof_lanes[k], (unsigned long long)pf[k]);
#if defined(HG_PARSE_PROF_SB)
    // the sub-block unit's phases (slots 8..13: header, sig loop, greater1/2,
    // signs + remainders + record, sig bins, -), the wave's time: one lane per run
    if (live) {
        for (int k = 0; k < 6; ++k) atomicAdd((unsigned long long *)&g_prof_lanes[8 + k], (unsigned long long)L.psb[k]);
        if (blockIdx.x < (unsigned)kWaveRecCap)  // and per wave (records 3 and 4 of the wave's breakdown)
            for (int k = 0; k < 6; ++k)
                atomicAdd((unsigned long long *)&g_ctu_t[kWaveRec + (3 + k / 3) * kWaveRecCap + blockIdx.x][k % 3],
                          (unsigned long long)L.psb[k]);
    }
#endif
    // per wave (the CTU-time slots, unused by this kernel): s_memrealtime at its start, its
    // duration and place, then the passes and its first three pictures (16 bits each; 0xffff: none)
    if (blockIdx.x < (unsigned)kCtuTimeCap) {
        const uint32_t p0 = (uint32_t)__builtin_amdgcn_readlane(in ? pic : 0xffff, 0);
        const uint32_t p1 = (uint32_t)__builtin_amdgcn_readlane(in ? pic : 0xffff, a.lane_rows < 64 ? a.lane_rows : 0);
        const uint32_t p2 =
            (uint32_t)__builtin_amdgcn_readlane(in ? pic : 0xffff, 2 * a.lane_rows < 64 ? 2 * a.lane_rows : 0);
        uint32_t hwid, xcc;  // where the wave ran: HW_ID (SIMD, CU, SH, SE) and the XCD
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        if (lane == 0) {
            g_ctu_t[blockIdx.x][0] = rt_start;
            // the wave's duration (low 32 bits), then HW_ID[15:0] and XCC_ID[3:0]
            g_ctu_t[blockIdx.x][1] = ((__builtin_amdgcn_s_memrealtime() - rt_start) & 0xffffffffu) |
                                     ((uint64_t)((hwid & 0xffffu) | ((xcc & 0xfu) << 16)) << 32);
            g_ctu_t[blockIdx.x][2] = (pf[1] & 0xffffu) | ((uint64_t)(p0 & 0xffffu) << 16) |
                                     ((uint64_t)(p1 & 0xffffu) << 32) | ((uint64_t)(p2 & 0xffffu) << 48);
            // the wave's own breakdown (tools/wave_times.py): s_memtime cycles of the
            // wave, per unit kind group (pf[2..6]), of the pass starts, the lanes x
            // units / 4, and the passes that ran each unit kind (16 bits each)
            if (blockIdx.x < (unsigned)kWaveRecCap) {
                uint64_t *r = &g_ctu_t[kWaveRec + blockIdx.x][0];
                uint64_t *r2 = &g_ctu_t[kWaveRec + kWaveRecCap + blockIdx.x][0];
                uint64_t *r3 = &g_ctu_t[kWaveRec + 2 * kWaveRecCap + blockIdx.x][0];
                r[0] = pf[0], r[1] = pf[2], r[2] = pf[3];
                r2[0] = pf[4], r2[1] = pf[5], r2[2] = pf[6];
                r3[0] = pw;
                r3[1] = (uint64_t)kc[0] | ((uint64_t)kc[1] << 16) | ((uint64_t)kc[2] << 32) | ((uint64_t)kc[3] << 48);
                r3[2] = (uint64_t)kc[4] | ((uint64_t)kc[5] << 16) | ((uint64_t)kc[6] << 32) |
                        (std::min<uint64_t>(pf[7] >> 2, 0xffffu) << 48);
            }
        }
    }
#endif
}

// Solo mode: one workgroup per picture, one wave per WPP row (rows beyond 16
// wrap round the waves).  All 64 lanes of a wave run the same substream in
// lockstep (identical state in every lane, so exec stays full: the window and
// state-row registers read with v_readlane are never left stale in inactive
// lanes by a copy the compiler placed inside a divergent region), and the
// lanes differ only in the window refill, where each loads its own dword.  WPP
// progress words and the row-to-row context copies are in the workgroup's
// LDS, so the 2-CTU lag needs no memory traffic; waves waiting for the row
// above sleep.
#endif  // HG_PARSE_WANT_LANES

#if HG_PARSE_WANT_SOLO
inline size_t solo_lds_bytes(int nw, bool ring) {
    return lane_blocks_bytes(nw) + sizeof(LanePic) + 64 * sizeof(uint32_t) + 16 * sizeof(uint64_t) +
           (ring ? (size_t)nw * CTX_PAD : 0);
}

// (r06: a 6-waves-per-SIMD register budget, 80 VGPRs with 36 B/lane of
// scratch, lost 4 % at 16 and 32 images and 0.5 % at one: DESIGN 5.13)
template <bool Spread>
__global__ void __launch_bounds__(Spread ? 64 : 64 * kSoloMaxWaves) k_parse_solo(BatchArgs a) {
    using EG = EngSoloT<Spread>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int NW = Spread ? 1 : a.solo_waves;
    LaneLds *s_lds = reinterpret_cast<LaneLds *>(smem);
    LanePic *s_pic = reinterpret_cast<LanePic *>(smem + lane_blocks_bytes(NW));
    uint32_t *s_prog = reinterpret_cast<uint32_t *>(s_pic + 1);
    uint64_t *s_seq = reinterpret_cast<uint64_t *>(s_prog + 64);
    uint8_t *s_wctx = a.wpp_ring ? reinterpret_cast<uint8_t *>(s_seq + 16) : nullptr;
    // wave index made scalar: every value of the substream state derives from uniform inputs, so the
    // compiler can keep the engine in SGPRs and branch with s_cbranch
    const int w = Spread ? 0 : __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), lane = (int)threadIdx.x & 63;
#if HG_PARSE_SETPRIO > 0
    // the substream chain wins issue arbitration against k_intra_stream's waves on its SIMD
    __builtin_amdgcn_s_setprio(HG_PARSE_SETPRIO);
#endif
    if (threadIdx.x < 15) s_seq[threadIdx.x] = sig_seq((int)threadIdx.x);
    if (threadIdx.x < 64) s_prog[threadIdx.x] = 0;
    const uint64_t trow = state_row(lane);
    const uint32_t tlo = (uint32_t)trow, thi = (uint32_t)(trow >> 32);
    const uint32_t scan8v = (uint32_t)kScanPos[3][0][lane] | ((uint32_t)kScanInv[3][0][lane] << 8);
    const uint64_t sq = lane < 15 ? sig_seq(lane) : 0;
    const uint32_t sqlo = (uint32_t)sq, sqhi = (uint32_t)(sq >> 32);
    // spread: the slot from the job counter (a row's predecessor is the slot
    // before it, so it is already held by a running wave whatever order the
    // workgroups are dispatched in); solo: the workgroup's own picture
    const int slot = Spread ? (int)dequeue_job(a.xjob) : (int)blockIdx.x;
    const int n_slots = a.parse_order ? a.n_slots : a.n_pics;
    const uint32_t ent = slot < n_slots ? (a.parse_order ? a.parse_order[slot] : (uint32_t)slot) : ~0u;
    const bool in = ent != ~0u;
    // spread: entry = row << 20 | picture, one wave per WPP row
    const int pic = a.pic0 + (int)(Spread ? (ent & 0xfffffu) : ent), row = Spread ? (int)(ent >> 20) : w;
    Lane L;
    LaneLds &ld = s_lds[w < NW ? w : 0];
    LanePic &P = s_pic[0];
    const bool live = in && w < NW && lane_init<false>(L, P, ld, a, pic, row, 0, Spread ? (1 << 20) : NW);  // every lane alike
    if (!live) L.st = U_DONE;
#if defined(HG_PARSE_PROF_SB)
    for (int k = 0; k < 6; ++k) L.psb[k] = 0;
#endif
    __syncthreads();
    if (!__builtin_amdgcn_readfirstlane(live ? 1 : 0)) return;
    const Env E = Spread ? Env{&a, s_lds, a.xprog + P.row_off, a.xctx + (size_t)P.row_off * CTX_PAD, row}
                         : Env{&a, s_lds, s_prog, s_wctx, w};
    const uint32_t lim = (P.bits_end + 64u) & ~3u;
    SoloWin sw;
    sw.r0 = sw.r1 = sw.f = 0;
    sw.ck = 0;
#if defined(HG_PARSE_PROF)
    uint64_t pf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint64_t t_start = __builtin_amdgcn_s_memtime();
    int want_seen = -1;  // the CTU whose want time is recorded
#endif
#if defined(HG_PARSE_PROF_SB)
    uint64_t pw[2] = {0, 0};  // cycles of not-run iterations (WPP polls + sleeps); driver cycles of run ones
#endif
    uint32_t stalled = 0;  // consecutive not-run iterations (bounded: never hang the device)
    for (;;) {
#if defined(HG_PARSE_PROF_SB)
        const uint64_t t_top = __builtin_amdgcn_s_memtime();
#endif
        // the wave's state (equal in every lane), made scalar
        int st = L.st, run = st != U_DONE && (st != U_CTU || ctu_ready<EG>(L, P, E));
#if defined(HG_PARSE_PROF)
        const int tix = (P.row_off + L.row) * 128 + L.c;
        if (st == U_CTU && L.c < 128 && tix < kCtuTimeCap) {
            const uint64_t now = __builtin_amdgcn_s_memrealtime();  // chip-wide 100 MHz clock
            if (want_seen != tix && lane == 0) g_ctu_t[tix][0] = now;
            want_seen = tix;
            if (run && lane == 0) g_ctu_t[tix][1] = now;
        }
#endif
        uint32_t start = run && st == U_CTU ? substream_start<false>(L, P, a) : ~0u;
        const uint32_t rd = L.lb;
        st = __builtin_amdgcn_readfirstlane(st);
        if (st == U_DONE) break;
        if (!__builtin_amdgcn_readfirstlane(run)) {
            // the row above is not 2 CTUs ahead: sleep (~64 cycles a unit), so the
            // busy waves on this SIMD keep the issue slots
            __builtin_amdgcn_s_sleep(HG_SOLO_SLEEP);
#if defined(HG_PARSE_PROF_SB)
            pw[0] += __builtin_amdgcn_s_memtime() - t_top;
#endif
            // a row waits at most one picture's parse (~1e6 iterations); far past
            // that the row above can never arrive (a dispatch-order assumption
            // broken): flag the picture and stop instead of spinning forever
            if (++stalled > (1u << 25)) {
                if (lane == 0) atomicOr(&a.status[P.pic], L.status | ST_SUBSTREAM_END);
                // publish the row as finished (the TU count as it stands), so the
                // rows below and k_intra_stream stop waiting on it at once
                if (Spread) {
                    if (a.xntu) store_agent(a.xntu + P.row_off + L.row, L.ntu);
                    stores_done();
                    store_agent(prog_word(E, P, L.row), kProgDone);
                }
                break;
            }
            continue;
        }
        stalled = 0;
        start = (uint32_t)__builtin_amdgcn_readfirstlane((int)start);
        if (start != ~0u) sw.restart(a.rbsp, start, lim, lane);
        else sw.advance(a.rbsp, (uint32_t)__builtin_amdgcn_readfirstlane((int)rd), lim, lane);
        // the rows above (contexts, SAO parameters, depth line: other workgroups'
        // agent-scope stores) after their progress words, before their readers
        if (st == U_CTU) {
            if (Spread) HG_ACQ_AGENT();
            else HG_FENCE_ACQ();
        }
#if defined(HG_PARSE_PROF)
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        ++pf[7];
#endif
        {
#if !defined(HG_SOLO_NO_UNI)
            uni_state(L);
#endif
            const EG G{ld.ctx, tlo, thi, s_seq, a.rbsp, lim, sw.view(), sqlo, sqhi, scan8v};
#if defined(HG_PARSE_PROF)
            const int eix = (P.row_off + L.row) * 128 + L.c;
#endif
            run_unit(st, L, ld, P, E, G);
#if defined(HG_PARSE_PROF)
            if (st == U_CTU_END && eix < kCtuTimeCap && lane == 0) g_ctu_t[eix][2] = __builtin_amdgcn_s_memrealtime();
#endif
        }
#if defined(HG_PARSE_PROF)
#if defined(HG_PARSE_PROF_SB)
        pw[1] += t1 - t_top;
#else
        pf[st <= U_CTU ? 2 : st <= U_TT ? 3 : st - 1] += __builtin_amdgcn_s_memtime() - t1;
        ++pf[1];
#endif
#endif
    }
#if defined(HG_PARSE_PROF_SB)
    for (int k = 0; k < 6; ++k) pf[2 + k] = L.psb[k];
    pf[1] = pw[0];
    if (lane == 0) atomicAdd((unsigned long long *)&g_prof_lanes[8], (unsigned long long)pw[1]);
#endif
#if defined(HG_PARSE_PROF)
    pf[0] = __builtin_amdgcn_s_memtime() - t_start;
    if (lane == 0)
        for (int k = 0; k < 8; ++k) atomicAdd((unsigned long long *)&g_prof_lanes[k], (unsigned long long)pf[k]);
#endif
}

// the solo and spread modes (launch_parse)
hipError_t launch_parse_solo(const BatchArgs &a, hipStream_t s) {
    if (a.parse_mode == PARSE_SOLO) {
        if (a.solo_waves < 1 || a.solo_waves > kSoloMaxWaves) return hipErrorInvalidValue;
        const int n = a.parse_order ? a.n_slots : a.n_pics;
        if (n <= 0) return hipSuccess;
        hipLaunchKernelGGL(k_parse_solo<false>, dim3(n), dim3(64 * a.solo_waves),
                           solo_lds_bytes(a.solo_waves, a.wpp_ring != 0), s, a);
        return hipGetLastError();
    }
    if (!a.parse_order || !a.xprog || !a.xctx || !a.xjob) return hipErrorInvalidValue;
    if (a.n_slots <= 0) return hipSuccess;
    // (the progress words start at 0: k_rbsp of this decode cleared them)
    hipLaunchKernelGGL(k_parse_solo<true>, dim3(a.n_slots), dim3(64), solo_lds_bytes(1, false), s, a);
    return hipGetLastError();
}
#endif  // HG_PARSE_WANT_SOLO

#if HG_PARSE_WANT_LANES
hipError_t launch_parse_solo(const BatchArgs &a, hipStream_t s);

hipError_t launch_parse(const BatchArgs &a0, hipStream_t s) {
    BatchArgs a = a0;
    if (a.lane_rows < 1 || a.lane_rows > 64) return hipErrorInvalidValue;
    if (a.parse_mode == PARSE_SOLO || a.parse_mode == PARSE_SPREAD) return launch_parse_solo(a, s);
    // the dealing of parse_order fixed the pictures per wave (lanes_parse_order)
    const int ppw = a.parse_order && a.parse_group > 0 ? a.parse_group : lanes_pics_per_wave(a.lane_rows, a.n_pics);
    a.parse_group = ppw;
    const int waves = ((a.parse_order ? a.n_slots : a.n_pics) + ppw - 1) / ppw;
    hipLaunchKernelGGL(k_parse_lanes, dim3(waves), dim3(64), lanes_lds_bytes(ppw, a.lane_rows, a.wpp_ring != 0), s, a);
    return hipGetLastError();
}
#endif  // HG_PARSE_WANT_LANES
#endif

}  // namespace hg

#if !defined(HG_HOST_EMU) && defined(HG_PARSE_PROF)
namespace hg {
namespace {
// this translation unit's counters (g_prof_lanes, g_ctu_t) copied out and zeroed
int prof_read(uint64_t *out, int n) {
    uint64_t tmp[16] = {};
    if (hipMemcpyFromSymbol(tmp, HIP_SYMBOL(hg::g_prof_lanes), sizeof(tmp)) != hipSuccess) return -1;
    const uint64_t zero[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(hg::g_prof_lanes), zero, sizeof(zero)) != hipSuccess) return -1;
#if defined(HG_PARSE_PROF_SB)
    const int head = 16;  // slots 16 on: g_ctu_t as in the prof build (the per-wave records)
#else
    const int head = 8;   // slots 8 on: the per-CTU times (3 per CTU) and the per-wave records
#endif
    for (int k = 0; k < n && k < head; ++k) out[k] = tmp[k];
    if (n <= head) return n < head ? n : head;
    const size_t m = std::min((size_t)(n - head), (size_t)hg::kCtuTimeCap * 3);
    if (hipMemcpyFromSymbol(out + head, HIP_SYMBOL(hg::g_ctu_t), m * sizeof(uint64_t)) != hipSuccess) return -1;
    std::vector<uint64_t> z((size_t)hg::kCtuTimeCap * 3, 0);
    if (hipMemcpyToSymbol(HIP_SYMBOL(hg::g_ctu_t), z.data(), z.size() * sizeof(uint64_t)) != hipSuccess) return -1;
    return (int)(head + m);
}
}  // namespace
}  // namespace hg
// The library builds the solo / spread kernels as a translation unit of their
// own (parse_solo.hip), whose device globals are a code object's own: their
// counters are read through this entry and added in heifgpu_debug_counters
#if defined(HG_PARSE_TU)
extern "C" int hg_debug_counters_solo(uint64_t *out, int n);
#if HG_PARSE_TU == 2
extern "C" int hg_debug_counters_solo(uint64_t *out, int n) { return hg::prof_read(out, n); }
#endif
#endif
#endif

#if !defined(HG_HOST_EMU) && HG_PARSE_WANT_LANES
// Tuning hook (include/heifgpu.h): copies out and zeroes k_parse_lanes'
// per-wave s_memtime counters.  Returns the number of counters written, or 0
// for the product library (counters compiled out; `make prof` has them).
extern "C" int heifgpu_debug_counters(uint64_t *out, int n) {
#if defined(HG_PARSE_PROF)
    const int r = hg::prof_read(out, n);
#if defined(HG_PARSE_TU)
    if (r > 0) {  // (one of the two kinds of kernel ran; the other's slots are zero)
        std::vector<uint64_t> o2((size_t)r, 0);
        const int r2 = hg_debug_counters_solo(o2.data(), r);
        if (r2 < 0) return -1;
        for (int k = 0; k < r2 && k < r; ++k) out[k] += o2[(size_t)k];
    }
#endif
    return r;
#else
    (void)out;
    (void)n;
    return 0;
#endif
}
#endif
