// intra.hip — intra sample prediction + reconstruction (pipeline stage 3).
//
// H.265 8.4.4.2.1-8.4.4.2.6 (neighbour availability via z-scan order 6.4.1,
// substitution, [1 2 1] / strong smoothing, planar, DC with edge filter,
// 33 angular modes with the mode-10/26 boundary filters) and 8.6.7
// (recSamples = Clip1(pred + res)).  The reference stops before any of this
// (src/hevc/slice.rs:253-255).
//
// Mapping: the serial part of HEVC intra decoding is the TB-to-TB
// dependency inside a CTU row.  One workgroup per picture, one wave per CTB
// row; row r starts CTU c once row r-1 has finished CTU c+1 (every
// above-right neighbour lies in CTU c+1 at most), signalled through per-wave
// progress counters in LDS with workgroup-scope release/acquire.
//
// Each wave reconstructs its current CTU in an LDS window: the CTU's samples,
// the column left of it (kept from the previous CTU), the row above it
// (2*ctb+1 samples incl. the corner and above-right, loaded once per CTU from
// the picture after the progress wait) and the CTU's residuals (one coalesced
// load per CTU).  Every TB then works on LDS only — neighbour gather,
// substitution (three 64-bit ballots + a nearest-available lookup),
// filtering, prediction and residual add run one sample per lane — and the
// finished CTU is written to the picture once.
#include "kernels.hpp"
#include "xform.hpp"
#if defined(HG_HOST_EMU)
#include <cstdio>
#include <cstdlib>
#endif

namespace hg {

namespace {

constexpr int kMaxWaves = 16;
constexpr int kResidentIntraWaves = 4096;  // ~16 per CU: enough pictures in flight to hide TB latency
constexpr size_t kIntraLdsBudget = 128 * 1024;

__constant__ int8_t c_angle[35] = {0, 0, 32, 26, 21, 17, 13, 9, 5, 2, 0, -2, -5, -9, -13, -17, -21, -26,
                                   -32, -26, -21, -17, -13, -9, -5, -2, 0, 2, 5, 9, 13, 17, 21, 26, 32};
__constant__ int16_t c_inv_angle[35] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, -4096, -1638, -910, -630, -482, -390, -315,
                                        -256, -315, -390, -482, -630, -910, -1638, -4096, 0, 0, 0, 0, 0, 0, 0, 0, 0};

struct alignas(16) IntraScratch {
    // TBs are at most 32x32 (MaxTbLog2SizeY <= 5): 2n + 1 <= 65 reference samples
    // per side.  Sized to that, not to the CTB, so more workgroups fit beside the
    // next decode's k_parse_lanes (which holds ~120 KB of each CU's LDS).
    int16_t left[66];  // [0] = p[-1][-1], [1+y] = p[-1][y]
    int16_t top[66];   // [0] = p[-1][-1], [1+x] = p[x][-1]
    int16_t fl[66];
    int16_t ft[66];
};

// Per-wave LDS block: scratch, then per component the CTU window.
struct WinLayout {
    int csx[3], csy[3];                          // component CTB width, height
    uint32_t cur[3], left[3], above[3], res[3];  // byte offsets in the block
    uint32_t bytes;                              // block size (16-aligned)
};

#if defined(HG_HOST_EMU)
inline
#else
__host__ __device__ inline
#endif
WinLayout win_layout(int log2ctb, int chroma, int bps) {
    WinLayout L{};
    uint32_t o = (uint32_t)((sizeof(IntraScratch) + 15) & ~size_t(15));
    const int ncomp = chroma ? 3 : 1;
    for (int k = 0; k < 3; ++k) {
        const int cx = k == 0 ? (1 << log2ctb) : (chroma ? (1 << log2ctb) >> chroma_sx(chroma) : 0);
        const int cy = k == 0 ? (1 << log2ctb) : (chroma ? (1 << log2ctb) >> chroma_sy(chroma) : 0);
        L.csx[k] = cx;
        L.csy[k] = cy;
        if (k >= ncomp) continue;
        L.cur[k] = o;
        o += (uint32_t)(cx * cy * bps + 15) & ~15u;
        L.left[k] = o;
        o += (uint32_t)(cy * bps + 15) & ~15u;
        L.above[k] = o;
        o += (uint32_t)((2 * cx + 1) * bps + 15) & ~15u;
        // residuals are read from the k_transform planes, not staged here: half
        // the block, so twice the workgroups fit beside the next decode's k_parse
        L.res[k] = 0;
    }
    L.bytes = o;
    return L;
}

int intra_waves(int log2ctb, int chroma, int bps, int max_rows) {
    const WinLayout L = win_layout(log2ctb, chroma, bps);
    int nw = (int)((kIntraLdsBudget - 64) / L.bytes);
    nw = nw < kMaxWaves ? nw : kMaxWaves;
    nw = nw < max_rows ? nw : max_rows;
    return nw < 1 ? 1 : nw;
}

#define wave_sync() HG_WAVE_SYNC()
// k_intra_stream's wait for the parse (tuning: HG_STREAM_SLEEP_N, s_sleep units of 64 clocks)
#if defined(HG_HOST_EMU) || !defined(HG_STREAM_SLEEP_N)
#define HG_STREAM_SLEEP() HG_SLEEP()
#else
#define HG_STREAM_SLEEP() __builtin_amdgcn_s_sleep(HG_STREAM_SLEEP_N)
#endif


// 6.4.1 availability of a neighbouring luma location (xl, yl) for a TB of the
// CTU at luma (bx0, by0), size csl.  Everything in the CTU row above (up to the
// above-right CTU, which the wavefront has finished) and in the CTU to the
// left is decoded; the CTUs below-left and right are not; inside the CTU a
// block is available iff it precedes the TB in z-scan order (MinTbAddrZs of
// 6.5.2 at 4x4 granularity: the CTU's quadtrees are decoded in z-order, so a
// 4x4 block is decoded before the TB iff its z-index is below the z-index zc
// of the TB's first luma 4x4 block).
__device__ __forceinline__ int zidx(int bx, int by) {  // bits of bx, by interleaved (bx, by < 16)
    auto spread = [](int v) {
        v = (v | (v << 2)) & 0x33;
        return (v | (v << 1)) & 0x55;
    };
    return spread(bx) | (spread(by) << 1);
}
// (r06 A/B: as one expression of bitwise ands / ors with the z-index always
// formed, k_intra VALU +0.45 G for SALU -0.2 G, the step not better: the early
// returns stay)
__device__ __forceinline__ bool nb_avail(int zc, int xl, int yl, int bx0, int by0, int csl) {
    const int lx = xl - bx0, ly = yl - by0;
    if (ly < 0) return true;
    if (ly >= csl || lx >= csl) return false;
    if (lx < 0) return true;
    return zidx(lx >> 2, ly >> 2) < zc;
}

// ref[k] of 8.4.4.2.6 read in place: the main-side neighbour for k >= 0, the
// projected side-side neighbour for k < 0 (only reached when
// (nTbS * intraPredAngle) >> 5 < -1, exactly where the spec extends ref)
// (r06 A/B: as an element index from one base, an integer select before one
// load: VALU +0.18 G with the two rows below, the step -0.3 %; not taken)
__device__ __forceinline__ const int16_t *ang_ref(const int16_t *main_, const int16_t *side, int inv, int k) {
    return k >= 0 ? main_ + k : side + ((k * inv + 128) >> 8);
}

// four samples as one store unit
template <typename Pel>
struct QuadT;
template <>
struct QuadT<uint8_t> {
    using type = uint32_t;
};
template <>
struct QuadT<uint16_t> {
    using type = uint64_t;
};
template <typename Pel>
using Quad = typename QuadT<Pel>::type;

// One component's CTU window in LDS.
template <typename Pel>
struct Win {
    Pel *cur, *left, *above;
    const int16_t *res;  // the component's residual plane (k_transform), or in streaming mode the
                         // current TB's residual in LDS
    int rp;              // residual pitch (the plane width; streaming mode: the TB width)
    int rx0, ry0;        // the sample res[0] holds (plane: 0, 0; streaming: the TB's origin)
    int csx, csy;        // CTB width, height in component samples (4:2:2 chroma: csy = 2 csx)
    int cx0, cy0;        // CTB origin in component samples
#if defined(HG_HOST_EMU)
    // emulation only: the LDS objects the pointers must stay inside (the r04
    // gain-map fault was a residual pointer moved before its LDS buffer, which
    // the host build could not see): the wave's window block, and the residual's
    // object when it is an LDS tile (null: a residual plane in global memory)
    const unsigned char *blk_lo = nullptr, *blk_hi = nullptr;
    const int16_t *res_lo = nullptr, *res_hi = nullptr;
    void check_blk(const void *p, size_t bytes) const {
        const unsigned char *q = static_cast<const unsigned char *>(p);
        if (blk_lo && (q < blk_lo || q + bytes > blk_hi)) {
            fprintf(stderr, "k_intra: window access %td bytes outside the wave's LDS block\n",
                    q < blk_lo ? q - blk_lo : q + bytes - blk_hi);
            abort();
        }
    }
    void check_res(const int16_t *p, size_t elems) const {
        if (res_lo && (p < res_lo || p + elems > res_hi)) {
            fprintf(stderr, "k_intra: residual access %td elements outside its LDS tile\n",
                    p < res_lo ? p - res_lo : p + elems - res_hi);
            abort();
        }
    }
#endif
    // a decoded neighbour (xn, yn) in picture coordinates; only called for
    // available samples, which lie in the row above, the column to the left
    // or the current CTU
    __device__ __forceinline__ int fetch(int xn, int yn) const {
        const int lx = xn - cx0, ly = yn - cy0;
#if defined(HG_HOST_EMU)
        check_blk(ly < 0 ? above + lx + 1 : lx < 0 ? left + ly : cur + ly * csx + lx, sizeof(Pel));
#endif
        if (ly < 0) return above[lx + 1];
        if (lx < 0) return left[ly];
        return cur[ly * csx + lx];
    }
};

// One picture's CTU windows, from which a component's Win is formed where it
// is used (a few scalar operations on the wave-uniform CTU and component)
// instead of being held: three Win and six plane pointers live across the TB
// loop kept k_intra at the 106-SGPR cap with 120-190 SGPRs spilled into VGPR
// lanes, a v_writelane / v_readlane per use.  The block
// layout is win_layout's: scratch, then per component the window, the left
// column and the row above, each 16-byte aligned.
template <typename Pel, int CF>
struct Frame {
    unsigned char *blk;    // the wave's window block (LDS)
    Pel *recon;            // the picture's Y plane; Cb, Cr follow
    const int16_t *resid;  // its Y residual plane (k_transform); Cb, Cr follow
    int W, H, cw, ch, log2ctb;
    uint32_t b0, b1;       // bytes of the Y and of one chroma component's part of the block
    static constexpr uint32_t al16(uint32_t v) { return (v + 15u) & ~15u; }
    static constexpr uint32_t kS0 = (uint32_t)((sizeof(IntraScratch) + 15) & ~size_t(15));
    __device__ __forceinline__ int csx(int k) const { return k ? (1 << log2ctb) >> chroma_sx(CF) : 1 << log2ctb; }
    __device__ __forceinline__ int csy(int k) const { return k ? (1 << log2ctb) >> chroma_sy(CF) : 1 << log2ctb; }
    __device__ __forceinline__ int pw(int k) const { return k ? cw : W; }
    __device__ __forceinline__ int ph(int k) const { return k ? ch : H; }
    __device__ __forceinline__ size_t plane_off(int k) const {
        return k ? (size_t)W * H + (k == 2 ? (size_t)cw * ch : 0) : 0;
    }
    __device__ __forceinline__ Pel *plane(int k) const { return recon + plane_off(k); }
    __device__ __forceinline__ void init(int log2, int w_, int h_, int cw_, int ch_) {
        log2ctb = log2, W = w_, H = h_, cw = cw_, ch = ch_;
        const uint32_t bps = sizeof(Pel), c0 = 1u << log2;
        b0 = al16(c0 * c0 * bps) + al16(c0 * bps) + al16((2 * c0 + 1) * bps);
        const uint32_t cx = CF ? c0 >> chroma_sx(CF) : 0, cy = CF ? c0 >> chroma_sy(CF) : 0;
        b1 = al16(cx * cy * bps) + al16(cy * bps) + al16((2 * cx + 1) * bps);
    }
    // component k's window at CTU column c of CTB row r
    __device__ __forceinline__ Win<Pel> win(int k, int c, int r) const {
        Win<Pel> w;
        const int sx = csx(k), sy = csy(k);
        const uint32_t cur = kS0 + (k ? b0 + (uint32_t)(k - 1) * b1 : 0u);
        const uint32_t left = cur + al16((uint32_t)(sx * sy) * sizeof(Pel));
        const uint32_t above = left + al16((uint32_t)sy * sizeof(Pel));
        w.cur = reinterpret_cast<Pel *>(blk + cur);
        w.left = reinterpret_cast<Pel *>(blk + left);
        w.above = reinterpret_cast<Pel *>(blk + above);
        w.res = resid + plane_off(k);
        w.rp = pw(k);
        w.rx0 = w.ry0 = 0;
        w.csx = sx;
        w.csy = sy;
        w.cx0 = c * sx;
        w.cy0 = r * sy;
#if defined(HG_HOST_EMU)
        w.blk_lo = blk;
        w.blk_hi = blk + kS0 + b0 + (CF ? 2 * b1 : 0u);
#endif
        return w;
    }
};

// Facts of one TB record that depend on the record and the picture only:
// formed for 64 records at once, one per lane, when the wave loads them (the
// per-TB checks on the scalar unit were a large part of k_intra's scalar
// instructions), read back with one v_readlane per TB.  Bit 0 (TBM_OK): the
// TB is this wave's component (cidx in [k0, k1)), has a mode of 8.4.2, and
// lies inside the picture and inside the window of CTB tu.ctu of row r (the
// parse keeps it so; the check keeps the tables in range).  Bit 1 (TBM_PAIR,
// set by the caller): a 4x4 / 8x8 Cb TB whose next record is its Cr TB.
// Bits 8-15: zc, the z-order index of the TB's first luma 4x4 block in its
// CTU (6.4.1 availability).
// Bit 2 (TBM_FILT): the TB's neighbours are filtered (8.4.4.2.3: luma, or
// chroma with 4:4:4; not DC, not 4x4; the mode farther from horizontal and
// vertical than the size's threshold).  A second word per record (tb_angle)
// holds intraPredAngle and invAngle (8.4.4.2.6), read by one vector load per
// 64 records instead of two scalar loads from constant memory per TB.
enum : uint32_t { TBM_OK = 1u, TBM_PAIR = 2u, TBM_FILT = 4u };
template <typename Pel, int CF>
__device__ __forceinline__ uint32_t tb_meta(const TuRec &q, const Frame<Pel, CF> &F, int r, int k0, int k1) {
    const int k = q.flags & TU_CIDX_MASK, n = 1 << q.log2;
    const int subx = k ? chroma_sx(CF) : 0, suby = k ? chroma_sy(CF) : 0;
    const int lcx = F.log2ctb - subx, lcy = F.log2ctb - suby;
    const int cx0 = (int)q.ctu << lcx, cy0 = r << lcy;
    const int PW = k ? F.cw : F.W, PH = k ? F.ch : F.H;
    const bool ok = k < (CF ? 3 : 1) && k >= k0 && k < k1 && q.mode <= 34 && q.log2 >= 2 && q.log2 <= 5 &&
                    q.x + n <= PW && q.y + n <= PH && q.x >= cx0 && q.y >= cy0 && q.x + n <= cx0 + (1 << lcx) &&
                    q.y + n <= cy0 + (1 << lcy);
    const int zc = ok ? zidx((((int)q.x - cx0) << subx) >> 2, (((int)q.y - cy0) << suby) >> 2) : 0;
    const int dist = min(abs((int)q.mode - 26), abs((int)q.mode - 10));
    const int thr = n == 8 ? 7 : (n == 16 ? 1 : 0);
    const bool filt = (k == 0 || CF == 3) && q.mode != 1 && n != 4 && dist > thr;
    return (ok ? TBM_OK : 0u) | (filt ? TBM_FILT : 0u) | ((uint32_t)zc << 8);
}
// intraPredAngle (low byte, signed) and invAngle (high half, signed) of a record's mode
__device__ __forceinline__ uint32_t tb_angle(const TuRec &q) {
    const int m = q.mode <= 34 ? q.mode : 0;
    return (uint32_t)(uint8_t)c_angle[m] | ((uint32_t)(uint16_t)c_inv_angle[m] << 16);
}

#if !defined(HG_HOST_EMU)
// the sum over the lanes of each aligned group of m (2 <= m <= 64, a power of
// two) lanes, in every lane of the group: ds_swizzle xor steps inside 32-lane
// halves (one LDS-crossbar instruction each, against __shfl_xor's address
// arithmetic and bounds select), ds_bpermute across them
__device__ __forceinline__ int group_sum(int v, int m) {
    if (m >= 64) v += __builtin_amdgcn_ds_bpermute(((int)__lane_id() ^ 32) << 2, v);
    if (m >= 32) v += __builtin_amdgcn_ds_swizzle(v, 0x1f | (16 << 10));
    if (m >= 16) v += __builtin_amdgcn_ds_swizzle(v, 0x1f | (8 << 10));
    if (m >= 8) v += __builtin_amdgcn_ds_swizzle(v, 0x1f | (4 << 10));
    if (m >= 4) v += __builtin_amdgcn_ds_swizzle(v, 0x1f | (2 << 10));
    return v + __builtin_amdgcn_ds_swizzle(v, 0x1f | (1 << 10));
}
#endif

template <typename Pel, int CF>
__device__ __attribute__((always_inline)) inline void predict_tb(IntraScratch *L, const TuRec &tu, const Win<Pel> &w,
                                                                 int PW, int PH, int cidx, int bd, bool strong,
                                                                 int zc, bool filt, uint32_t am, int lane) {
    constexpr int chroma = CF;
    const int log2n = tu.log2, n = 1 << log2n, mode = tu.mode;
    const int x0 = tu.x, y0 = tu.y;
    // component → luma coordinates (6.4.1 takes luma locations)
    const int subx = cidx ? chroma_sx(chroma) : 0, suby = cidx ? chroma_sy(chroma) : 0;
    const int bx0 = w.cx0 << subx, by0 = w.cy0 << suby, csl = w.csx << subx;
    const int ns = 4 * n + 1;
    const bool cbf = (tu.flags & TU_CBF) != 0;
    // residual of a 4x4 / 8x8 TB (one sample per lane): loaded now, used after
    // the neighbour and filter phases, so the load latency hides behind them
    // (the TB's first residual, formed only where it is in bounds: a pointer moved
    // before an LDS buffer is out of the object, and its flat address lost the aperture on the GPU)
    const int16_t *rt = cbf ? w.res + ((ptrdiff_t)(y0 - w.ry0) * w.rp + (x0 - w.rx0)) : w.res;
#if defined(HG_HOST_EMU)
    if (cbf) w.check_res(rt, (size_t)(n - 1) * w.rp + n);
    w.check_blk(w.cur + ((y0 - w.cy0) * w.csx + (x0 - w.cx0)), ((size_t)(n - 1) * w.csx + n) * sizeof(Pel));
#endif
    const int r0 = (cbf && n <= 8 && lane < n * n) ? rt[(lane >> log2n) * w.rp + (lane & (n - 1))] : 0;
#if defined(HG_IABL_TB)  // measurement builds only (wrong pixels): the TB's work dropped
    if (r0 != 12345) return;
#endif
    // 1. gather neighbours in search order (8.4.4.2.2): s < 2n left column bottom-up,
    //    s == 2n corner, s > 2n top row left-to-right
#if defined(HG_HOST_EMU)
    {  // scalar equivalent of the ballot-based gather + substitution below
        int sv[129];
        bool sa[129];
        bool any_av = false;
        for (int s = 0; s < ns; ++s) {
            int xn, yn;
            if (s < 2 * n) {
                xn = x0 - 1;
                yn = y0 + 2 * n - 1 - s;
            } else if (s == 2 * n) {
                xn = x0 - 1;
                yn = y0 - 1;
            } else {
                xn = x0 + s - 2 * n - 1;
                yn = y0 - 1;
            }
            sa[s] = xn >= 0 && yn >= 0 && xn < PW && yn < PH && nb_avail(zc, xn << subx, yn << suby, bx0, by0, csl);
            sv[s] = sa[s] ? w.fetch(xn, yn) : 0;
            any_av |= sa[s];
        }
        int first = -1;
        for (int s = 0; s < ns && first < 0; ++s)
            if (sa[s]) first = s;
        int last = -1;
        for (int s = 0; s < ns; ++s) {
            int v;
            if (!any_av) v = 1 << (bd - 1);
            else if (sa[s]) v = sv[s], last = s;
            else v = last >= 0 ? sv[last] : sv[first];
            if (s < 2 * n) L->left[2 * n - s] = (int16_t)v;
            else if (s == 2 * n) L->left[0] = L->top[0] = (int16_t)v;
            else L->top[s - 2 * n] = (int16_t)v;
        }
    }
#elif defined(HG_IABL_GATHER)  // measurement builds only: no neighbour gather
#else
    if (ns <= 64) {  // 4x4 and 8x8 TBs (most of them): one chunk of 4n + 1 <= 33 samples
        const int s = lane;
#if !defined(HG_INTRA_GATHER_R04)
        // every step formed for all lanes with selects (the branchy form
        // split the wave into three exec regions per step): the column left
        // of the TB bottom-up, the corner, the row above left to right
        const int xn = s <= 2 * n ? x0 - 1 : x0 + s - 2 * n - 1;
        const int yn = s < 2 * n ? y0 + 2 * n - 1 - s : y0 - 1;
        const bool av = s < ns && xn >= 0 && yn >= 0 && xn < PW && yn < PH &&
                        nb_avail(zc, xn << subx, yn << suby, bx0, by0, csl);
        const int lx = xn - w.cx0, ly = yn - w.cy0;
        const Pel *src = ly < 0 ? w.above + lx + 1 : (lx < 0 ? w.left + ly : w.cur + ly * w.csx + lx);
        const int val = (int)*(av ? src : w.cur);  // (an unavailable lane reads the window's first sample)
        const uint64_t msk = __ballot(av);
        const uint64_t below = msk & ((1ull << lane) - 1ull);
        const int sub = below ? 63 - __clzll(below) : __ffsll((unsigned long long)msk) - 1;
        const int sv = __shfl(val, av ? lane : sub, 64);
        const int v = msk ? sv : (1 << (bd - 1));
        int16_t *dp = s < 2 * n ? L->left + (2 * n - s) : L->top + (s - 2 * n);
        if (s < ns) *dp = (int16_t)v;
        if (s == 2 * n) L->left[0] = (int16_t)v;
#else
        int xn, yn;
        if (s < 2 * n) {
            xn = x0 - 1;
            yn = y0 + 2 * n - 1 - s;
        } else if (s == 2 * n) {
            xn = x0 - 1;
            yn = y0 - 1;
        } else {
            xn = x0 + s - 2 * n - 1;
            yn = y0 - 1;
        }
        const bool av = s < ns && xn >= 0 && yn >= 0 && xn < PW && yn < PH &&
                        nb_avail(zc, xn << subx, yn << suby, bx0, by0, csl);
        const int val = av ? w.fetch(xn, yn) : 0;
        const uint64_t msk = __ballot(av);
        int sl = lane;
        if (!av && msk) {
            const uint64_t below = msk & ((1ull << lane) - 1ull);
            sl = below ? 63 - __clzll(below) : __ffsll((unsigned long long)msk) - 1;
        }
        const int sv = __shfl(val, sl, 64);
        const int v = msk ? sv : (1 << (bd - 1));
        if (s < 2 * n) L->left[2 * n - s] = (int16_t)v;
        else if (s == 2 * n) {
            L->left[0] = (int16_t)v;
            L->top[0] = (int16_t)v;
        } else if (s < ns) {
            L->top[s - 2 * n] = (int16_t)v;
        }
#endif
    } else {
    // 16x16 (65 samples) needs two chunks, 32x32 (129) three
    const int nch = ns <= 128 ? 2 : 3;
    int val[3] = {0, 0, 0};
    uint64_t msk[3] = {0, 0, 0};
    for (int k = 0; k < nch; ++k) {
        // (as the one-chunk path: positions and the source by selects)
        const int s = lane + 64 * k;
        const int xn = s <= 2 * n ? x0 - 1 : x0 + s - 2 * n - 1;
        const int yn = s < 2 * n ? y0 + 2 * n - 1 - s : y0 - 1;
        const bool av = s < ns && xn >= 0 && yn >= 0 && xn < PW && yn < PH &&
                        nb_avail(zc, xn << subx, yn << suby, bx0, by0, csl);
        const int lx = xn - w.cx0, ly = yn - w.cy0;
        const Pel *src = ly < 0 ? w.above + lx + 1 : (lx < 0 ? w.left + ly : w.cur + ly * w.csx + lx);
        val[k] = av ? (int)*src : 0;
        msk[k] = __ballot(av);
    }
    // 2. substitution: nearest available predecessor in search order, else the first available
    const bool any = (msk[0] | msk[1] | msk[2]) != 0;
    for (int k = 0; k < nch; ++k) {
        const int s = lane + 64 * k;
        int sc = k, sl = lane;  // source (chunk, lane) of this sample's value
        if (any && !((msk[k] >> lane) & 1)) {
            sc = -1;
            uint64_t below = msk[k] & ((1ull << lane) - 1ull);
            if (below) {
                sc = k;
                sl = 63 - __clzll(below);
            } else {
                for (int j = k - 1; j >= 0 && sc < 0; --j)
                    if (msk[j]) {
                        sc = j;
                        sl = 63 - __clzll(msk[j]);
                    }
            }
            if (sc < 0) {  // no predecessor: value of the first available sample
                for (int j = 0; j < 3 && sc < 0; ++j)
                    if (msk[j]) {
                        sc = j;
                        sl = __ffsll((unsigned long long)msk[j]) - 1;
                    }
            }
        }
        // all lanes active for the cross-lane reads
        const int v0 = __shfl(val[0], sl, 64), v1 = __shfl(val[1], sl, 64);
        const int v2 = nch > 2 ? __shfl(val[2], sl, 64) : 0;
        const int v = !any ? (1 << (bd - 1)) : (sc == 0 ? v0 : (sc == 1 ? v1 : v2));
        int16_t *dp = s < 2 * n ? L->left + (2 * n - s) : L->top + (s - 2 * n);
        if (s < ns) *dp = (int16_t)v;
        if (s == 2 * n) L->left[0] = (int16_t)v;
    }
    }
#endif
    wave_sync();
    // 3. filtering (8.4.4.2.3): luma, and chroma with 4:4:4
    const int16_t *lf = L->left, *tp = L->top;
    {
        if (filt) {  // (tb_meta: luma or 4:4:4 chroma, not DC, not 4x4, the mode past the threshold)
            const int c = L->left[0];
            const bool bi = strong && cidx == 0 && n == 32 && abs(c + L->top[64] - 2 * L->top[32]) < (1 << (bd - 5)) &&
                            abs(c + L->left[64] - 2 * L->left[32]) < (1 << (bd - 5));
            // (selects, not a lane-dependent if / else chain: one exec-mask region
            // per arm cost more scalar instructions than the arithmetic)
            const int corner = (L->left[1] + 2 * c + L->top[1] + 2) >> 2;
            for (int i = lane; i <= 2 * n; i += kWave) {
                int a, b;
                if (bi) {  // (uniform; i == 0 and i == 64 are the interpolation's end points)
                    a = ((64 - i) * c + i * L->left[64] + 32) >> 6;
                    b = ((64 - i) * c + i * L->top[64] + 32) >> 6;
                } else {
                    const int im = i > 0 ? i - 1 : 0, ip = i < 2 * n ? i + 1 : i;
                    const int li = L->left[i], ti = L->top[i];
                    a = (L->left[ip] + 2 * li + L->left[im] + 2) >> 2;
                    b = (L->top[ip] + 2 * ti + L->top[im] + 2) >> 2;
                    a = i == 0 ? corner : (i == 2 * n ? li : a);
                    b = i == 0 ? corner : (i == 2 * n ? ti : b);
                }
                L->fl[i] = (int16_t)a;
                L->ft[i] = (int16_t)b;
            }
            wave_sync();
            lf = L->fl;
            tp = L->ft;
        }
    }
    const int maxv = (1 << bd) - 1;
    // 4. prediction (+ residual)
    int dc = 0;
    if (mode == 1) {  // DC: the 2n <= 64 references summed over lanes 0 .. 2n - 1, then broadcast
#if !defined(HG_HOST_EMU)
        int sum = lane < 2 * n ? (lane < n ? tp[1 + lane] : lf[1 + lane - n]) : 0;
        sum = __builtin_amdgcn_readlane(group_sum(sum, 2 * n), 0);
#else
        int sum = 0;
        for (int i = lane; i < 2 * n; i += kWave) sum += i < n ? tp[1 + i] : lf[1 + i - n];
#endif
        dc = (sum + n) >> (log2n + 1);
    }
    const int lx0 = x0 - w.cx0, ly0 = y0 - w.cy0;
    auto predict_sample = [&](int o) {
        const int x = o & (n - 1), y = o >> log2n;
        int pv;
        if (mode == 0) {
            pv = ((n - 1 - x) * lf[1 + y] + (x + 1) * tp[1 + n] + (n - 1 - y) * tp[1 + x] + (y + 1) * lf[1 + n] + n) >>
                 (log2n + 1);
        } else if (mode == 1) {
            pv = dc;
            if (cidx == 0 && n < 32) {
                // the DC edge filter as selects over both reference reads (the
                // lane-dependent if / else chain cost an exec-mask region per arm)
                const int t = tp[1 + x], l = lf[1 + y];
                const int e = (x == 0 ? l : t) + (x == 0 && y == 0 ? t : dc) + 2 * dc + 2;
                pv = (x == 0 || y == 0) ? e >> 2 : dc;
            }
        } else {
            const int ang = (int)(int8_t)(am & 0xffu), inv = (int)(int16_t)(am >> 16);  // (tb_angle)
            const int16_t *main_ = mode >= 18 ? tp : lf, *side = mode >= 18 ? lf : tp;
            const int a = mode >= 18 ? x : y, b = mode >= 18 ? y : x;  // a along the main direction
            const int idx = ((b + 1) * ang) >> 5, fact = ((b + 1) * ang) & 31;
            // both references read unconditionally (the second index is at most
            // 2n + 1, inside the 66-entry arrays): with iFact 0 the weighted sum
            // is the first reference exactly, so no lane-dependent branch
            const int p0 = *ang_ref(main_, side, inv, a + idx + 1), p1 = *ang_ref(main_, side, inv, a + idx + 2);
            pv = ((32 - fact) * p0 + fact * p1 + 16) >> 5;
            if (cidx == 0 && n < 32) {
                if (mode == 26) {
                    const int v = min(max(tp[1] + ((lf[1 + y] - lf[0]) >> 1), 0), maxv);
                    pv = x == 0 ? v : pv;
                }
                if (mode == 10) {
                    const int v = min(max(lf[1] + ((tp[1 + x] - tp[0]) >> 1), 0), maxv);
                    pv = y == 0 ? v : pv;
                }
            }
        }
        const int li = (ly0 + y) * w.csx + lx0 + x;
        if (tu.flags & TU_PCM) pv = 0;  // the residual is the PCM sample itself
        if (cbf) pv += (n <= 8 && o == lane) ? r0 : rt[y * w.rp + x];
        pv = min(max(pv, 0), maxv);
        w.cur[li] = (Pel)pv;
    };
#if defined(HG_IABL_PRED)  // measurement builds only: no prediction
    if (lane == 1000) predict_sample(0);
    if (false)
#elif !defined(HG_HOST_EMU)
    if (n <= 8) {  // one sample per lane: no loop
        if (lane < n * n) predict_sample(lane);
    } else
#endif
    {
        for (int o = lane; o < n * n; o += kWave) predict_sample(o);
    }
    wave_sync();
}

#if !defined(HG_HOST_EMU)
// The Cb and Cr TBs of one 4:2:0 chroma TU (n = 4 or 8) in one pass: lanes
// 0-31 predict Cb, lanes 32-63 Cr.  The two TBs share position, size,
// IntraPredModeC and neighbour availability, and chroma has no reference
// filtering (8.4.4.2.3) and no DC / angular edge filters (8.4.4.2.6, cIdx 0
// only), so each step of predict_tb runs once for both: 4n + 1 <= 33
// neighbours per half (a second chunk for the 33rd of an 8x8), a 32-lane DC
// reduction, and n * n <= 64 samples in two rounds of 32.  Scratch halves:
// left / top at + 33 * h.
template <typename Pel>
__device__ __attribute__((always_inline)) inline void predict_pair(IntraScratch *L, const TuRec &tb, const TuRec &tr,
                                                                   const Win<Pel> &wb, const Win<Pel> &wr, int PW,
                                                                   int PH, int bd, int zc, uint32_t am, int lane) {
    // lanes 0-31 predict Cb and 32-63 Cr: the pairing needs a full 64-lane wave
    static_assert(kWave == 64, "predict_pair splits a 64-lane wave into two halves");
    const int log2n = tb.log2, n = 1 << log2n, mode = tb.mode;
    const int x0 = tb.x, y0 = tb.y;
    const int h = lane >> 5, sl = lane & 31;
    // per-field selects (a lane-dependent reference into the caller's win[] would put it in scratch)
    Win<Pel> w;
    w.cur = h ? wr.cur : wb.cur;
    w.left = h ? wr.left : wb.left;
    w.above = h ? wr.above : wb.above;
    w.res = h ? wr.res : wb.res;
    w.rp = wb.rp;
    w.csx = wb.csx;
    w.csy = wb.csy;
    w.cx0 = wb.cx0;
    w.cy0 = wb.cy0;
    const bool cbf = ((h ? tr.flags : tb.flags) & TU_CBF) != 0;
    const bool pcm = ((h ? tr.flags : tb.flags) & TU_PCM) != 0;
    const int bx0 = w.cx0 << 1, by0 = w.cy0 << 1, csl = w.csx << 1;
    const int ns = 4 * n + 1, nch = n == 8 ? 2 : 1;
    // residuals (sample sl and sl + 32 of this half), used after the neighbour phase
    int r0 = 0, r1 = 0;
    if (cbf && sl < n * n) r0 = w.res[(ptrdiff_t)(y0 + (sl >> log2n)) * w.rp + x0 + (sl & (n - 1))];
    if (cbf && sl + 32 < n * n) r1 = w.res[(ptrdiff_t)(y0 + ((sl + 32) >> log2n)) * w.rp + x0 + ((sl + 32) & (n - 1))];
    int16_t *left = L->left + 33 * h, *top = L->top + 33 * h;
    // 1. neighbours in search order (8.4.4.2.2), chunk k = search positions sl + 32 k
    // (two named registers, not arrays: indexed by a runtime chunk they went to scratch)
    int val0 = 0, val1 = 0;
    uint32_t hm0 = 0, hm1 = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (k >= nch) break;
        const int s = sl + 32 * k;
        // (positions and the source by selects, as predict_tb's one-chunk path)
        const int xn = s <= 2 * n ? x0 - 1 : x0 + s - 2 * n - 1;
        const int yn = s < 2 * n ? y0 + 2 * n - 1 - s : y0 - 1;
        const bool av = s < ns && xn >= 0 && yn >= 0 && xn < PW && yn < PH &&
                        nb_avail(zc, xn << 1, yn << 1, bx0, by0, csl);
        const int lx = xn - w.cx0, ly = yn - w.cy0;
        const Pel *srcp = ly < 0 ? w.above + lx + 1 : (lx < 0 ? w.left + ly : w.cur + ly * w.csx + lx);
        const int vk = av ? (int)*srcp : 0;
        const uint32_t hk = (uint32_t)(__ballot(av) >> (32 * h));
        if (k == 0) {
            val0 = vk;
            hm0 = hk;
        } else {
            val1 = vk;
            hm1 = hk;
        }
    }
    // 2. substitution: nearest available predecessor, else the first available
    const bool any = (hm0 | hm1) != 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (k >= nch) break;
        const int s = sl + 32 * k;
        const uint32_t hmk = k ? hm1 : hm0;
        int sc = k, src = sl;
        if (any && !((hmk >> sl) & 1u)) {
            const uint32_t below = hmk & ((1u << sl) - 1u);
            if (below) {
                src = 31 - __builtin_clz(below);
            } else if (k == 1 && hm0) {
                sc = 0;
                src = 31 - __builtin_clz(hm0);
            } else {
                sc = hm0 ? 0 : 1;
                src = __builtin_ctz(sc ? hm1 : hm0);
            }
        }
        const int v0 = __shfl(val0, 32 * h + src, 64);
        const int v1 = nch > 1 ? __shfl(val1, 32 * h + src, 64) : 0;
        const int v = !any ? (1 << (bd - 1)) : (sc == 0 ? v0 : v1);
        int16_t *dp = s < 2 * n ? left + (2 * n - s) : top + (s - 2 * n);
        if (s < ns) *dp = (int16_t)v;
        if (s == 2 * n) left[0] = (int16_t)v;
    }
    wave_sync();
    const int16_t *lf = left, *tp = top;
    const int maxv = (1 << bd) - 1;
    int dc = 0;
    const int ang = (int)(int8_t)(am & 0xffu), inv = (int)(int16_t)(am >> 16);  // (tb_angle)
    const int16_t *main_ = mode >= 18 ? tp : lf, *side = mode >= 18 ? lf : tp;
    if (mode == 1) {  // each half sums its 2n <= 16 references in its lanes 0 .. 2n - 1
        const int sum = group_sum(sl < 2 * n ? (sl < n ? tp[1 + sl] : lf[1 + sl - n]) : 0, 2 * n);
        const int s0 = __builtin_amdgcn_readlane(sum, 0), s1 = __builtin_amdgcn_readlane(sum, 32);
        dc = ((h ? s1 : s0) + n) >> (log2n + 1);
    }
    const int lx0 = x0 - w.cx0, ly0 = y0 - w.cy0;
    for (int it = 0; it < nch; ++it) {
        const int o = sl + 32 * it;
        if (o < n * n) {
            const int x = o & (n - 1), y = o >> log2n;
            int pv;
            if (mode == 0) {
                pv = ((n - 1 - x) * lf[1 + y] + (x + 1) * tp[1 + n] + (n - 1 - y) * tp[1 + x] + (y + 1) * lf[1 + n] +
                      n) >> (log2n + 1);
            } else if (mode == 1) {
                pv = dc;
            } else {
                const int a = mode >= 18 ? x : y, b = mode >= 18 ? y : x;
                const int idx = ((b + 1) * ang) >> 5, fact = ((b + 1) * ang) & 31;
                // (both references unconditionally, as predict_tb: index <= 2n + 1 inside the half's 33)
                const int p0 = *ang_ref(main_, side, inv, a + idx + 1), p1 = *ang_ref(main_, side, inv, a + idx + 2);
                pv = ((32 - fact) * p0 + fact * p1 + 16) >> 5;
            }
            if (pcm) pv = 0;  // the residual is the PCM sample itself
            if (cbf) pv += it ? r1 : r0;
            pv = min(max(pv, 0), maxv);
            w.cur[(ly0 + y) * w.csx + lx0 + x] = (Pel)pv;
        }
    }
    wave_sync();
}
#endif

}  // namespace

// Register budget: at most 5 waves per SIMD (<= 102 VGPRs, 76 used).  r04
// measured 7 (72 VGPRs) best against 8 and the compiler's own; with r05's
// lighter parse and transform, same-box pairs at 128 images gave 7: 19,690,
// 5: 20,210, 4: 20,020 Mpix/s (profiles/r05/ab/ab_b128_dot4.txt): fewer
// resident k_intra waves take less issue from the parse beside them.
// HG_INTRA_WPE=0 leaves it to the compiler.
#ifndef HG_INTRA_WPE
#define HG_INTRA_WPE 5
#endif
#if HG_INTRA_WPE > 0
#define HG_INTRA_ATTR __attribute__((amdgpu_waves_per_eu(HG_INTRA_WPE)))
#else
#define HG_INTRA_ATTR
#endif
// CF: the batch's chroma_format_idc (a compile-time constant: the 4:2:0 build
// carries no per-format arithmetic)
// LDS of k_intra's streaming mode beyond the windows: the transform tables
// (workgroup) and per wave the transform tiles (transform_tb, xform.hpp)
// (the transposed matrices s_mt; per wave the d tile 32 x 34, the g tile 32 x 32, the extent pair)
constexpr size_t kXfTablesBytes = sizeof(XfTab);
constexpr size_t kXfDBytes = 32 * kXfDStride32 * sizeof(int16_t), kXfGBytes = 32 * 32 * sizeof(int16_t);
constexpr size_t kXfWaveBytes = kXfDBytes + kXfGBytes + 16;
static_assert(kXfTablesBytes % 16 == 0 && kXfWaveBytes % 16 == 0, "transform scratch alignment");
constexpr int kIntraPlanes = 0, kIntraStream = 1;
constexpr uint32_t kGaveUp = ~0u;                 // a wave's progress word: it gave its rows up
constexpr uint64_t kRedoPatience = 200000000ull;  // 2 s (10 ns ticks): the parse is over by then

// Mode kIntraPlanes: k_intra, residuals from k_transform's planes.
// Mode kIntraStream: k_intra_stream, launched beside the spread parse of the same decode:
// each row's TU records are consumed as the parse publishes them (agent-scope
// per-row TU counts behind its progress words) and every coded TB is
// transformed by the wave itself (transform_tb into LDS) right before its
// prediction, so no k_transform pass and no residual planes; the
// reconstruction trails the parse by a CTU instead of starting after it.
// (r04's third mode, k_intra_fused: the in-line transform after the parse
// instead of k_transform + k_intra, lost beside the next parse, 12.2-12.9
// against 18.6 Gpix/s; removed in r05)
template <typename Pel, int CF, int Mode>
__device__ __attribute__((always_inline)) inline void intra_body(const BatchArgs &a, unsigned char *smem) {
    constexpr bool Poll = Mode == kIntraStream;       // rows consumed while the parse writes them
    constexpr bool XfInline = Poll;                   // each TB transformed by the wave (no k_transform)
    const int nw = (int)HG_UNI(blockDim.x >> 6);
    const int pic = a.pic0 + blockIdx.x;
    const int wave = (int)HG_UNI(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const PicDesc pd = a.pics[pic];
    if (pd.flags & PD_ASSEMBLY) return;  // no coded data of its own (uniform: the whole workgroup leaves)
    // second launch: only the pictures the first gave up (its done word, after the TU counts)
    if (Poll && a.stream_redo && hg_load_agent(a.xntu + a.total_rows + pic) != 0) return;
    const SeqParams sp = a.seqs[pd.seq];
    const int W = sp.width, H = sp.height, log2ctb = sp.log2_ctb;
    const int wctb = (W + (1 << log2ctb) - 1) >> log2ctb, hctb = (H + (1 << log2ctb) - 1) >> log2ctb;
    constexpr int chroma = CF;  // = sp.chroma_format (launch_intra picks the instantiation)
    const int cw = chroma ? W >> chroma_sx(chroma) : 0, ch = chroma ? H >> chroma_sy(chroma) : 0;
    const int ncomp = chroma ? 3 : 1;
    const bool strong = (sp.flags & SP_STRONG_INTRA) != 0;
    const WinLayout lay = win_layout(log2ctb, chroma, (int)sizeof(Pel));
    uint32_t *progress = reinterpret_cast<uint32_t *>(smem);  // [nw], 64 B reserved
    Frame<Pel, CF> F;
    F.blk = smem + 64 + (size_t)wave * lay.bytes;
    F.recon = reinterpret_cast<Pel *>(a.recon + pd.recon_off);
    F.resid = a.resid + pd.resid_off;
    F.init(log2ctb, W, H, cw, ch);
    XfScratch X{};
    if constexpr (XfInline) {
        unsigned char *tab = smem + 64 + (size_t)nw * lay.bytes;
        unsigned char *xw = tab + kXfTablesBytes + (size_t)wave * kXfWaveBytes;
        X = XfScratch{reinterpret_cast<int16_t *>(xw), reinterpret_cast<int16_t *>(xw + kXfDBytes),
                      reinterpret_cast<int32_t *>(xw + kXfDBytes + kXfGBytes), reinterpret_cast<const XfTab *>(tab)};
        xf_tables(reinterpret_cast<XfTab *>(tab), lane);
    }
    IntraScratch *S = reinterpret_cast<IntraScratch *>(F.blk);
    progress[wave] = 0;  // every lane writes the same value
    __syncthreads();
    const uint32_t stride = (uint32_t)wctb + 1;
    // split (a.intra_split): waves in pairs per CTB row, luma on the even one and
    // Cb, Cr on the odd one.  Chroma prediction reads chroma neighbours only, so
    // the two TB chains of a CTU run side by side instead of one after the other
    const bool split = a.intra_split != 0 && ncomp == 3;
    const int cls = split ? (wave & 1) : 0, rw = split ? wave >> 1 : wave, nrw = split ? nw >> 1 : nw;
    const int k0 = split && cls ? 1 : 0, k1 = split && !cls ? 1 : ncomp;  // this wave's components
    const int prev_wave = split ? ((rw + nrw - 1) % nrw) * 2 + cls : (wave + nw - 1) % nw;
    const bool wpp = (sp.flags & SP_WPP) != 0;
    bool gave_up = false;  // (streaming, first launch: no parse progress for a while)
    for (int r = rw; r < hctb; r += nrw) {
        // streaming: TUs [0, ntu) of the row are known written; `done` once the parse finished the row
        uint32_t ntu = Poll ? 0u : a.row_counts[2 * (pd.row_off + r)];
        bool row_done = !Poll;
        const TuRec *tus = a.tus + pd.tu_off + (uint64_t)r * pd.tu_cap_row;
        const CoefSrc<Poll> coefs{a.coefs + pd.coef_off + (uint64_t)r * pd.coef_cap_row};
        int cur = -1;
#if !defined(HG_HOST_EMU)
        uint4 tblk = make_uint4(0, 0, 0, 0);  // lane l: TuRec t0 + l (one coalesced load per 64 TBs)
        uint32_t metav = 0, anglev = 0;       // lane l: tb_meta and tb_angle of that record
        uint32_t t0 = 0;
#endif
        for (uint32_t t = 0;; ++t) {
            bool reload = false;
            if constexpr (Poll) {
                if (t >= ntu && !row_done) {
                    // wait until the parse has published TU t of this row or finished the row
                    const uint32_t *pw = a.xprog + pd.row_off + (wpp ? r : 0);
                    const uint32_t *nw_ = a.xntu + pd.row_off + r;
                    const uint32_t fin = (uint32_t)(r + 1) * (uint32_t)wctb;
                    // Patience: nothing guarantees that the parse runs beside this kernel (a
                    // profiler that serialises dispatches, a busy device), so after `patience`
                    // without progress the first launch gives the picture up, and the second
                    // launch (after the parse) reconstructs it; there a stall is an error.
                    const uint64_t patience = (uint64_t)a.stream_patience_us * 100u;
                    uint32_t seen_n = ~0u, seen_p = ~0u;
                    uint64_t t_last = 0;
                    for (;;) {
                        if (!a.stream_redo && !patience) {  // (test knob: every picture to the second launch)
                            gave_up = true;
                            break;
                        }
                        const uint32_t n_ = (uint32_t)HG_UNI(hg_load_agent(nw_));
                        if (n_ > t) {
                            ntu = n_;
                            break;
                        }
                        const uint32_t pv = (uint32_t)HG_UNI(hg_load_agent(pw));
                        if (pv >= fin) {  // row finished (or stopped: kProgDone)
                            ntu = (uint32_t)HG_UNI(hg_load_agent(nw_));
                            row_done = true;
                            break;
                        }
                        const uint64_t now = hg_clock_10ns();
                        if (n_ != seen_n || pv != seen_p) {
                            seen_n = n_;
                            seen_p = pv;
                            t_last = now;
                        } else if (now - t_last > (a.stream_redo ? kRedoPatience : patience)) {
                            if (!a.stream_redo) {
                                gave_up = true;
                            } else {  // bounded: never hang the device
                                if (lane == 0) atomicOr(&a.status[pic], ST_SUBSTREAM_END);
                                row_done = true;
                            }
                            break;
                        }
                        HG_STREAM_SLEEP();
                    }
                    if (gave_up) break;
                    // the records behind the count / progress word: formally ordered
                    // after the poll (the parse published them with an agent release)
                    HG_ACQ_AGENT();
                    reload = true;
                }
            }
            if (t > ntu || (t == ntu && !row_done)) break;  // (stalled: the status says so)
            TuRec tu{};
            int c = wctb;  // sentinel after the last TB: finish the open CTU
            if (t < ntu) {
#if defined(HG_HOST_EMU)
                tu = tus[t];
                (void)reload;
#else
                if ((t & 63u) == 0 || reload) {
                    t0 = t & ~63u;
                    const uint32_t i = t0 + (uint32_t)lane;
                    if constexpr (Poll) {
                        const uint64_t *q = reinterpret_cast<const uint64_t *>(tus + i);
                        const uint64_t lo = i < ntu ? __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
                        const uint64_t hi = i < ntu ? __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
                        tblk = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
                    } else {
                        tblk = i < ntu ? *reinterpret_cast<const uint4 *>(tus + i) : make_uint4(0, 0, 0, 0);
                    }
                    TuRec q;
                    __builtin_memcpy(&q, &tblk, sizeof(q));
                    metav = i < ntu ? tb_meta(q, F, r, k0, k1) : 0u;
                    anglev = tb_angle(q);
#if !defined(HG_INTRA_NO_PAIR)
                    if constexpr (!XfInline && CF == 1) {
                        // the next record (lane + 1; none past this block): its Cr TB?
                        const int nl = min(lane + 1, 63);
                        const uint4 nb = make_uint4((uint32_t)__shfl((int)tblk.x, nl, 64), (uint32_t)__shfl((int)tblk.y, nl, 64),
                                                    (uint32_t)__shfl((int)tblk.z, nl, 64), (uint32_t)__shfl((int)tblk.w, nl, 64));
                        TuRec nq;
                        __builtin_memcpy(&nq, &nb, sizeof(nq));
                        const bool pair = (metav & TBM_OK) && lane < 63 && i + 1 < ntu && (q.flags & TU_CIDX_MASK) == 1 &&
                                          q.log2 <= 3 && (nq.flags & TU_CIDX_MASK) == 2 && nq.x == q.x && nq.y == q.y &&
                                          nq.log2 == q.log2 && nq.mode == q.mode && nq.ctu == q.ctu;
                        metav |= pair ? TBM_PAIR : 0u;
                    }
#endif
                }
                const int sel = (int)(t - t0);
                const uint4 r = make_uint4((uint32_t)__builtin_amdgcn_readlane((int)tblk.x, sel),
                                           (uint32_t)__builtin_amdgcn_readlane((int)tblk.y, sel),
                                           (uint32_t)__builtin_amdgcn_readlane((int)tblk.z, sel),
                                           (uint32_t)__builtin_amdgcn_readlane((int)tblk.w, sel));
                __builtin_memcpy(&tu, &r, sizeof(tu));
#endif
                c = (int)HG_UNI((uint32_t)tu.ctu);
            }
            if (c != cur) {
                if (cur >= 0) {
                    // finish CTU `cur`: write the window back, keep its last column as `left`
                    _Pragma("nounroll") for (int k = 0; k < 3; ++k) {
                        if (k >= ncomp) break;
                        if (k < k0 || k >= k1) continue;
                        const Win<Pel> w = F.win(k, cur, r);
                        Pel *const plane = F.plane(k);
                        const int PW = F.pw(k), PH = F.ph(k);
                        const int vw = min(w.csx, PW - w.cx0), vh = min(w.csy, PH - w.cy0);
                        if (vw == w.csx && !(PW & 3) &&
                            !(reinterpret_cast<uintptr_t>(plane) & (4 * sizeof(Pel) - 1))) {
                            // full-width CTU: four samples per lane, one 4- (8-) byte store
                            const int lq = __builtin_ctz((unsigned)w.csx) - 2;
                            for (int o = lane; o < (vh << lq); o += kWave) {
                                const int x = (o & ((1 << lq) - 1)) << 2, y = o >> lq;
                                *reinterpret_cast<Quad<Pel> *>(plane + (size_t)(w.cy0 + y) * PW + w.cx0 + x) =
                                    *reinterpret_cast<const Quad<Pel> *>(w.cur + y * w.csx + x);
                            }
                        } else {
                            for (int o = lane; o < vw * vh; o += kWave) {
                                const int x = o % vw, y = o / vw;
                                plane[(size_t)(w.cy0 + y) * PW + w.cx0 + x] = w.cur[y * w.csx + x];
                            }
                        }
                        for (int y = lane; y < w.csy; y += kWave) w.left[y] = w.cur[y * w.csx + w.csx - 1];
                    }
                    wave_sync();
                    HG_FENCE_REL();
                    hg_atomic_store(&progress[wave], (uint32_t)r * stride + (uint32_t)cur + 1u);
                }
                if (c >= wctb) break;
                cur = c;
                if (r > 0) {
                    const uint32_t need = (uint32_t)(r - 1) * stride + (uint32_t)min(c + 2, wctb);
                    for (uint32_t spin = 0;; ++spin) {
                        const uint32_t v = (uint32_t)HG_UNI(hg_atomic_load(&progress[prev_wave]));
                        if (Poll && v == kGaveUp) {  // the row above was given up: so is this one
                            gave_up = true;
                            break;
                        }
                        if (v >= need) break;
                        if (spin > (1u << 24)) {  // bounded: never hang the device
                            if (lane == 0) atomicOr(&a.status[pic], ST_SUBSTREAM_END);
                            break;
                        }
                        HG_SLEEP();
                    }
                    if (gave_up) break;
                    HG_FENCE_ACQ();
                }
                // start CTU c: the row above (corner .. above-right) and the residuals
                _Pragma("nounroll") for (int k = 0; k < 3; ++k) {
                    if (k >= ncomp) break;
                    if (k < k0 || k >= k1) continue;
                    const Win<Pel> w = F.win(k, c, r);
                    const Pel *const plane = F.plane(k);
                    const int PW = F.pw(k);
                    const int yg = w.cy0 - 1;
                    for (int i = lane; i <= 2 * w.csx; i += kWave) {
                        const int xg = w.cx0 - 1 + i;
                        w.above[i] = (yg >= 0 && xg >= 0 && xg < PW) ? plane[(size_t)yg * PW + xg] : (Pel)0;
                    }
                }
                wave_sync();
            }
            // this wave's component, a valid TB of CTB `cur` (tb_meta): its facts for 64 records
            // were formed at the block load
#if defined(HG_HOST_EMU)
            const uint32_t m = tb_meta(tu, F, r, k0, k1);
#else
            const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)metav, (int)(t - t0));
#endif
            if (!(m & TBM_OK)) continue;
#if defined(HG_HOST_EMU)
            const uint32_t am = tb_angle(tu);
#else
            const uint32_t am = (uint32_t)__builtin_amdgcn_readlane((int)anglev, (int)(t - t0));
#endif
            const int cidx = tu.flags & TU_CIDX_MASK, zc = (int)((m >> 8) & 0xffu);
            // the TB's component window, formed here from the wave-uniform cidx and CTU
            Win<Pel> w = F.win(cidx, cur, r);
            const int PW = cidx ? cw : W, PH = cidx ? ch : H;
            if constexpr (XfInline) {
                // the TB's residual, transformed by this wave into LDS (pitch n, origin the TB's)
                if (tu.flags & TU_CBF) {
                    const int n = 1 << tu.log2;
                    transform_tb<Poll>(tu, coefs, sp, a.sf, X, X.d, n, lane);
                    w.res = X.d;
                    w.rp = n;
                    w.rx0 = tu.x;
                    w.ry0 = tu.y;
#if defined(HG_HOST_EMU)
                    w.res_lo = X.d;
                    w.res_hi = X.d + 32 * 32;  // (the 2 KB residual tile of XfScratch)
#endif
                }
            }
#if !defined(HG_HOST_EMU) && !defined(HG_INTRA_NO_PAIR)
            // a 4x4 / 8x8 Cb TB followed by its Cr TB (same TU; the next record of this 64-record block):
            // both in one pass
            if (!XfInline && (m & TBM_PAIR)) {  // (the next record is its Cr TB: tb_meta)
                TuRec tr = tu;  // same position, size, mode and CTU; the flags are the Cr TB's
                tr.flags = (uint8_t)((uint32_t)__builtin_amdgcn_readlane((int)tblk.y, (int)(t + 1 - t0)) >> 8);
                predict_pair<Pel>(S, tu, tr, F.win(1, cur, r), F.win(2, cur, r), PW, PH, sp.bit_depth_c, zc, am, lane);
                ++t;
                continue;
            }
#endif
            predict_tb<Pel, CF>(S, tu, w, PW, PH, cidx, cidx ? sp.bit_depth_c : sp.bit_depth_y, strong, zc,
                                (m & TBM_FILT) != 0, am, lane);
        }
        if (gave_up) {  // (the waves below see it and give up too)
            hg_atomic_store(&progress[wave], kGaveUp);
            break;
        }
        HG_FENCE_REL();
        hg_atomic_store(&progress[wave], (uint32_t)r * stride + (uint32_t)wctb);
    }
    if constexpr (Poll) {
        // first launch: the picture is done unless a wave gave up (its words then say kGaveUp)
        __syncthreads();
        if (!a.stream_redo && wave == 0) {
            bool ok = true;
            for (int w = 0; w < nw; ++w) ok = ok && hg_atomic_load(&progress[w]) != kGaveUp;
            if (lane == 0) a.xntu[a.total_rows + pic] = ok ? 1u : 0u;
        }
    }
}

template <typename Pel, int CF>
__global__ void __launch_bounds__(kMaxWaves * 64) HG_INTRA_ATTR k_intra(BatchArgs a) {
#if defined(HG_HOST_EMU)
    unsigned char *smem = g_emu.smem;
#else
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
#endif
    intra_body<Pel, CF, kIntraPlanes>(a, smem);
}

// (no waves-per-EU cap: the transform's registers come on top of the prediction's)
template <typename Pel, int CF>
__global__ void __launch_bounds__(kMaxWaves * 64) k_intra_stream(BatchArgs a) {
#if defined(HG_HOST_EMU)
    unsigned char *smem = g_emu.smem;
#else
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
#endif
    intra_body<Pel, CF, kIntraStream>(a, smem);
}

// luma / chroma wave pairs (k_intra's split): for batches of few pictures,
// where the per-picture TB chain is the latency (HEIFGPU_INTRA_SPLIT=0/1 forces it)
static bool intra_split_for(const BatchArgs &a, int nw) {
    static const int forced = [] {
        const char *e = std::getenv("HEIFGPU_INTRA_SPLIT");
        return e ? std::atoi(e) : -1;
    }();
    if (a.chroma_format == 0) return false;
    if (forced >= 0) return forced != 0;
    return nw >= 4 && (long)a.n_pics * a.max_rows <= 4096;
}

// waves of a split workgroup: two per row in flight, within the LDS budget and kMaxWaves
static int intra_split_waves(const BatchArgs &a, int nw) {
    int cap = intra_waves(a.max_log2ctb, a.chroma_format, a.bytes_per_sample, 2 * a.max_rows);
    int w = 2 * nw < cap ? 2 * nw : cap;
    w &= ~1;
    return w < 2 ? 2 : w;
}

static int intra_launch_waves(const BatchArgs &a) {
    // all pictures of a batch share bit depth and chroma format; the CTB size
    // may differ, so size for the largest one.  HEIFGPU_INTRA_WAVES caps the
    // waves per picture (tuning: fewer waves = more pictures per CU).
    // Measured (128 x 48 tiles): 16 waves/picture 142 ms, 8: 71, 4: 48, 1: 61 —
    // many pictures per CU beat deep per-picture row parallelism, so waves per
    // picture shrink as the batch grows.  Floor 2: alone 4 and 2 waves tie
    // (~40 ms), but beside the next decode's k_parse (pipelined) the smaller
    // workgroup fits the LDS that k_parse leaves free (bench 12.0 -> 12.5-13.0 Gpix/s).
    static const int forced = [] {
        const char *e = std::getenv("HEIFGPU_INTRA_WAVES");
        return e ? std::atoi(e) : 0;
    }();
    int cap = forced > 0 ? forced : kResidentIntraWaves / (a.n_pics > 0 ? a.n_pics : 1);
    if (forced <= 0) cap = cap < 2 ? 2 : cap;
    const int nw = intra_waves(a.max_log2ctb, a.chroma_format, a.bytes_per_sample, a.max_rows);
    return cap < nw ? cap : nw;
}

// k_intra_stream: four waves per picture (rows r, r + 4, ...), no luma / chroma
// split.  It only has to keep up with the parse, and its waves share the CUs
// with the parse's: one image, same box, 4 waves 28.2-28.3 ms per pipelined
// step against 28.9-29.4 with 16 (latency 28.0-28.1 either way, the parse's)
static int stream_waves(int nw) {
    static const int forced = [] {
        const char *e = std::getenv("HEIFGPU_INTRA_WAVES");
        return e ? std::atoi(e) : 0;
    }();
    if (forced > 0) return nw;
    return nw < 4 ? nw : 4;
}

static size_t intra_lds_bytes(const BatchArgs &a, int nw) {
    size_t b = 64 + (size_t)nw * win_layout(a.max_log2ctb, a.chroma_format, a.bytes_per_sample).bytes;
    if (a.intra_stream) b += kXfTablesBytes + (size_t)nw * kXfWaveBytes;
    return b;
}

// waves of a launch, the streaming mode's extra LDS included (pairs stay pairs)
static int intra_fit_waves(const BatchArgs &a, int nw) {
    while (nw > 1 && intra_lds_bytes(a, nw) > kIntraLdsBudget) nw -= a.intra_split ? 2 : 1;
    return nw < 1 ? 1 : nw;
}

#if defined(HG_HOST_EMU)
template <int CF>
static void emu_intra_cf(const BatchArgs &a, int nw) {
    const size_t lds = intra_lds_bytes(a, nw);
    if (a.intra_stream) {
        if (a.bytes_per_sample == 1) emu_launch(k_intra_stream<uint8_t, CF>, a.n_pics, 1, nw, a, false, lds);
        else emu_launch(k_intra_stream<uint16_t, CF>, a.n_pics, 1, nw, a, false, lds);
        return;
    }
    if (a.bytes_per_sample == 1) emu_launch(k_intra<uint8_t, CF>, a.n_pics, 1, nw, a, false, lds);
    else emu_launch(k_intra<uint16_t, CF>, a.n_pics, 1, nw, a, false, lds);
}
void emu_intra(const BatchArgs &a0) {
    BatchArgs a = a0;
    int nw = intra_launch_waves(a);
    if (a.intra_stream) nw = stream_waves(nw);
    a.intra_split = !a.intra_stream && intra_split_for(a, nw) ? 1 : 0;
    if (a.intra_split) nw = intra_split_waves(a, nw);
    nw = intra_fit_waves(a, nw);
    switch (a.chroma_format) {
    case 0: emu_intra_cf<0>(a, nw); break;
    case 2: emu_intra_cf<2>(a, nw); break;
    case 3: emu_intra_cf<3>(a, nw); break;
    default: emu_intra_cf<1>(a, nw); break;
    }
}
#else
template <int CF>
static void launch_intra_cf(const BatchArgs &a, int nw, size_t lds, hipStream_t s) {
    if (a.intra_stream) {
        if (a.bytes_per_sample == 1)
            hipLaunchKernelGGL((k_intra_stream<uint8_t, CF>), dim3(a.n_pics), dim3(nw * 64), lds, s, a);
        else
            hipLaunchKernelGGL((k_intra_stream<uint16_t, CF>), dim3(a.n_pics), dim3(nw * 64), lds, s, a);
        return;
    }
    if (a.bytes_per_sample == 1)
        hipLaunchKernelGGL((k_intra<uint8_t, CF>), dim3(a.n_pics), dim3(nw * 64), lds, s, a);
    else
        hipLaunchKernelGGL((k_intra<uint16_t, CF>), dim3(a.n_pics), dim3(nw * 64), lds, s, a);
}
hipError_t launch_intra(const BatchArgs &a0, hipStream_t s) {
    BatchArgs a = a0;
    int nw = intra_launch_waves(a);
    if (a.intra_stream) nw = stream_waves(nw);
    a.intra_split = !a.intra_stream && intra_split_for(a, nw) ? 1 : 0;
    if (a.intra_split) nw = intra_split_waves(a, nw);
    nw = intra_fit_waves(a, nw);
    const size_t lds = intra_lds_bytes(a, nw);
    switch (a.chroma_format) {
    case 0: launch_intra_cf<0>(a, nw, lds, s); break;
    case 2: launch_intra_cf<2>(a, nw, lds, s); break;
    case 3: launch_intra_cf<3>(a, nw, lds, s); break;
    default: launch_intra_cf<1>(a, nw, lds, s); break;
    }
    return hipGetLastError();
}
#endif

// The streaming knobs, read from the environment when a context is created
// (heifgpu_create; the emulation driver reads them once per run):
// HEIFGPU_STREAM=0 turns k_intra_stream off, HEIFGPU_STREAM_MAX_PICS moves its
// batch limit (tuning), HEIFGPU_STREAM_PATIENCE_US is how long the first
// launch waits without parse progress before it gives a picture up to the
// second launch (0: every picture, a test knob).
StreamKnobs stream_knobs_from_env() {
    StreamKnobs k;
    const char *e = std::getenv("HEIFGPU_STREAM");
    k.enabled = !(e && std::atoi(e) == 0);
    const char *m = std::getenv("HEIFGPU_STREAM_MAX_PICS");
    k.max_pics = m && *m ? std::atoi(m) : kStreamMaxPics;
    const char *p = std::getenv("HEIFGPU_STREAM_PATIENCE_US");
    k.patience_us = p && *p ? (uint32_t)std::strtoul(p, nullptr, 10) : 200000u;
    return k;
}

// Streaming reconstruction (k_intra_stream beside the spread parse) for the
// small batches (up to 192 pictures: four 4032x3024 images, kStreamMaxPics)
bool intra_stream_for(int parse_mode, int n_pics, bool has_assembly, const StreamKnobs &k) {
    return k.enabled && parse_mode == PARSE_SPREAD && !has_assembly && n_pics > 0 && n_pics <= k.max_pics;
}

}  // namespace hg
