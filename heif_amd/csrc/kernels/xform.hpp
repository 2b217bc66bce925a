// xform.hpp — scaling + inverse transform of one TB by one wave (8.6.2-8.6.4),
// shared by k_transform (pass B) and k_intra's streaming mode, which
// transforms each TB just before predicting it.  The two matrix stages run as
// packed int16 dot products (4x4, 8x8 and the host emulation) or as int8
// MFMAs on split operands (16x16, 32x32; transform_mfma), bit-exact either way.
#pragma once
#include "kernels.hpp"
#include "tables.hpp"

namespace hg {
namespace {

// transMatrix of 8.6.4.2 (32x32 DCT; smaller sizes use rows k * 32/n)
struct TransMatrix {
    int8_t m[32][32];
};
constexpr TransMatrix make_matrix() {
    TransMatrix t{};
    constexpr int odd[16] = {90, 90, 88, 85, 82, 78, 73, 67, 61, 54, 46, 38, 31, 22, 13, 4};
    constexpr int e2[8] = {90, 87, 80, 70, 57, 43, 25, 9};
    constexpr int e4[4] = {89, 75, 50, 18};
    int cv[33] = {};
    cv[0] = 64;
    cv[8] = 83;
    cv[16] = 64;
    cv[24] = 36;
    cv[32] = 0;
    for (int i = 0; i < 16; ++i) cv[2 * i + 1] = odd[i];
    for (int i = 0; i < 8; ++i) cv[2 * (2 * i + 1)] = e2[i];
    for (int i = 0; i < 4; ++i) cv[4 * (2 * i + 1)] = e4[i];
    for (int k = 0; k < 32; ++k)
        for (int n = 0; n < 32; ++n) {
            int j = ((2 * n + 1) * k) % 128;
            int v = j <= 32 ? cv[j] : j <= 64 ? -cv[64 - j] : j <= 96 ? -cv[j - 64] : cv[128 - j];
            t.m[k][n] = (int8_t)v;
        }
    return t;
}
__constant__ TransMatrix c_tm = make_matrix();
__constant__ int8_t c_dst[4][4] = {{29, 55, 74, 84}, {74, 74, 0, -74}, {84, -29, -74, 55}, {55, -84, 74, -29}};
__constant__ int16_t c_level_scale[6] = {40, 45, 51, 57, 64, 72};

#define xf_sync() HG_WAVE_SYNC()

__device__ __forceinline__ int clip16(int64_t v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : (int)v); }

// A row's coefficient words.  Coherent: read with agent-scope loads, for a
// reader that runs beside the parse writing them (k_intra's streaming mode:
// the lines may sit stale in this XCD's L2 from an earlier decode).
template <bool Coherent>
struct CoefSrc {
    const Coef *p;
    __device__ __forceinline__ uint32_t word(uint32_t i) const {
#if !defined(HG_HOST_EMU)
        if constexpr (Coherent) return __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
        return p[i];
    }
};

// One sub-block record (SbRec, desc.hpp) of a TB's coefficient words.
struct SbRec {
    uint32_t w0, w1, w2, w3;
    __device__ __forceinline__ uint32_t sig() const { return w0 & 0xffffu; }
    __device__ __forceinline__ uint64_t nib() const { return (uint64_t)w1 | ((uint64_t)w2 << 32); }
    // nibble mask of the escapes (bit 4n set where abs - 1 is coded as 15)
    __device__ __forceinline__ uint64_t esc() const {
        const uint64_t x = nib();
        return x & (x >> 1) & (x >> 2) & (x >> 3) & 0x1111111111111111ull;
    }
    __device__ __forceinline__ uint32_t esc0() const { return w3 >> 9; }
    // raster position in an n-wide TB (log2n) of scan position nn
    __device__ __forceinline__ int pos(int nn, int log2n) const {
        const uint32_t sc = (w3 >> 6) & 3u;  // (selected, not indexed: the words stay immediates)
        const uint64_t sw = sc == 0 ? kScan4Pos[0] : (sc == 1 ? kScan4Pos[1] : kScan4Pos[2]);
        const uint32_t pp = (uint32_t)(sw >> (4 * nn)) & 15u;
        const int x = (int)((w3 & 7u) << 2) + (int)(pp & 3u), y = (int)(((w3 >> 3) & 7u) << 2) + (int)(pp >> 2);
        return (y << log2n) + x;
    }
    // the hidden sign's parity: the sum of the sub-block's levels
    template <class Src>
    __device__ __forceinline__ int sum_abs(const Src &row) const {
        const uint64_t x = nib();
        const uint64_t t = (x & 0x0f0f0f0f0f0f0f0full) + ((x >> 4) & 0x0f0f0f0f0f0f0f0full);
        int s = __builtin_popcount(sig()) + (int)((t * 0x0101010101010101ull) >> 56);
        const int ne = __builtin_popcountll(esc());
        for (int k = 0; k < ne; ++k) s += (int)row.word(esc0() - (uint32_t)k) - 16;
        return s;
    }
    // TransCoeffLevel at scan position nn (significant), given the number of
    // escapes at higher positions
    template <class Src>
    __device__ __forceinline__ int level(int nn, int esc_above, const Src &row) const {
        const int a = (int)((nib() >> (4 * nn)) & 15u);
        const int abs_v = a < 15 ? a + 1 : (int)row.word(esc0() - (uint32_t)esc_above);
        const uint32_t s = sig();
        bool neg;
        if (((w3 >> 8) & 1u) && nn == __builtin_ctz(s)) {
            neg = (sum_abs(row) & 1) != 0;
        } else {
            const int rank = __builtin_popcount(s >> (nn + 1));
            neg = ((w0 << rank) >> 31) != 0;
        }
        const int v = neg ? -abs_v : abs_v;
        return v < -32768 ? -32768 : (v > 32767 ? 32767 : v);
    }
};
template <bool Coherent>
__device__ __forceinline__ SbRec load_rec(const CoefSrc<Coherent> &src, uint32_t i) {
#if defined(HG_HOST_EMU)
    const Coef *p = src.p + i;
    return SbRec{p[0], p[1], p[2], p[3]};
#else
    if constexpr (Coherent) {  // two agent-scope 8-byte loads
        const uint64_t *q = reinterpret_cast<const uint64_t *>(src.p + i);
        const uint64_t lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return SbRec{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
    }
    const uint4 v = *reinterpret_cast<const uint4 *>(src.p + i);  // one 16-byte load
    return SbRec{v.x, v.y, v.z, v.w};
#endif
}


// 8x8 .. 32x32 TBs: both stages as dot products of packed int16 pairs
// (v_dot2c_i32_i16: two multiply-adds per instruction, four per pair of
// 8-byte LDS reads).  The first stage reads d column-wise, so d is scattered
// transposed (dT[x][y], row stride n + 2: columns of a 32-wide tile in
// distinct banks); the matrix is kept transposed per size, mtT_n[y][j] =
// transMatrix[j * 32 / n][y], same stride, so both operands of every dot run
// along j.  (r04's loops: one int8 matrix load, one int16 load and a
// multiply-add per term, ~7 instructions per term.)
// 4x4: the DCT and the DST (luma) matrices, transposed the same way, row
// stride 4 (an 8-byte read per row, four lanes per TB column).
constexpr int kXfDStride32 = 32 + 2;
constexpr int kMt4Dct = 8 * 10 + 16 * 18 + 32 * 34, kMt4Dst = kMt4Dct + 16;
constexpr int kMtElems = kMt4Dst + 16;  // int16
__device__ __forceinline__ int mt_off(int log2n) { return log2n == 3 ? 0 : (log2n == 4 ? 8 * 10 : 8 * 10 + 16 * 18); }

// The workgroup's transform tables (LDS copy of c_xf, built at compile time:
// filling them per workgroup with an integer division per entry cost
// k_transform 7 % of its VALU): the transposed matrices of the dot products,
// which the MFMA path's operands are packed from as well.
struct alignas(16) XfTab {
    int16_t mt[kMtElems];
};
static_assert(sizeof(XfTab) % 16 == 0 && (sizeof(int16_t) * kMtElems) % 16 == 0, "XfTab layout");

// a wave's transform scratch: d (int16, 32 x 34: the transposed layout's
// padding) and g (32x32) tiles, the extent pair, and the workgroup's tables
struct XfScratch {
    int16_t *d, *g;
    int32_t *extent;
    const XfTab *tab;
};

constexpr XfTab make_xf_tab() {
    XfTab t{};
    const TransMatrix m = make_matrix();
    constexpr int dst4[4][4] = {{29, 55, 74, 84}, {74, 74, 0, -74}, {84, -29, -74, 55}, {55, -84, 74, -29}};
    for (int i = 0; i < kMtElems; ++i) {
        if (i >= kMt4Dct) {  // 4x4: mtT[y][k] = M[k][y]
            const int k = i & 3, y = (i >> 2) & 3;
            t.mt[i] = (int16_t)(i >= kMt4Dst ? dst4[k][y] : m.m[k * 8][y]);
            continue;
        }
        const int l2 = i < 80 ? 3 : (i < 80 + 288 ? 4 : 5), n = 1 << l2, sn = n + 2;
        const int k = i - (l2 == 3 ? 0 : (l2 == 4 ? 80 : 80 + 288));
        const int y = k / sn, j = k % sn;
        t.mt[i] = (int16_t)(j < n ? m.m[j << (5 - l2)][y] : 0);
    }
    return t;
}
__constant__ XfTab c_xf = make_xf_tab();

// the tables from the constant copy, thread `tid` of `nth` (as dwords)
__device__ __forceinline__ void xf_tables(XfTab *dst, int tid, int nth = kWave) {
    for (int i = tid; i < (int)(sizeof(XfTab) / 4); i += nth)
        reinterpret_cast<uint32_t *>(dst)[i] = reinterpret_cast<const uint32_t *>(&c_xf)[i];
}

#if !defined(HG_HOST_EMU) && !defined(HG_XF_NO_MFMA)
// 16x16 and 32x32 TBs on the int8 MFMA (v_mfma_i32_32x32x32_i8, 16x16 zero
// padded), bit-exact: an int16 operand v is split as v = 256 hi + lo' + 128
// with hi = v >> 8 and lo' = (v & 255) - 128 both int8, so a product is
// 256 (hi . B) + (lo' . B) + 128 colsum(B), the last term the accumulator's
// start value (corr, the column sums by dot products of the packed B).  Stage 1 computes G^T = D^T M with D^T rows from the
// transposed tile (lane = TB column x, k = 16h .. 16h + 15); its result holds
// G[y][x] with y on the lane and x = (i & 3) + 8 (i >> 2) + 4h in register i,
// which is stage 2's A operand (R = G M) as it stands, with B's rows permuted
// to match (b2).  Both B operands are packed per TB from the int16 table mt
// (mtT_n, row y = M_n[.][y] at stride sn): an LDS copy of int8 tables took
// the workgroup below 7 per CU (A/B: 0.6 ms of k_transform).  Operand maps checked on the hardware
// (tools/probe/mfma_i8_probe.cpp).  Four MFMAs and ~150 VALU per TB against
// ~2,400 instructions of dot products for a 32x32 TB.
typedef int xf_v4i __attribute__((ext_vector_type(4)));
typedef int xf_v16i __attribute__((ext_vector_type(16)));
__device__ __forceinline__ int xf_hi(uint32_t w0, uint32_t w1) {
    return (int)__builtin_amdgcn_perm(w1, w0, 0x07050301u);
}
__device__ __forceinline__ int xf_lo(uint32_t w0, uint32_t w1) {
    return (int)(__builtin_amdgcn_perm(w1, w0, 0x06040200u) ^ 0x80808080u);
}
// four int16 values held in int32 registers to their packed high bytes / low bytes ^ 0x80
__device__ __forceinline__ int xf_hi4(int g0, int g1, int g2, int g3) {
    return (int)(__builtin_amdgcn_perm((uint32_t)g1, (uint32_t)g0, 0x0c0c0501u) |
                 (__builtin_amdgcn_perm((uint32_t)g3, (uint32_t)g2, 0x0c0c0501u) << 16));
}
__device__ __forceinline__ int xf_lo4(int g0, int g1, int g2, int g3) {
    return (int)((__builtin_amdgcn_perm((uint32_t)g1, (uint32_t)g0, 0x0c0c0400u) |
                  (__builtin_amdgcn_perm((uint32_t)g3, (uint32_t)g2, 0x0c0c0400u) << 16)) ^ 0x80808080u);
}
// the low bytes of the int16 pairs (w0, w1): four int8 values
__device__ __forceinline__ int xf_b8(uint32_t w0, uint32_t w1) {
    return (int)__builtin_amdgcn_perm(w1, w0, 0x06040200u);
}
template <class DstPtr>
__device__ __forceinline__ void transform_mfma(const int16_t *dT, int sn, int log2n, const int16_t *mt, DstPtr dst,
                                               int pitch, int bd2, int lane) {
    const int n = 1 << log2n, r = lane & 31, h = lane >> 5;
    // lane (r, h): b1 = M[16h + jj][r], b2 = M[8q + 4h + (jj & 3)][r] in register q (zero past n)
    const bool live = r < n, live1 = live && 16 * h < n;
    const uint32_t *pm = reinterpret_cast<const uint32_t *>(mt + (live ? r : 0) * sn);
    const uint32_t *pm1 = pm + (live1 ? 8 * h : 0);
    const xf_v4i b1 = {live1 ? xf_b8(pm1[0], pm1[1]) : 0, live1 ? xf_b8(pm1[2], pm1[3]) : 0,
                       live1 ? xf_b8(pm1[4], pm1[5]) : 0, live1 ? xf_b8(pm1[6], pm1[7]) : 0};
    const uint32_t *pm2 = pm + 2 * h;
    const bool live2 = live && n == 32;  // (registers 2, 3 hold k >= 16)
    const xf_v4i b2 = {live ? xf_b8(pm2[0], pm2[1]) : 0, live ? xf_b8(pm2[4], pm2[5]) : 0,
                       live2 ? xf_b8(pm2[8], pm2[9]) : 0, live2 ? xf_b8(pm2[12], pm2[13]) : 0};
    // 128 colsum_r(M): this lane's 16 entries of b1 and its partner's (lane ^ 32)
    int cs = __builtin_amdgcn_sdot4(b1.x, 0x01010101, 0, false);
    cs = __builtin_amdgcn_sdot4(b1.y, 0x01010101, cs, false);
    cs = __builtin_amdgcn_sdot4(b1.z, 0x01010101, cs, false);
    cs = __builtin_amdgcn_sdot4(b1.w, 0x01010101, cs, false);
    const int corr = 128 * (cs + __shfl_xor(cs, 32, 64));
    const uint32_t *pa = reinterpret_cast<const uint32_t *>(dT + r * sn + 16 * h);
    const xf_v4i ah = {xf_hi(pa[0], pa[1]), xf_hi(pa[2], pa[3]), xf_hi(pa[4], pa[5]), xf_hi(pa[6], pa[7])};
    const xf_v4i al = {xf_lo(pa[0], pa[1]), xf_lo(pa[2], pa[3]), xf_lo(pa[4], pa[5]), xf_lo(pa[6], pa[7])};
    // the high bytes' product, scaled and corrected, starts the low bytes' one
    xf_v16i acc = {};
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(ah, b1, acc, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = (acc[i] << 8) + corr;
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(al, b1, acc, 0, 0, 0);
    int g[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) g[i] = min(max((acc[i] + 64) >> 7, -32768), 32767);
    const xf_v4i gh = {xf_hi4(g[0], g[1], g[2], g[3]), xf_hi4(g[4], g[5], g[6], g[7]),
                       xf_hi4(g[8], g[9], g[10], g[11]), xf_hi4(g[12], g[13], g[14], g[15])};
    const xf_v4i gl = {xf_lo4(g[0], g[1], g[2], g[3]), xf_lo4(g[4], g[5], g[6], g[7]),
                       xf_lo4(g[8], g[9], g[10], g[11]), xf_lo4(g[12], g[13], g[14], g[15])};
    acc = xf_v16i{};
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(gh, b2, acc, 0, 0, 0);
    const int rnd = 1 << (bd2 - 1);
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = (acc[i] << 8) + corr + rnd;
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(gl, b2, acc, 0, 0, 0);
    // rows y = (i & 3) + 8 (i >> 2) + 4h: all inside a 32x32 TB; inside a 16x16
    // one exactly for i < 8, with the columns r < 16 (one lane-dependent region
    // instead of a compare and an exec-mask region per store)
    auto out = [&](int i) {
        const int y = (i & 3) + 8 * (i >> 2) + 4 * h;
        dst[y * pitch + r] = (int16_t)min(max(acc[i] >> bd2, -32768), 32767);
    };
    if (n == 32) {
#pragma unroll
        for (int i = 0; i < 16; ++i) out(i);
    } else if (r < n) {
#pragma unroll
        for (int i = 0; i < 8; ++i) out(i);
    }
}
#endif

// the transposed matrix of a TB of size 1 << log2n (DST: 4x4 luma), and its row stride
__device__ __forceinline__ const int16_t *mt_of(const int16_t *mt, int log2n, bool dst_tr) {
    return log2n == 2 ? mt + (dst_tr ? kMt4Dst : kMt4Dct) : mt + mt_off(log2n);
}
__device__ __forceinline__ int mt_stride(int log2n) { return log2n == 2 ? 4 : (1 << log2n) + 2; }

// s + a.lo * b.lo + a.hi * b.hi (signed 16-bit halves)
__device__ __forceinline__ int dot2_i16(uint32_t a, uint32_t b, int s) {
#if defined(HG_HOST_EMU)
    return s + (int)(int16_t)(a & 0xffffu) * (int)(int16_t)(b & 0xffffu) + (int)(int16_t)(a >> 16) * (int)(int16_t)(b >> 16);
#else
    typedef short short2_t __attribute__((ext_vector_type(2)));
    short2_t va, vb;
    __builtin_memcpy(&va, &a, 4);
    __builtin_memcpy(&vb, &b, 4);
    return __builtin_amdgcn_sdot2(va, vb, s, false);
#endif
}

// Residual of coded TB `tu` into dst (row pitch `pitch` samples) by one wave.
// The caller has checked that the TB lies inside its plane.
// dst: the residual plane (global) or, in k_intra's streaming mode, X.d itself
// (pitch n: the last pass no longer reads d)
template <bool Coherent, class DstPtr>
__device__ __forceinline__ void transform_tb(const TuRec &tu, const CoefSrc<Coherent> &coefs, const SeqParams &sp,
                                             const uint8_t *sf, const XfScratch &X, DstPtr dst, int pitch, int lane) {
    int16_t *d = X.d, *g = X.g;
    const bool scaling = (sp.flags & SP_SCALING_LIST) != 0;
    const int cidx = tu.flags & TU_CIDX_MASK;
    const int log2n = tu.log2, n = 1 << log2n;
    if (log2n < 2 || log2n > 5 || cidx > 2) return;
    const int bd = cidx ? sp.bit_depth_c : sp.bit_depth_y;
    const bool bypass = (tu.flags & TU_BYPASS) != 0, ts = (tu.flags & TU_TSKIP) != 0;
    // 1. zero the tile, scatter d[y][x] (scaled unless bypass; transposed for the dot-product stages)
    const bool dots = !bypass && !ts;
    const int sn = mt_stride(log2n);
    for (int i = lane; i < (dots ? n * sn : n * n) / 2; i += kWave) reinterpret_cast<int32_t *>(d)[i] = 0;
    if (lane == 0) X.extent[0] = X.extent[1] = 0;
    xf_sync();
    const int qp = tu.qp;
    const int bd_shift = bd + log2n - 5;
    const int64_t rnd = (int64_t)1 << (bd_shift - 1);
    const int ls = c_level_scale[qp % 6] << (qp / 6);
    const bool use_m = scaling && !(ts && n > 4);
    const uint8_t *mtab = sf + sp.sf_off + sf_size_offset(log2n - 2) + (uint32_t)cidx * (uint32_t)(n * n);
    int my_row = 0, my_col = 0;
    auto put = [&](int pos, int v) {
        pos &= n * n - 1;
        int dv;
        if (bypass) {
            dv = v;
        } else {
            const int m = use_m ? mtab[pos] : 16;
            dv = clip16(((int64_t)v * m * ls + rnd) >> bd_shift);
        }
        d[dots ? (pos & (n - 1)) * sn + (pos >> log2n) : pos] = (int16_t)dv;
        my_row = max(my_row, pos >> log2n);
        my_col = max(my_col, pos & (n - 1));
    };
    if (tu.flags & TU_PCM) {  // one word per sample
        for (int k = lane; k < tu.ncoef; k += kWave) {
            const Coef c = coefs.word(tu.coef + (uint32_t)k);
            put((int)(c & 0xffffu), (int)(int16_t)(c >> 16));
        }
    } else {  // 16 lanes per sub-block record, a scan position each (no serial loop per lane)
        const int nrec = (int)(tu.ncoef >> 2);
        for (int q = lane; q < 16 * nrec; q += kWave) {
            const SbRec r = load_rec(coefs, tu.coef + 4u * (uint32_t)(q >> 4));  // (16 lanes, one address)
            const int nn = q & 15;
            if (!((r.sig() >> nn) & 1u)) continue;
            const int above = nn < 15 ? __builtin_popcountll(r.esc() >> (4 * nn + 4)) : 0;
            put(r.pos(nn, log2n), r.level(nn, above, coefs));
        }
    }
    if (my_row) atomicMax(&X.extent[0], my_row);
    if (my_col) atomicMax(&X.extent[1], my_col);
    xf_sync();
    const int rows = X.extent[0] + 1, cols = X.extent[1] + 1;  // d is zero beyond these
    const int bd2 = 20 - bd;
    if (bypass || ts) {
        // bypass: r = TransCoeffLevel; transform skip: r = (d << tsShift) then >> bdShift
        const int ts_shift = 5 + log2n;
        for (int i = lane; i < n * n; i += kWave) {
            int r = d[i];
            if (!bypass) r = (r * (1 << ts_shift) + (1 << (bd2 - 1))) >> bd2;
            dst[(i >> log2n) * pitch + (i & (n - 1))] = (int16_t)clip16(r);
        }
        xf_sync();
        return;
    }
    const bool dst_tr = (tu.flags & TU_DST) != 0;
    if (!dst_tr && rows == 1 && cols == 1) {
        // DC only: both stages are constant (transMatrix[0][*] = 64)
        const int g0 = clip16(((int64_t)64 * d[0] + 64) >> 7);
        const int16_t r = (int16_t)clip16(((int64_t)64 * g0 + (1 << (bd2 - 1))) >> bd2);
        for (int i = lane; i < n * n; i += kWave) dst[(i >> log2n) * pitch + (i & (n - 1))] = r;
        xf_sync();
        return;
    }
#if !defined(HG_HOST_EMU) && !defined(HG_XF_NO_MFMA)
    // 16x16 / 32x32 on the int8 MFMA, every such TB past the DC shortcut (A/B in DESIGN
    // 5.11, also against sparse TBs left on the dot products); the host emulation and
    // the smaller TBs take the dot products below, which the MFMA path matches bit for bit
    if (log2n >= 4) {
        transform_mfma(d, sn, log2n, mt_of(X.tab->mt, log2n, false), dst, pitch, bd2, lane);
        xf_sync();
        return;
    }
#endif
    // 2. e[y][x] = sum_{j < rows} M[j][y] dT[x][j] over the nonzero columns, rounded up to a
    //    multiple of four (d is zero there, so g is too): the row pass's dots read whole quads
    const int16_t *mt = mt_of(X.tab->mt, log2n, dst_tr);
    const int rows4 = (rows + 3) & ~3, cols4 = (cols + 3) & ~3;
    const int lc = cols4 > 4 ? 32 - __builtin_clz((unsigned)(cols4 - 1)) : 2;
    for (int o = lane; o < (n << lc); o += kWave) {
        const int y = o >> lc, x = o & ((1 << lc) - 1);
        if (x >= cols4) continue;
        const uint32_t *pa = reinterpret_cast<const uint32_t *>(mt + y * sn);
        const uint32_t *pb = reinterpret_cast<const uint32_t *>(d + x * sn);
        int s = 0;
#pragma unroll 2
        for (int j = 0; j < rows4 / 2; j += 2) {
            s = dot2_i16(pa[j], pb[j], s);
            s = dot2_i16(pa[j + 1], pb[j + 1], s);
        }
        g[y * n + x] = (int16_t)min(max((s + 64) >> 7, -32768), 32767);  // (|s| < 2^27: 32-bit)
    }
    xf_sync();
    // 3. r[y][x] = sum_{j < cols} M[j][x] g[y][j]: (r + rnd) >> (20 - bitDepth)
    for (int o = lane; o < n * n; o += kWave) {
        const int y = o >> log2n, x = o & (n - 1);
        const uint32_t *pa = reinterpret_cast<const uint32_t *>(mt + x * sn);
        const uint32_t *pb = reinterpret_cast<const uint32_t *>(g + y * n);
        int s = 0;
#pragma unroll 2
        for (int j = 0; j < cols4 / 2; j += 2) {
            s = dot2_i16(pa[j], pb[j], s);
            s = dot2_i16(pa[j + 1], pb[j + 1], s);
        }
        dst[y * pitch + x] = (int16_t)min(max((s + (1 << (bd2 - 1))) >> bd2, -32768), 32767);
    }
    xf_sync();
}

}  // namespace
}  // namespace hg
