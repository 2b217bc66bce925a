// transform.hip — scaling + inverse transform (pipeline stage 2).
//
// H.265 8.6.2 (residual derivation), 8.6.3 (scaling with ScalingFactor m and
// levelScale, 64-bit products, clip to 16 bits), 8.6.4.2 (two-stage inverse
// DST-VII 4x4 / DCT 4..32, first-stage (e + 64) >> 7 clipped to 16 bits,
// second stage + (20 - bitDepth) shift).  No reference code exists for this
// (slice.rs:253-255 is todo!()).
//
// Mapping: every coded TB is independent, so this stage runs at full chip
// parallelism: one 256-thread workgroup per CTB row of a picture, each wave
// taking every 4th TB of the row's TU list.  Coefficients arrive sparse
// (value, raster position) and are scattered into a per-wave int16 LDS tile
// (17 KiB per workgroup, so blocks fit beside the next decode's k_parse
// waves); the first stage only runs over the nonzero columns and rows, the
// second only over the nonzero first-stage columns, and a DC-only TB is a
// fill.  Integer sums on VALU with the DCT matrix in LDS — no MFMA (the
// products are exact int32, and TBs are at most 32x32).
#include "kernels.hpp"
#include "tables.hpp"

namespace hg {

namespace {

#ifndef HG_XF_WAVES
#define HG_XF_WAVES 4
#endif
constexpr int kWaves = HG_XF_WAVES;

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

#define wave_sync() HG_WAVE_SYNC()

__device__ __forceinline__ int clip16(int64_t v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : (int)v); }

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
    __device__ __forceinline__ int sum_abs(const Coef *row) const {
        const uint64_t x = nib();
        const uint64_t t = (x & 0x0f0f0f0f0f0f0f0full) + ((x >> 4) & 0x0f0f0f0f0f0f0f0full);
        int s = __builtin_popcount(sig()) + (int)((t * 0x0101010101010101ull) >> 56);
        const int ne = __builtin_popcountll(esc());
        for (int k = 0; k < ne; ++k) s += (int)row[esc0() - (uint32_t)k] - 16;
        return s;
    }
    // TransCoeffLevel at scan position nn (significant), given the number of
    // escapes at higher positions
    __device__ __forceinline__ int level(int nn, int esc_above, const Coef *row) const {
        const int a = (int)((nib() >> (4 * nn)) & 15u);
        const int abs_v = a < 15 ? a + 1 : (int)row[esc0() - (uint32_t)esc_above];
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
__device__ __forceinline__ SbRec load_rec(const Coef *p) {
#if defined(HG_HOST_EMU)
    return SbRec{p[0], p[1], p[2], p[3]};
#else
    const uint4 v = *reinterpret_cast<const uint4 *>(p);  // one 16-byte load
    return SbRec{v.x, v.y, v.z, v.w};
#endif
}

}  // namespace

__global__ void __launch_bounds__(kWaves * 64) k_transform(BatchArgs a) {
    // per wave: the scaled coefficients d and the first-stage output g, both
    // clipped to 16 bits by 8.6.2 / 8.6.4.2, so int16 tiles (4 KiB per wave);
    // the 32x32 DCT matrix in LDS (lane-varying rows: LDS, not constant loads).
    // (Computing g in place of d through registers halves the LDS but raised
    // VGPRs 34 -> 70 and measured 14.6 -> 18.6 ms.)
    HG_BLOCK_SHARED int16_t tile[kWaves][2][32 * 32];
    HG_BLOCK_SHARED int32_t extent[kWaves][2];  // last nonzero row / column of d
    HG_BLOCK_SHARED int8_t s_tm[32 * 32];
    HG_BLOCK_SHARED int8_t s_dst[16];
    // every wave fills the tables (same values; the host emulation runs one lane per wave)
    for (int i = (int)(threadIdx.x & 63); i < 32 * 32; i += kWave) s_tm[i] = c_tm.m[i >> 5][i & 31];
    for (int i = (int)(threadIdx.x & 63); i < 16; i += kWave) s_dst[i] = c_dst[i >> 2][i & 3];
    __syncthreads();
    const int pic = a.pic0 + blockIdx.y, row = blockIdx.x;
    const PicDesc pd = a.pics[pic];
    if (pd.flags & PD_ASSEMBLY) return;  // no coded data of its own
    const SeqParams sp = a.seqs[pd.seq];
    const int hctb = (sp.height + (1 << sp.log2_ctb) - 1) >> sp.log2_ctb;
    if (row >= hctb) return;
    const int wave = (int)HG_UNI(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t ntu = a.row_counts[2 * (pd.row_off + row)];
    const TuRec *tus = a.tus + pd.tu_off + (uint64_t)row * pd.tu_cap_row;
    const Coef *coefs = a.coefs + pd.coef_off + (uint64_t)row * pd.coef_cap_row;
    const int W = sp.width, H = sp.height;
    const int cw = sp.chroma_format ? W >> chroma_sx(sp.chroma_format) : 0;
    const int ch = sp.chroma_format ? H >> chroma_sy(sp.chroma_format) : 0;
    // global memory in the type: selected by cidx the pointers would be flat,
    // and flat stores count in lgkmcnt, so every LDS wait would wait for them
    int16_t HG_GAS *const res0 = (int16_t HG_GAS *)(a.resid + pd.resid_off);
    int16_t HG_GAS *res_plane[3] = {res0, res0 + (size_t)W * H, res0 + (size_t)W * H + (size_t)cw * ch};
    const int pitch[3] = {W, cw, cw};
    const bool scaling = (sp.flags & SP_SCALING_LIST) != 0;
    int16_t *d = tile[wave][0];
    int16_t *g = tile[wave][1];

    // Pass A: 4x4 TBs, four at a time, 16 lanes each (sub-tile q of d / g).
    // A 4x4 TB has 16 outputs; run one per wave it left 48 lanes idle and paid
    // a full round of tile zeroing, extent atomics and wave syncs per TB.
    // Every phase loops over the 64 virtual lanes (one iteration on the GPU;
    // the host emulation runs one lane per wave).
    {
        const uint32_t mine = ntu > (uint32_t)wave ? (ntu - (uint32_t)wave + kWaves - 1) / kWaves : 0;
        for (uint32_t j = 0; j < mine; j += 4) {
            // TB of group q = vl >> 4 in this round, if it is a coded 4x4 TB
            auto group_tb = [&](int vl, TuRec &tu) -> bool {
                const uint32_t jq = j + (uint32_t)(vl >> 4);
                if (jq >= mine) return false;
                tu = tus[(uint32_t)wave + kWaves * jq];
                const int cidx = tu.flags & TU_CIDX_MASK;
                return (tu.flags & TU_CBF) && tu.log2 == 2 && cidx <= 2 && tu.x + 4 <= pitch[cidx] &&
                       tu.y + 4 <= (cidx ? ch : H);
            };
            // the lane's record, loaded once per round (each phase below would
            // otherwise re-load it after the wave syncs)
#if defined(HG_HOST_EMU)
            auto grp = group_tb;
#else
            // one record per lane: each `vl` loop below runs once per lane (vl == lane)
            static_assert(kWave == 64, "the cached record assumes vl == lane");
            TuRec tu_c;
            const bool ok_c = group_tb(lane, tu_c);
            auto grp = [&](int, TuRec &tu) -> bool {
                tu = tu_c;
                return ok_c;
            };
#endif
            for (int vl = lane; vl < 64; vl += kWave) d[vl] = 0;
            wave_sync();
            for (int vl = lane; vl < 64; vl += kWave) {
                TuRec tu;
                const int l16 = vl & 15;
                if (!grp(vl, tu)) continue;
                const int cidx = tu.flags & TU_CIDX_MASK;
                const int bd = cidx ? sp.bit_depth_c : sp.bit_depth_y;
                int pos, dv;
                if (tu.flags & TU_PCM) {  // one word per sample
                    if (l16 >= (int)tu.ncoef) continue;
                    const Coef c = coefs[tu.coef + l16];
                    pos = (int)(c & 15u);
                    dv = (int)(int16_t)(c >> 16);
                } else {  // one sub-block record; lane l16 decodes scan position l16
                    if (tu.ncoef < 4) continue;
                    const SbRec r = load_rec(coefs + tu.coef);
                    if (!((r.sig() >> l16) & 1u)) continue;
                    const int above = l16 < 15 ? __builtin_popcountll(r.esc() >> (4 * l16 + 4)) : 0;  // (a shift by 64 is undefined)
                    dv = r.level(l16, above, coefs);
                    pos = r.pos(l16, 2);
                }
                if (!(tu.flags & TU_BYPASS)) {
                    const int qp = tu.qp, bd_shift = bd - 3;
                    const int ls = c_level_scale[qp % 6] << (qp / 6);
                    // pass B's use_m (scaling && !(ts && n > 4)) is just `scaling` at 4x4
                    const int m =
                        scaling ? a.sf[sp.sf_off + sf_size_offset(0) + (uint32_t)cidx * 16u + (uint32_t)pos] : 16;
                    dv = clip16(((int64_t)dv * m * ls + ((int64_t)1 << (bd_shift - 1))) >> bd_shift);
                }
                d[(vl & 48) + pos] = (int16_t)dv;
            }
            wave_sync();
            // first stage: g[y][x] = clip16((sum_k M[k][y] d[k][x] + 64) >> 7)
            for (int vl = lane; vl < 64; vl += kWave) {
                TuRec tu;
                if (!grp(vl, tu) || (tu.flags & (TU_BYPASS | TU_TSKIP))) continue;
                const int16_t *dq = d + (vl & 48);
                const int y = (vl & 15) >> 2, x = vl & 3;
                const bool dst_tr = (tu.flags & TU_DST) != 0;
                int32_t s = 0;
                for (int k = 0; k < 4; ++k)
                    s += (int32_t)(dst_tr ? s_dst[k * 4 + y] : s_tm[(k * 8) * 32 + y]) * dq[k * 4 + x];
                g[vl] = (int16_t)clip16(((int64_t)s + 64) >> 7);
            }
            wave_sync();
            // second stage (or bypass / transform skip) and the residual store
            for (int vl = lane; vl < 64; vl += kWave) {
                TuRec tu;
                if (!grp(vl, tu)) continue;
                const int cidx = tu.flags & TU_CIDX_MASK;
                const int bd2 = 20 - (cidx ? sp.bit_depth_c : sp.bit_depth_y);
                const int y = (vl & 15) >> 2, x = vl & 3;
                const int16_t *dq = d + (vl & 48), *gq = g + (vl & 48);
                int r;
                if (tu.flags & TU_BYPASS) {
                    r = dq[vl & 15];
                } else if (tu.flags & TU_TSKIP) {
                    r = (dq[vl & 15] * (1 << 7) + (1 << (bd2 - 1))) >> bd2;  // tsShift = 5 + log2(4)
                } else {
                    const bool dst_tr = (tu.flags & TU_DST) != 0;
                    int32_t s = 0;  // 4 terms of |g| <= 2^15 times |M| <= 90
                    for (int k = 0; k < 4; ++k)
                        s += (int32_t)(dst_tr ? s_dst[k * 4 + x] : s_tm[(k * 8) * 32 + x]) * gq[y * 4 + k];
                    r = (int)((s + (1 << (bd2 - 1))) >> bd2);
                }
                res_plane[cidx][(size_t)(tu.y + y) * pitch[cidx] + tu.x + x] = (int16_t)clip16(r);
            }
            wave_sync();
        }
    }

    // Pass B: every larger TB, one per wave
    for (uint32_t t = wave; t < ntu; t += kWaves) {
        const TuRec tu = tus[t];
        if (!(tu.flags & TU_CBF)) continue;
        if (tu.log2 == 2) continue;  // pass A
        const int cidx = tu.flags & TU_CIDX_MASK;
        const int log2n = tu.log2, n = 1 << log2n;
        if (log2n < 2 || log2n > 5 || cidx > 2 || tu.x + n > pitch[cidx] || tu.y + n > (cidx ? ch : H)) continue;
        const int bd = cidx ? sp.bit_depth_c : sp.bit_depth_y;
        const bool bypass = (tu.flags & TU_BYPASS) != 0, ts = (tu.flags & TU_TSKIP) != 0;
        // 1. zero the tile, scatter d[y][x] (scaled unless bypass)
        for (int i = lane; i < n * n / 2; i += kWave) reinterpret_cast<int32_t *>(d)[i] = 0;
        if (lane == 0) extent[wave][0] = extent[wave][1] = 0;
        wave_sync();
        const int qp = tu.qp;
        const int bd_shift = bd + log2n - 5;
        const int64_t rnd = (int64_t)1 << (bd_shift - 1);
        const int ls = c_level_scale[qp % 6] << (qp / 6);
        const bool use_m = scaling && !(ts && n > 4);
        const uint8_t *mtab = a.sf + sp.sf_off + sf_size_offset(log2n - 2) + (uint32_t)cidx * (uint32_t)(n * n);
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
            d[pos] = (int16_t)dv;
            my_row = max(my_row, pos >> log2n);
            my_col = max(my_col, pos & (n - 1));
        };
        if (tu.flags & TU_PCM) {  // one word per sample
            for (int k = lane; k < tu.ncoef; k += kWave) {
                const Coef c = coefs[tu.coef + k];
                put((int)(c & 0xffffu), (int)(int16_t)(c >> 16));
            }
        } else {  // 16 lanes per sub-block record, a scan position each (no serial loop per lane)
            const int nrec = (int)(tu.ncoef >> 2);
            for (int q = lane; q < 16 * nrec; q += kWave) {
                const SbRec r = load_rec(coefs + tu.coef + 4 * (q >> 4));  // (16 lanes, one address)
                const int nn = q & 15;
                if (!((r.sig() >> nn) & 1u)) continue;
                const int above = nn < 15 ? __builtin_popcountll(r.esc() >> (4 * nn + 4)) : 0;
                put(r.pos(nn, log2n), r.level(nn, above, coefs));
            }
        }
        if (my_row) atomicMax(&extent[wave][0], my_row);
        if (my_col) atomicMax(&extent[wave][1], my_col);
        wave_sync();
        const int rows = extent[wave][0] + 1, cols = extent[wave][1] + 1;  // d is zero beyond these
        const int bd2 = 20 - bd;
        int16_t HG_GAS *dst = res_plane[cidx] + (size_t)tu.y * pitch[cidx] + tu.x;
        if (bypass || ts) {
            // bypass: r = TransCoeffLevel; transform skip: r = (d << tsShift) then >> bdShift
            const int ts_shift = 5 + log2n;
            for (int i = lane; i < n * n; i += kWave) {
                int r = d[i];
                if (!bypass) r = (r * (1 << ts_shift) + (1 << (bd2 - 1))) >> bd2;
                dst[(i >> log2n) * pitch[cidx] + (i & (n - 1))] = (int16_t)clip16(r);
            }
            wave_sync();
            continue;
        }
        const bool dst_tr = (tu.flags & TU_DST) != 0;
        const int kstep = 32 >> log2n;
        if (!dst_tr && rows == 1 && cols == 1) {
            // DC only: both stages are constant (transMatrix[0][*] = 64)
            const int g0 = clip16(((int64_t)64 * d[0] + 64) >> 7);
            const int16_t r = (int16_t)clip16(((int64_t)64 * g0 + (1 << (bd2 - 1))) >> bd2);
            for (int i = lane; i < n * n; i += kWave) dst[(i >> log2n) * pitch[cidx] + (i & (n - 1))] = r;
            wave_sync();
            continue;
        }
        // 2. vertical (column) pass over the nonzero columns:
        //    e[y][x] = sum_{j < rows} M[j][y] d[j][x]; g = clip16((e + 64) >> 7)
        // columns padded to a power of two: shifts instead of a division per output
        const int lc = cols > 1 ? 32 - __builtin_clz((unsigned)(cols - 1)) : 0;
        for (int o = lane; o < (n << lc); o += kWave) {
            const int y = o >> lc, x = o & ((1 << lc) - 1);
            if (x >= cols) continue;
            int32_t s = 0;
            if (dst_tr) {
                for (int j = 0; j < rows; ++j) s += (int32_t)s_dst[j * 4 + y] * d[j * n + x];
            } else {
                for (int j = 0; j < rows; ++j) s += (int32_t)s_tm[(j * kstep) * 32 + y] * d[j * n + x];
            }
            g[y * n + x] = (int16_t)clip16(((int64_t)s + 64) >> 7);
        }
        wave_sync();
        // 3. horizontal (row) pass: r[y][x] = sum_{j < cols} M[j][x] g[y][j]; (r + rnd) >> (20 - bitDepth)
        //    (|g| <= 2^15 after clipping and |M| <= 90, so |sum| < 32 * 90 * 2^15 < 2^31: 32-bit)
        for (int o = lane; o < n * n; o += kWave) {
            const int y = o >> log2n, x = o & (n - 1);
            int32_t s = 0;
            if (dst_tr) {
                for (int j = 0; j < cols; ++j) s += (int32_t)s_dst[j * 4 + x] * g[y * n + j];
            } else {
                for (int j = 0; j < cols; ++j) s += (int32_t)s_tm[(j * kstep) * 32 + x] * g[y * n + j];
            }
            dst[y * pitch[cidx] + x] = (int16_t)clip16((s + (1 << (bd2 - 1))) >> bd2);
        }
        wave_sync();
    }
}

#if defined(HG_HOST_EMU)
void emu_transform(const BatchArgs &a) { emu_launch(k_transform, a.max_rows, a.n_pics, kWaves, a); }
#else
hipError_t launch_transform(const BatchArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(k_transform, dim3(a.max_rows, a.n_pics), dim3(kWaves * 64), 0, s, a);
    return hipGetLastError();
}
#endif

}  // namespace hg
