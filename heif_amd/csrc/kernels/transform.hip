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
#include "xform.hpp"

namespace hg {

namespace {

#ifndef HG_XF_WAVES
#define HG_XF_WAVES 4
#endif
constexpr int kWaves = HG_XF_WAVES;

#define wave_sync() HG_WAVE_SYNC()

}  // namespace

// 7 waves per SIMD (72 VGPRs, one of them spilled): the MFMA path of transform_tb
// alone takes the kernel to 112 (4 waves); at 6 waves k_transform alone is 8.0 ms,
// at 7 7.5 ms (A/B in DESIGN 5.11)
#if !defined(HG_XF_WPE)
#define HG_XF_WPE 7
#endif
__global__ void __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(HG_XF_WPE))) k_transform(BatchArgs a) {
    // per wave: the scaled coefficients d and the first-stage output g, both
    // clipped to 16 bits by 8.6.2 / 8.6.4.2, so int16 tiles (4 KiB per wave);
    // the 32x32 DCT matrix in LDS (lane-varying rows: LDS, not constant loads).
    // (Computing g in place of d through registers halves the LDS but raised
    // VGPRs 34 -> 70 and measured 14.6 -> 18.6 ms.)
    HG_BLOCK_SHARED __attribute__((aligned(16))) int16_t dtile[kWaves][32 * kXfDStride32];
    HG_BLOCK_SHARED __attribute__((aligned(16))) int16_t gtile[kWaves][32 * 32];
    HG_BLOCK_SHARED int32_t extent[kWaves][2];  // last nonzero row / column of d
    HG_BLOCK_SHARED XfTab s_tab;
    // the workgroup's threads copy the tables (the host emulation runs one thread per wave)
#if defined(HG_HOST_EMU)
    xf_tables(&s_tab, 0, 1);
#else
    xf_tables(&s_tab, (int)threadIdx.x, (int)blockDim.x);
#endif
    const int16_t *s_mt = s_tab.mt;
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
    const CoefSrc<false> coefs{a.coefs + pd.coef_off + (uint64_t)row * pd.coef_cap_row};
    const int W = sp.width, H = sp.height;
    // (made scalar: formed with VALU selects they took a VGPR each, and at the
    // 72-VGPR budget one of them spilled to scratch)
    const int cw = HG_UNI(sp.chroma_format ? W >> chroma_sx(sp.chroma_format) : 0);
    const int ch = HG_UNI(sp.chroma_format ? H >> chroma_sy(sp.chroma_format) : 0);
    // global memory in the type: selected by cidx the pointers would be flat,
    // and flat stores count in lgkmcnt, so every LDS wait would wait for them
    int16_t HG_GAS *const res0 = (int16_t HG_GAS *)(a.resid + pd.resid_off);
    int16_t HG_GAS *res_plane[3] = {res0, res0 + (size_t)W * H, res0 + (size_t)W * H + (size_t)cw * ch};
    const int pitch[3] = {W, cw, cw};
    const bool scaling = (sp.flags & SP_SCALING_LIST) != 0;
    int16_t *d = dtile[wave];
    int16_t *g = gtile[wave];

    // Pass A: 4x4 TBs, four at a time, 16 lanes each (sub-tile q of d / g).
    // A 4x4 TB has 16 outputs; run one per wave it left 48 lanes idle and paid
    // a full round of tile zeroing, extent atomics and wave syncs per TB.
    // Every phase loops over the 64 virtual lanes (one iteration on the GPU;
    // the host emulation runs one lane per wave).
    {
        const uint32_t mine = ntu > (uint32_t)wave ? (ntu - (uint32_t)wave + kWaves - 1) / kWaves : 0;
        // the wave's j-th record: a coded 4x4 TB inside its plane?
        auto want4 = [&](const TuRec &tu) -> bool {
            const int cidx = tu.flags & TU_CIDX_MASK;
            return (tu.flags & TU_CBF) && tu.log2 == 2 && cidx <= 2 && tu.x + 4 <= pitch[cidx] &&
                   tu.y + 4 <= (cidx ? ch : H);
        };
        // one round: up to four TBs, group q = vl >> 4 runs TB q (grp(vl, tu))
        auto round4 = [&](auto &&grp) {
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
                    const Coef c = coefs.word(tu.coef + (uint32_t)l16);
                    pos = (int)(c & 15u);
                    dv = (int)(int16_t)(c >> 16);
                } else {  // one sub-block record; lane l16 decodes scan position l16
                    if (tu.ncoef < 4) continue;
                    const SbRec r = load_rec(coefs, tu.coef);
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
                d[(vl & 48) + ((pos & 3) << 2) + (pos >> 2)] = (int16_t)dv;  // transposed: dT[x][y]
            }
            wave_sync();
            // first stage: g[y][x] = clip16((sum_k M[k][y] dT[x][k] + 64) >> 7), two dot products
            for (int vl = lane; vl < 64; vl += kWave) {
                TuRec tu;
                if (!grp(vl, tu) || (tu.flags & (TU_BYPASS | TU_TSKIP))) continue;
                const int y = (vl & 15) >> 2, x = vl & 3;
                const uint32_t *pa = reinterpret_cast<const uint32_t *>(mt_of(s_mt, 2, (tu.flags & TU_DST) != 0) + y * 4);
                const uint32_t *pb = reinterpret_cast<const uint32_t *>(d + (vl & 48) + x * 4);
                const int s = dot2_i16(pa[1], pb[1], dot2_i16(pa[0], pb[0], 0));
                g[vl] = (int16_t)min(max((s + 64) >> 7, -32768), 32767);
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
                    r = dq[x * 4 + y];
                } else if (tu.flags & TU_TSKIP) {
                    r = (dq[x * 4 + y] * (1 << 7) + (1 << (bd2 - 1))) >> bd2;  // tsShift = 5 + log2(4)
                } else {  // 4 terms of |g| <= 2^15 times |M| <= 90
                    const uint32_t *pa = reinterpret_cast<const uint32_t *>(mt_of(s_mt, 2, (tu.flags & TU_DST) != 0) + x * 4);
                    const uint32_t *pb = reinterpret_cast<const uint32_t *>(gq + y * 4);
                    const int s = dot2_i16(pa[1], pb[1], dot2_i16(pa[0], pb[0], 0));
                    r = (s + (1 << (bd2 - 1))) >> bd2;
                }
                res_plane[cidx][(size_t)(tu.y + y) * pitch[cidx] + tu.x + x] = (int16_t)clip16(r);
            }
            wave_sync();
        };
#if defined(HG_HOST_EMU)
        for (uint32_t j = 0; j < mine; j += 4) {
            round4([&](int vl, TuRec &tu) -> bool {
                const uint32_t jq = j + (uint32_t)(vl >> 4);
                if (jq >= mine) return false;
                tu = tus[(uint32_t)wave + kWaves * jq];
                return want4(tu);
            });
        }
#else
        // the rounds take the coded 4x4 TBs only: 64 of the wave's records per
        // coalesced load, a ballot of the wanted ones, four set bits per round
        // (rounds over consecutive records, coded or not, ran mostly empty groups)
        static_assert(kWave == 64, "one record per lane");
        for (uint32_t c0 = 0; c0 < mine; c0 += 64) {
            const uint32_t jl = c0 + (uint32_t)lane;
            uint4 rec = make_uint4(0, 0, 0, 0);
            if (jl < mine) rec = *reinterpret_cast<const uint4 *>(tus + (uint32_t)wave + kWaves * jl);
            TuRec rl;
            __builtin_memcpy(&rl, &rec, sizeof(rl));
            uint64_t todo = __ballot(jl < mine && want4(rl));
            while (todo) {
                int src = -1;
                for (int q = 0; q < 4 && todo; ++q) {
                    const int jq = __builtin_ctzll(todo);
                    todo &= todo - 1;
                    if (q == (lane >> 4)) src = jq;
                }
                const int sl = src < 0 ? 0 : src;
                const uint4 r = make_uint4((uint32_t)__shfl((int)rec.x, sl, 64), (uint32_t)__shfl((int)rec.y, sl, 64),
                                           (uint32_t)__shfl((int)rec.z, sl, 64), (uint32_t)__shfl((int)rec.w, sl, 64));
                TuRec tu_c;
                __builtin_memcpy(&tu_c, &r, sizeof(tu_c));
                const bool ok_c = src >= 0;
                round4([&](int, TuRec &tu) -> bool {
                    tu = tu_c;
                    return ok_c;
                });
            }
        }
#endif
    }

    // Pass B: every larger TB, one per wave
    auto pass_b = [&](const TuRec &tu) {
        const int cidx = tu.flags & TU_CIDX_MASK;
        transform_tb(tu, coefs, sp, a.sf, XfScratch{d, g, extent[wave], &s_tab},
                     res_plane[cidx] + (size_t)tu.y * pitch[cidx] + tu.x, pitch[cidx], lane);
    };
    auto wanted = [&](const TuRec &tu) {
        const int cidx = tu.flags & TU_CIDX_MASK, n = 1 << tu.log2;
        return (tu.flags & TU_CBF) && tu.log2 != 2 && tu.log2 <= 5 && cidx <= 2 && tu.x + n <= pitch[cidx] &&
               tu.y + n <= (cidx ? ch : H);
    };
#if defined(HG_HOST_EMU)
    for (uint32_t t = wave; t < ntu; t += kWaves)
        if (wanted(tus[t])) pass_b(tus[t]);
#else
    // the wave's next 64 records in one coalesced load, one per lane; the TBs it
    // transforms are the set bits of a ballot (a scalar load and its wait per
    // record, coded or not, before)
    for (uint32_t t0 = wave; t0 < ntu; t0 += 64u * kWaves) {
        const uint32_t t = t0 + (uint32_t)lane * kWaves;
        uint4 rec = make_uint4(0, 0, 0, 0);
        if (t < ntu) rec = *reinterpret_cast<const uint4 *>(tus + t);
        TuRec mine;
        __builtin_memcpy(&mine, &rec, sizeof(mine));
        uint64_t todo = __ballot(t < ntu && wanted(mine));
        while (todo) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint4 r = make_uint4((uint32_t)__builtin_amdgcn_readlane((int)rec.x, j),
                                       (uint32_t)__builtin_amdgcn_readlane((int)rec.y, j),
                                       (uint32_t)__builtin_amdgcn_readlane((int)rec.z, j),
                                       (uint32_t)__builtin_amdgcn_readlane((int)rec.w, j));
            TuRec tu;
            __builtin_memcpy(&tu, &r, sizeof(tu));
            pass_b(tu);
        }
    }
#endif
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
