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
// row; row r starts CTU c once row r-1 has finished CTU c+1 (every above-right
// neighbour lies in CTU c+1 at most), signalled through per-wave progress
// counters in LDS with workgroup-scope release/acquire — all waves of a
// picture share one CU, so the reconstructed samples they exchange through
// global memory stay coherent in that CU's L1.  Inside a TB all 64 lanes
// work: reference samples are gathered one per lane, the substitution
// process (8.4.4.2.2) becomes three 64-bit ballots + a nearest-available
// lookup, and prediction/residual-add run one sample per lane.
#include "kernels.hpp"

namespace hg {

namespace {

constexpr int kWaves = 16;

__constant__ int8_t c_angle[35] = {0, 0, 32, 26, 21, 17, 13, 9, 5, 2, 0, -2, -5, -9, -13, -17, -21, -26,
                                   -32, -26, -21, -17, -13, -9, -5, -2, 0, 2, 5, 9, 13, 17, 21, 26, 32};
__constant__ int16_t c_inv_angle[35] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, -4096, -1638, -910, -630, -482, -390, -315,
                                        -256, -315, -390, -482, -630, -910, -1638, -4096, 0, 0, 0, 0, 0, 0, 0, 0, 0};

struct alignas(16) IntraLds {
    int16_t left[132];  // [0] = p[-1][-1], [1+y] = p[-1][y]
    int16_t top[132];   // [0] = p[-1][-1], [1+x] = p[x][-1]
    int16_t fl[132];
    int16_t ft[132];
    int16_t ref[200];   // angular reference, index + 64
    int32_t dc;
};

#define wave_sync() HG_WAVE_SYNC()

// 6.4.1 MinTbAddrZs for a luma location
__device__ __forceinline__ int zscan(int xl, int yl, int log2ctb, int min_tb, int wctb) {
    const int tbx = xl >> min_tb, tby = yl >> min_tb, sh = log2ctb - min_tb;
    int v = ((tbx >> sh) + (tby >> sh) * wctb) << (2 * sh);
    for (int i = 0; i < sh; ++i) v |= (((tbx >> i) & 1) << (2 * i)) | (((tby >> i) & 1) << (2 * i + 1));
    return v;
}

template <typename Pel>
__device__ __attribute__((always_inline)) inline void predict_tb(IntraLds *L, const TuRec &tu, Pel *plane, int pitch, int PW, int PH, int cidx,
                           const int16_t *res, int res_pitch, int bd, bool strong, int log2ctb, int min_tb,
                           int wctb, int lane) {
    const int log2n = tu.log2, n = 1 << log2n, mode = tu.mode;
    const int x0 = tu.x, y0 = tu.y;
    const int sub = cidx ? 1 : 0;  // 4:2:0 chroma → luma = 2x
    const int zcur = zscan(x0 << sub, y0 << sub, log2ctb, min_tb, wctb);
    const int ns = 4 * n + 1;
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
            sa[s] = xn >= 0 && yn >= 0 && xn < PW && yn < PH &&
                    zscan(xn << sub, yn << sub, log2ctb, min_tb, wctb) <= zcur;
            sv[s] = sa[s] ? (int)plane[(size_t)yn * pitch + xn] : 0;
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
#else
    int val[3];
    uint64_t msk[3];
    for (int k = 0; k < 3; ++k) {
        const int s = lane + 64 * k;
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
        bool av = s < ns && xn >= 0 && yn >= 0 && xn < PW && yn < PH &&
                  zscan(xn << sub, yn << sub, log2ctb, min_tb, wctb) <= zcur;
        val[k] = av ? (int)plane[(size_t)yn * pitch + xn] : 0;
        msk[k] = __ballot(av);
    }
    // 2. substitution: nearest available predecessor in search order, else the first available
    const bool any = (msk[0] | msk[1] | msk[2]) != 0;
    for (int k = 0; k < 3; ++k) {
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
        const int v0 = __shfl(val[0], sl, 64), v1 = __shfl(val[1], sl, 64), v2 = __shfl(val[2], sl, 64);
        const int v = !any ? (1 << (bd - 1)) : (sc == 0 ? v0 : (sc == 1 ? v1 : v2));
        if (s < 2 * n) L->left[2 * n - s] = (int16_t)v;
        else if (s == 2 * n) {
            L->left[0] = (int16_t)v;
            L->top[0] = (int16_t)v;
        } else if (s < ns) {
            L->top[s - 2 * n] = (int16_t)v;
        }
    }
#endif
    wave_sync();
    // 3. filtering (8.4.4.2.3), luma only for 4:2:0
    const int16_t *lf = L->left, *tp = L->top;
    if (cidx == 0 && mode != 1 && n != 4) {
        const int dist = min(abs(mode - 26), abs(mode - 10));
        const int thr = n == 8 ? 7 : (n == 16 ? 1 : 0);
        if (dist > thr) {
            const int c = L->left[0];
            const bool bi = strong && n == 32 && abs(c + L->top[64] - 2 * L->top[32]) < (1 << (bd - 5)) &&
                            abs(c + L->left[64] - 2 * L->left[32]) < (1 << (bd - 5));
            for (int i = lane; i <= 2 * n; i += kWave) {
                int a, b;
                if (bi) {
                    if (i == 0) a = b = c;
                    else if (i == 64) {
                        a = L->left[64];
                        b = L->top[64];
                    } else {
                        a = ((64 - i) * c + i * L->left[64] + 32) >> 6;
                        b = ((64 - i) * c + i * L->top[64] + 32) >> 6;
                    }
                } else if (i == 0) {
                    a = b = (L->left[1] + 2 * c + L->top[1] + 2) >> 2;
                } else if (i == 2 * n) {
                    a = L->left[i];
                    b = L->top[i];
                } else {
                    a = (L->left[i + 1] + 2 * L->left[i] + L->left[i - 1] + 2) >> 2;
                    b = (L->top[i + 1] + 2 * L->top[i] + L->top[i - 1] + 2) >> 2;
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
    if (mode == 1) {  // DC: wave reduction of the 2n references
        int sum = 0;
        for (int i = lane; i < 2 * n; i += kWave) sum += i < n ? tp[1 + i] : lf[1 + i - n];
#if !defined(HG_HOST_EMU)
        for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
#endif
        L->dc = (sum + n) >> (log2n + 1);
        wave_sync();
    } else if (mode >= 2) {
        const int ang = c_angle[mode];
        int16_t *ref = L->ref + 64;
        const int16_t *main_ = mode >= 18 ? tp : lf;
        const int16_t *side = mode >= 18 ? lf : tp;
        for (int i = lane; i <= 2 * n; i += kWave) {
            if (i <= n || ang >= 0) ref[i] = main_[i];
        }
        if (ang < 0) {
            const int lo = (n * ang) >> 5;
            if (lo < -1) {
                const int inv = c_inv_angle[mode];
                for (int xx = lo + lane; xx <= -1; xx += kWave) ref[xx] = side[(xx * inv + 128) >> 8];
            }
        }
        wave_sync();
    }
    const int dc = mode == 1 ? L->dc : 0;
    for (int o = lane; o < n * n; o += kWave) {
        const int x = o & (n - 1), y = o >> log2n;
        int pv;
        if (mode == 0) {
            pv = ((n - 1 - x) * lf[1 + y] + (x + 1) * tp[1 + n] + (n - 1 - y) * tp[1 + x] + (y + 1) * lf[1 + n] + n) >>
                 (log2n + 1);
        } else if (mode == 1) {
            pv = dc;
            if (cidx == 0 && n < 32) {
                if (x == 0 && y == 0) pv = (lf[1] + 2 * dc + tp[1] + 2) >> 2;
                else if (y == 0) pv = (tp[1 + x] + 3 * dc + 2) >> 2;
                else if (x == 0) pv = (lf[1 + y] + 3 * dc + 2) >> 2;
            }
        } else {
            const int ang = c_angle[mode];
            const int16_t *ref = L->ref + 64;
            const int a = mode >= 18 ? x : y, b = mode >= 18 ? y : x;  // a along the main direction
            const int idx = ((b + 1) * ang) >> 5, fact = ((b + 1) * ang) & 31;
            pv = fact ? ((32 - fact) * ref[a + idx + 1] + fact * ref[a + idx + 2] + 16) >> 5 : ref[a + idx + 1];
            if (cidx == 0 && n < 32) {
                if (mode == 26 && x == 0) pv = min(max(tp[1] + ((lf[1 + y] - lf[0]) >> 1), 0), maxv);
                if (mode == 10 && y == 0) pv = min(max(lf[1] + ((tp[1 + x] - tp[0]) >> 1), 0), maxv);
            }
        }
        if (tu.flags & TU_CBF) pv += res[(size_t)(y0 + y) * res_pitch + x0 + x];
        pv = min(max(pv, 0), maxv);
        plane[(size_t)(y0 + y) * pitch + x0 + x] = (Pel)pv;
    }
    wave_sync();
}

}  // namespace

template <typename Pel>
__global__ void __launch_bounds__(kWaves * 64) k_intra(BatchArgs a) {
    HG_BLOCK_SHARED IntraLds lds[kWaves];
    HG_BLOCK_SHARED uint32_t progress[kWaves];
    const int pic = blockIdx.x;
    const int wave = (int)HG_UNI(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const PicDesc pd = a.pics[pic];
    const SeqParams sp = a.seqs[pd.seq];
    const int W = sp.width, H = sp.height, log2ctb = sp.log2_ctb;
    const int wctb = (W + (1 << log2ctb) - 1) >> log2ctb, hctb = (H + (1 << log2ctb) - 1) >> log2ctb;
    const int cw = sp.chroma_format ? W >> 1 : 0, ch = sp.chroma_format ? H >> 1 : 0;
    Pel *planes[3];
    planes[0] = reinterpret_cast<Pel *>(a.recon + pd.recon_off);
    planes[1] = planes[0] + (size_t)W * H;
    planes[2] = planes[1] + (size_t)cw * ch;
    const int16_t *res[3] = {a.resid + pd.resid_off, a.resid + pd.resid_off + (size_t)W * H,
                             a.resid + pd.resid_off + (size_t)W * H + (size_t)cw * ch};
    const bool strong = (sp.flags & SP_STRONG_INTRA) != 0;
    if (lane == 0) progress[wave] = 0;
    __syncthreads();
    const uint32_t stride = (uint32_t)wctb + 1;
    const int prev_wave = (wave + kWaves - 1) % kWaves;
    IntraLds *L = &lds[wave];
    for (int r = wave; r < hctb; r += kWaves) {
        const uint32_t ntu = a.row_counts[2 * (pd.row_off + r)];
        const TuRec *tus = a.tus + pd.tu_off + (uint64_t)r * pd.tu_cap_row;
        int cur = -1;
        for (uint32_t t = 0; t < ntu; ++t) {
            const TuRec tu = tus[t];
            const int c = (int)HG_UNI((uint32_t)tu.ctu);
            if (c != cur) {
                if (cur >= 0) {
                    HG_FENCE_REL();
                    if (lane == 0) hg_atomic_store(&progress[wave], (uint32_t)r * stride + (uint32_t)c);
                }
                cur = c;
                if (r > 0) {
                    const uint32_t need = (uint32_t)(r - 1) * stride + (uint32_t)min(c + 2, wctb);
                    for (uint32_t spin = 0; (uint32_t)HG_UNI(hg_atomic_load(&progress[prev_wave])) < need; ++spin) {
                        if (spin > (1u << 24)) {  // bounded: never hang the device
                            if (lane == 0) atomicOr(&a.status[pic], ST_SUBSTREAM_END);
                            break;
                        }
                        HG_SLEEP();
                    }
                    HG_FENCE_ACQ();
                }
            }
            const int cidx = tu.flags & TU_CIDX_MASK;
            const int PW = cidx ? cw : W, PH = cidx ? ch : H;
            if (tu.log2 < 2 || tu.log2 > 5 || cidx > 2 || tu.x + (1 << tu.log2) > PW || tu.y + (1 << tu.log2) > PH)
                continue;
            predict_tb<Pel>(L, tu, planes[cidx], PW, PW, PH, cidx, res[cidx], PW,
                            cidx ? sp.bit_depth_c : sp.bit_depth_y, strong, log2ctb, sp.log2_min_tb, wctb, lane);
        }
        HG_FENCE_REL();
        if (lane == 0) hg_atomic_store(&progress[wave], (uint32_t)r * stride + (uint32_t)wctb);
    }
}

#if defined(HG_HOST_EMU)
void emu_intra(const BatchArgs &a) {
    if (a.bytes_per_sample == 1) emu_launch(k_intra<uint8_t>, a.n_pics, 1, kWaves, a);
    else emu_launch(k_intra<uint16_t>, a.n_pics, 1, kWaves, a);
}
#else
hipError_t launch_intra(const BatchArgs &a, hipStream_t s) {
    if (a.bytes_per_sample == 1)
        hipLaunchKernelGGL(k_intra<uint8_t>, dim3(a.n_pics), dim3(kWaves * 64), 0, s, a);
    else
        hipLaunchKernelGGL(k_intra<uint16_t>, dim3(a.n_pics), dim3(kWaves * 64), 0, s, a);
    return hipGetLastError();
}
#endif

}  // namespace hg
