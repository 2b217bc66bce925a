// loopfilter.hip — deblocking (stage 4) and SAO + output placement (stage 5).
//
// Deblocking, H.265 8.7.2: transform/prediction edges on the 8x8 grid, bS = 2
// for intra, beta'/tC' tables 8-12, luma strong/normal decisions (dE, dEp,
// dEq), chroma filtered only for bS = 2 on the 8x8 chroma grid with
// QpC = table 8-10((QpQ + QpP + 1) >> 1 + cQpPicOffset); samples of
// cu_transquant_bypass CUs are left untouched.  All vertical edges of a
// picture are filtered before any horizontal edge, and the edges of one
// direction never share a modified sample, so each direction is one launch
// with one thread per 4-line edge segment (in place).
//
// SAO, H.265 8.7.3: band offset / edge offset per CTB on the deblocked
// picture, EO neighbours outside the picture leave the sample unchanged.
// The same pass crops the conformance window and writes the picture into
// its grid position of the caller's output planes (coalesced along rows),
// clipping to the grid's output size (ISO/IEC 23008-12 ImageGrid).  No
// reference code exists for either stage (src/hevc/slice.rs:249-255).
#include "kernels.hpp"

#include <algorithm>
#include <string>

namespace hg {

namespace {

__constant__ uint8_t c_beta[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  6,  7,
                                   8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32,
                                   34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};
__constant__ uint8_t c_tc[54] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};

__device__ __forceinline__ int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ int chroma_qp_map(int qpi, int chroma) {
    if (chroma != 1) return qpi < 51 ? qpi : 51;
    if (qpi < 30) return qpi;
    if (qpi > 43) return qpi - 6;
    constexpr int t[14] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37};
    return t[qpi - 30];
}

// one 4-line luma edge segment; q0 at `q`, step across the edge `sx`, along it `sk`
template <typename Pel>
__device__ void luma_segment(Pel *q, int sx, int sk, int qpP, int qpQ, bool nofp, bool nofq, int beta_off,
                             int tc_off, int bd) {
#define PS(i, k) q[(k) * sk - ((i) + 1) * sx]
#define QS(i, k) q[(k) * sk + (i) * sx]
    const int qpl = (qpQ + qpP + 1) >> 1;
    const int beta = c_beta[clip3(0, 51, qpl + (beta_off << 1))] * (1 << (bd - 8));
    const int tc = c_tc[clip3(0, 53, qpl + 2 + (tc_off << 1))] * (1 << (bd - 8));
    const int dp0 = abs(PS(2, 0) - 2 * PS(1, 0) + PS(0, 0)), dp3 = abs(PS(2, 3) - 2 * PS(1, 3) + PS(0, 3));
    const int dq0 = abs(QS(2, 0) - 2 * QS(1, 0) + QS(0, 0)), dq3 = abs(QS(2, 3) - 2 * QS(1, 3) + QS(0, 3));
    const int dpq0 = dp0 + dq0, dpq3 = dp3 + dq3, dp = dp0 + dp3, dq = dq0 + dq3;
    if (dpq0 + dpq3 >= beta) return;
    auto dsam = [&](int k, int dpq) {
        return dpq < (beta >> 2) && abs(PS(3, k) - PS(0, k)) + abs(QS(0, k) - QS(3, k)) < (beta >> 3) &&
               abs(PS(0, k) - QS(0, k)) < ((5 * tc + 1) >> 1);
    };
    const bool strong = dsam(0, 2 * dpq0) && dsam(3, 2 * dpq3);
    const bool dEp = dp < ((beta + (beta >> 1)) >> 3), dEq = dq < ((beta + (beta >> 1)) >> 3);
    const int maxv = (1 << bd) - 1;
    for (int k = 0; k < 4; ++k) {
        const int p0 = PS(0, k), p1 = PS(1, k), p2 = PS(2, k), p3 = PS(3, k);
        const int q0 = QS(0, k), q1 = QS(1, k), q2 = QS(2, k), q3 = QS(3, k);
        if (strong) {
            if (!nofp) {
                PS(0, k) = (Pel)clip3(p0 - 2 * tc, p0 + 2 * tc, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
                PS(1, k) = (Pel)clip3(p1 - 2 * tc, p1 + 2 * tc, (p2 + p1 + p0 + q0 + 2) >> 2);
                PS(2, k) = (Pel)clip3(p2 - 2 * tc, p2 + 2 * tc, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
            }
            if (!nofq) {
                QS(0, k) = (Pel)clip3(q0 - 2 * tc, q0 + 2 * tc, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
                QS(1, k) = (Pel)clip3(q1 - 2 * tc, q1 + 2 * tc, (p0 + q0 + q1 + q2 + 2) >> 2);
                QS(2, k) = (Pel)clip3(q2 - 2 * tc, q2 + 2 * tc, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3);
            }
        } else {
            int delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
            if (abs(delta) < tc * 10) {
                delta = clip3(-tc, tc, delta);
                if (!nofp) PS(0, k) = (Pel)clip3(0, maxv, p0 + delta);
                if (!nofq) QS(0, k) = (Pel)clip3(0, maxv, q0 - delta);
                if (dEp && !nofp)
                    PS(1, k) = (Pel)clip3(0, maxv, p1 + clip3(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + delta) >> 1));
                if (dEq && !nofq)
                    QS(1, k) = (Pel)clip3(0, maxv, q1 + clip3(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - delta) >> 1));
            }
        }
    }
#undef PS
#undef QS
}

}  // namespace

// Assembly pictures (PD_ASSEMBLY, see desc.hpp): each child's samples, QpY /
// edge-flag maps and SAO parameters copied to its position in the assembly
// (a child whose slice has SAO off wrote no parameters: zero them).  Runs
// before deblocking; one workgroup row per picture, the others leave at once.
template <typename Pel>
__global__ void __launch_bounds__(256) k_assemble(BatchArgs a) {
    const int pic = a.pic0 + blockIdx.y;
    const PicDesc pd = a.pics[pic];
    if (!(pd.flags & PD_ASSEMBLY)) return;
    const SeqParams sp = a.seqs[pd.seq];
    const int W = sp.width, H = sp.height, w4 = (W + 3) >> 2, h4 = (H + 3) >> 2;
    const int wctb = (W + (1 << sp.log2_ctb) - 1) >> sp.log2_ctb;
    const int sx = chroma_sx(sp.chroma_format), sy = chroma_sy(sp.chroma_format);
    const int cw = sp.chroma_format ? W >> sx : 0, ch = sp.chroma_format ? H >> sy : 0;
    Pel *dY = reinterpret_cast<Pel *>(a.recon + pd.recon_off);
    uint8_t *dmap = a.maps + pd.map_off;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
    for (uint32_t c = 0; c < pd.nchild; ++c) {
        const PicDesc cd = a.pics[pd.child0 + c];
        const SeqParams cs = a.seqs[cd.seq];
        const int cW = cs.width, cH = cs.height, cw4 = (cW + 3) >> 2, ch4 = (cH + 3) >> 2;
        const int ccw = cs.chroma_format ? cW >> sx : 0, cch = cs.chroma_format ? cH >> sy : 0;
        const Pel *sY = reinterpret_cast<const Pel *>(a.recon + cd.recon_off);
        // samples: Y then Cb, Cr (origins are CTB-aligned, so chroma at org >> sx, sy)
        const int nl = cW * cH, nc = ccw * cch;
        for (int t = tid; t < nl + 2 * nc; t += nth) {
            if (t < nl) {
                const int x = t % cW, y = t / cW;
                dY[(size_t)(cd.org_y + y) * W + cd.org_x + x] = sY[t];
            } else {
                const int u = t - nl, k = u / nc, v = u % nc, x = v % ccw, y = v / ccw;
                dY[(size_t)W * H + (size_t)k * cw * ch + (size_t)((cd.org_y >> sy) + y) * cw + (cd.org_x >> sx) + x] = sY[t];
            }
        }
        // QpY and edge flags (4x4 units), then SAO parameters (CTBs)
        const uint8_t *smap = a.maps + cd.map_off;
        const int nm = cw4 * ch4;
        for (int t = tid; t < 2 * nm; t += nth) {
            const int k = t / nm, v = t % nm, x = v % cw4, y = v / cw4;
            dmap[(size_t)k * w4 * h4 + (size_t)((cd.org_y >> 2) + y) * w4 + (cd.org_x >> 2) + x] = smap[t];
        }
        const int cwctb = (cW + (1 << cs.log2_ctb) - 1) >> cs.log2_ctb;
        const int chctb = (cH + (1 << cs.log2_ctb) - 1) >> cs.log2_ctb;
        const bool sao = cd.sao_luma || cd.sao_chroma;
        for (int t = tid; t < cwctb * chctb * 8; t += nth) {
            const int b = t >> 3, x = b % cwctb, y = b / cwctb;
            uint32_t *dst = reinterpret_cast<uint32_t *>(
                a.sao + pd.sao_off + (size_t)((cd.org_y >> sp.log2_ctb) + y) * wctb + (cd.org_x >> sp.log2_ctb) + x);
            dst[t & 7] = sao ? reinterpret_cast<const uint32_t *>(a.sao + cd.sao_off + b)[t & 7] : 0u;
        }
    }
    (void)h4;
}

// VERT: edges between columns (x-1 | x); otherwise between rows.
template <typename Pel, bool VERT>
__global__ void __launch_bounds__(256) k_deblock(BatchArgs a) {
    const int pic = a.pic0 + blockIdx.y;
    const PicDesc pd = a.pics[pic];
    if (pd.dbk_disabled || (pd.flags & PD_CHILD)) return;  // a child is filtered as part of its assembly
    const SeqParams sp = a.seqs[pd.seq];
    const int W = sp.width, H = sp.height;
    const int w4 = (W + 3) >> 2, h4 = (H + 3) >> 2;
    const int8_t *qpy = reinterpret_cast<const int8_t *>(a.maps + pd.map_off);
    const uint8_t *flg = a.maps + pd.map_off + (size_t)w4 * h4;
    Pel *Y = reinterpret_cast<Pel *>(a.recon + pd.recon_off);
    const int sx = chroma_sx(sp.chroma_format), sy = chroma_sy(sp.chroma_format);
    const int cw = sp.chroma_format ? W >> sx : 0, ch = sp.chroma_format ? H >> sy : 0;
    // luma segments
    const int ne_l = VERT ? (W - 1) >> 3 : (H - 1) >> 3;  // edges excluding the picture boundary
    const int ns_l = VERT ? H >> 2 : W >> 2;               // 4-sample segments along each edge
    const int nl = ne_l * ns_l;
    // chroma: edges on the 8x8 chroma-sample grid, segments of the lines one
    // 4-line luma segment covers (bS, QpY and flags come from that segment)
    const int ne_c = VERT ? (cw - 1) >> 3 : (ch - 1) >> 3;
    const int lc = VERT ? 4 >> sy : 4 >> sx;
    const int ns_c = VERT ? ch / lc : cw / lc;
    const int nc = sp.chroma_format ? ne_c * ns_c : 0;
    const int total = nl + 2 * nc;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        if (t < nl) {
            int x, y;
            if (VERT) {
                x = 8 * (t % ne_l + 1);
                y = 4 * (t / ne_l);
            } else {
                x = 4 * (t % ns_l);
                y = 8 * (t / ns_l + 1);
            }
            const int fq = flg[(y >> 2) * w4 + (x >> 2)];
            if (!(fq & (VERT ? MF_EDGE_V : MF_EDGE_H))) continue;
            const int xp = VERT ? x - 1 : x, yp = VERT ? y : y - 1;
            const int fp = flg[(yp >> 2) * w4 + (xp >> 2)];
            luma_segment<Pel>(Y + (size_t)y * W + x, VERT ? 1 : W, VERT ? W : 1, qpy[(yp >> 2) * w4 + (xp >> 2)],
                              qpy[(y >> 2) * w4 + (x >> 2)], fp & MF_NOFILT, fq & MF_NOFILT, pd.beta_off, pd.tc_off,
                              sp.bit_depth_y);
        } else {
            const int u = t - nl;
            const int cidx = 1 + u / nc, v = u % nc;
            int xc, yc;
            if (VERT) {
                xc = 8 * (v % ne_c + 1);
                yc = lc * (v / ne_c);
            } else {
                xc = lc * (v % ns_c);
                yc = 8 * (v / ns_c + 1);
            }
            const int xl = xc << sx, yl = yc << sy;
            const int fq = flg[(yl >> 2) * w4 + (xl >> 2)];
            if (!(fq & (VERT ? MF_EDGE_V : MF_EDGE_H))) continue;
            const int xlp = VERT ? xl - 1 : xl, ylp = VERT ? yl : yl - 1;
            const int fp = flg[(ylp >> 2) * w4 + (xlp >> 2)];
            const int qpP = qpy[(ylp >> 2) * w4 + (xlp >> 2)], qpQ = qpy[(yl >> 2) * w4 + (xl >> 2)];
            const int off = cidx == 1 ? sp.cb_qp_offset : sp.cr_qp_offset;
            const int qpc = chroma_qp_map(((qpQ + qpP + 1) >> 1) + off, sp.chroma_format);
            const int bd = sp.bit_depth_c;
            const int tc = c_tc[clip3(0, 53, qpc + 2 + (pd.tc_off << 1))] * (1 << (bd - 8));
            const int maxv = (1 << bd) - 1;
            Pel *C = Y + (size_t)W * H + (size_t)(cidx - 1) * cw * ch;
            Pel *q = C + (size_t)yc * cw + xc;
            const int sa = VERT ? 1 : cw, sk = VERT ? cw : 1;  // across / along the edge
            for (int k = 0; k < lc; ++k) {
                const int p0 = q[k * sk - sa], p1 = q[k * sk - 2 * sa], q0 = q[k * sk], q1 = q[k * sk + sa];
                const int delta = clip3(-tc, tc, ((((q0 - p0) * 4) + p1 - q1 + 4) >> 3));
                if (!(fp & MF_NOFILT)) q[k * sk - sa] = (Pel)clip3(0, maxv, p0 + delta);
                if (!(fq & MF_NOFILT)) q[k * sk] = (Pel)clip3(0, maxv, q0 - delta);
            }
        }
    }
}

// SAO (8.7.3) of one sample at picture position (xs, ys) of component cidx
template <typename Pel>
__device__ __forceinline__ int sao_sample(const Pel *P, int PW, int PH, int xs, int ys, int cidx, int subx,
                                          int suby, const SaoParams *sao, int wctb, int log2ctb, const uint8_t *flg,
                                          int w4, int bd) {
    int v = P[(size_t)ys * PW + xs];
    const SaoParams &s = sao[(ys >> (log2ctb - suby)) * wctb + (xs >> (log2ctb - subx))];
    const int type = s.type[cidx];
    if (!type || (flg[((ys << suby) >> 2) * w4 + ((xs << subx) >> 2)] & MF_NOFILT)) return v;
    int o = 0;
    if (type == 2) {
        const int cl = s.band_eo[cidx];
        const int hx = cl == 0 ? 1 : (cl == 1 ? 0 : (cl == 2 ? 1 : -1));
        const int vy = cl == 0 ? 0 : 1;
        const int ax = xs - hx, ay = ys - vy, bx = xs + hx, by = ys + vy;
        if (ax >= 0 && ay >= 0 && ax < PW && ay < PH && bx >= 0 && by >= 0 && bx < PW && by < PH) {
            const int na = P[(size_t)ay * PW + ax], nb = P[(size_t)by * PW + bx];
            int e = 2 + (v > na) - (v < na) + (v > nb) - (v < nb);
            if (e <= 2) e = e == 2 ? 0 : e + 1;
            o = e ? s.off[cidx][e - 1] : 0;
        }
    } else {
        const int band = v >> (bd - 5);
        const int k = (band - s.band_eo[cidx]) & 31;
        o = k < 4 ? s.off[cidx][k] : 0;
    }
    return clip3(0, (1 << bd) - 1, v + o);
}

// SAO + crop + grid placement: one thread per four consecutive output samples
// of a row (one 4- or 8-byte store; per sample at a row's ragged end or an
// unaligned caller plane)
template <typename Pel>
__global__ void __launch_bounds__(256) k_sao_out(BatchArgs a) {
    const int pic = a.pic0 + blockIdx.y;
    const PicDesc pd = a.pics[pic];
    if (pd.flags & PD_CHILD) return;  // output through its assembly
    const SeqParams sp = a.seqs[pd.seq];
    const OutImage oi = a.outs[pd.image];
    const int W = sp.width, H = sp.height, log2ctb = sp.log2_ctb;
    const int wctb = (W + (1 << log2ctb) - 1) >> log2ctb;
    const int w4 = (W + 3) >> 2, h4 = (H + 3) >> 2;
    const uint8_t *flg = a.maps + pd.map_off + (size_t)w4 * h4;
    const Pel *Y = reinterpret_cast<const Pel *>(a.recon + pd.recon_off);
    const int sx = chroma_sx(sp.chroma_format), sy = chroma_sy(sp.chroma_format);
    const int cw = sp.chroma_format ? W >> sx : 0, ch = sp.chroma_format ? H >> sy : 0;
    const SaoParams *sao = a.sao + pd.sao_off;
    // visible region of this picture in the output image (luma)
    const int vw = min(sp.out_w, oi.width - pd.out_x), vh = min(sp.out_h, oi.height - pd.out_y);
    if (vw <= 0 || vh <= 0) return;
    const int vcw = sp.chroma_format ? (vw + (1 << sx) - 1) >> sx : 0;
    const int vch = sp.chroma_format ? (vh + (1 << sy) - 1) >> sy : 0;
    const int qw = (vw + 3) >> 2, qcw = (vcw + 3) >> 2;  // quads per row
    const int nl = qw * vh, nc = qcw * vch;
    const int total = nl + 2 * nc;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        int cidx, q, y;
        if (t < nl) {
            cidx = 0;
            q = t % qw;
            y = t / qw;
        } else {
            const int u = t - nl;
            cidx = 1 + u / nc;
            q = (u % nc) % qcw;
            y = (u % nc) / qcw;
        }
        const int subx = cidx ? sx : 0, suby = cidx ? sy : 0;
        const int PW = cidx ? cw : W, PH = cidx ? ch : H;
        const int vwc = cidx ? vcw : vw;
        const Pel *P = cidx == 0 ? Y : Y + (size_t)W * H + (size_t)(cidx - 1) * cw * ch;
        const int x0 = q * 4, n = min(4, vwc - x0);
        const int ys = y + (sp.conf_t >> suby), xs0 = x0 + (sp.conf_l >> subx);  // picture coords
        const bool on = pd.sao_luma || pd.sao_chroma;  // SaoTypeIdx is 0 for a component whose flag is off
        const int bd = cidx ? sp.bit_depth_c : sp.bit_depth_y;
        int v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v[j] = 0;
            if (j < n)
                v[j] = on ? sao_sample(P, PW, PH, xs0 + j, ys, cidx, subx, suby, sao, wctb, log2ctb, flg, w4, bd)
                          : (int)P[(size_t)ys * PW + xs0 + j];
        }
        // component fields by select: a lane-varying index into the OutImage copy made
        // the compiler keep it in LDS (12 KB per workgroup, 519 M bank-conflict cycles per launch)
        const uint64_t plane = cidx == 0 ? oi.plane[0] : (cidx == 1 ? oi.plane[1] : oi.plane[2]);
        const int pitch = cidx == 0 ? oi.pitch[0] : (cidx == 1 ? oi.pitch[1] : oi.pitch[2]);
        const int ox = (pd.out_x >> subx) + x0, oy = (pd.out_y >> suby) + y;
        Pel *dst = reinterpret_cast<Pel *>(plane + (size_t)oy * pitch) + ox;
        if (n == 4 && (reinterpret_cast<uintptr_t>(dst) & (4 * sizeof(Pel) - 1)) == 0) {
            if (sizeof(Pel) == 1)
                *reinterpret_cast<uint32_t *>(dst) = (uint32_t)v[0] | (uint32_t)v[1] << 8 | (uint32_t)v[2] << 16 |
                                                     (uint32_t)v[3] << 24;
            else
                *reinterpret_cast<uint64_t *>(dst) = (uint64_t)v[0] | (uint64_t)v[1] << 16 | (uint64_t)v[2] << 32 |
                                                     (uint64_t)v[3] << 48;
        } else {
            for (int j = 0; j < n; ++j) dst[j] = (Pel)v[j];
        }
    }
}

// ---------------------------------------------------------------- fused
// k_loopfilter: deblocking (both directions), SAO, crop and grid placement of
// one 64x64 luma tile (and its chroma tiles) per workgroup, in LDS.  The tile
// and a halo (luma 8, chroma 4 samples) are loaded once; the vertical edges
// of every halo row are filtered, then the horizontal edges of every halo
// column, then SAO reads the 3x3 neighbourhoods and the visible samples go to
// the caller's planes.  Why the halo suffices: an edge modifies at most 3
// samples on each side and reads 4 (luma; chroma 1 and 2), edges of one
// direction never share a modified sample, and SAO reads one sample around
// each output sample, so the final deblocked values of the tile plus a
// one-sample ring depend only on edges inside the tile's range and on
// unfiltered samples at most 4 outside it.  Replaces k_deblock<V>,
// k_deblock<H> and k_sao_out (three passes over the picture in HBM) with one
// read of the reconstruction and one write of the output.
constexpr int kLfT = 64, kLfHaloY = 8, kLfHaloC = 4, kLfWaves = 4;

struct LfDims {
    int ly_w, ly_h, lc_w, lc_h;  // LDS region sizes (samples)
};
__host__ __device__ inline LfDims lf_dims(int chroma_format) {
    const int sx = chroma_sx(chroma_format), sy = chroma_sy(chroma_format);
    LfDims d;
    d.ly_w = d.ly_h = kLfT + 2 * kLfHaloY;
    d.lc_w = chroma_format ? (kLfT >> sx) + 2 * kLfHaloC : 0;
    d.lc_h = chroma_format ? (kLfT >> sy) + 2 * kLfHaloC : 0;
    return d;
}
inline size_t lf_lds_bytes(int bytes_per_sample, int chroma_format) {
    const LfDims d = lf_dims(chroma_format);
    return (size_t)bytes_per_sample * ((size_t)d.ly_w * d.ly_h + 2 * (size_t)d.lc_w * d.lc_h);
}

// f(t) for t in [0, n) over the workgroup's kLfWaves waves (host emulation:
// one thread per wave walks its wave's 64 lanes)
template <class F>
__device__ __forceinline__ void lf_for(int n, F f) {
    const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    for (int b = wave * 64; b < n; b += 64 * kLfWaves)
        for (int l = lane; l < 64 && b + l < n; l += kWave) f(b + l);
}

template <typename Pel>
__global__ void __launch_bounds__(kLfWaves * 64) k_loopfilter(BatchArgs a) {
#if defined(HG_HOST_EMU)
    unsigned char *smem = g_emu.smem;
#else
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
#endif
    const int pic = a.pic0 + blockIdx.y;
    const PicDesc pd = a.pics[pic];
    if (pd.flags & PD_CHILD) return;  // filtered and output through its assembly
    const SeqParams sp = a.seqs[pd.seq];
    const int W = sp.width, H = sp.height, log2ctb = sp.log2_ctb;
    const int tiles_x = (W + kLfT - 1) / kLfT;
    const int x0 = (int)(blockIdx.x % (unsigned)tiles_x) * kLfT, y0 = (int)(blockIdx.x / (unsigned)tiles_x) * kLfT;
    if (y0 >= H) return;
    const OutImage oi = a.outs[pd.image];
    // visible region of this picture in the output image (luma, window coordinates)
    const int vw = min(sp.out_w, oi.width - pd.out_x), vh = min(sp.out_h, oi.height - pd.out_y);
    if (vw <= 0 || vh <= 0) return;
    if (x0 >= sp.conf_l + vw || x0 + kLfT <= sp.conf_l || y0 >= sp.conf_t + vh || y0 + kLfT <= sp.conf_t) return;
    const int cf = sp.chroma_format, sx = chroma_sx(cf), sy = chroma_sy(cf);
    const int cw = cf ? W >> sx : 0, ch = cf ? H >> sy : 0;
    const int w4 = (W + 3) >> 2, h4 = (H + 3) >> 2;
    const int wctb = (W + (1 << log2ctb) - 1) >> log2ctb;
    const int8_t *qpy = reinterpret_cast<const int8_t *>(a.maps + pd.map_off);
    const uint8_t *flg = a.maps + pd.map_off + (size_t)w4 * h4;
    const Pel *gY = reinterpret_cast<const Pel *>(a.recon + pd.recon_off);
    const LfDims d = lf_dims(cf);
    Pel *sY = reinterpret_cast<Pel *>(smem);
    Pel *sC[2] = {sY + d.ly_w * d.ly_h, sY + d.ly_w * d.ly_h + d.lc_w * d.lc_h};
    const int ry0 = y0 - kLfHaloY, rx0 = x0 - kLfHaloY;
    const int cx0 = x0 >> sx, cy0 = y0 >> sy, ctw = kLfT >> sx, cth = kLfT >> sy;
    const int cry0 = cy0 - kLfHaloC, crx0 = cx0 - kLfHaloC;
    const int ncomp = cf ? 3 : 1;

    // 1. the region, in dwords (region origins and plane widths are multiples
    //    of 4 samples, so no dword straddles a plane's edge); samples outside
    //    the picture are never read as filter or SAO inputs
    {
        constexpr int per = 4 / (int)sizeof(Pel);  // samples per dword
        const int ny = d.ly_h * (d.ly_w / per), nc = d.lc_h * (d.lc_w / per);
        lf_for(ny + 2 * nc, [&](int t) {
            int comp = 0, u = t;
            if (u >= ny) {
                u -= ny;
                comp = 1 + u / nc;
                u %= nc;
            }
            const int rw = comp ? d.lc_w : d.ly_w, PW = comp ? cw : W, PH = comp ? ch : H;
            const int r = u / (rw / per), xq = (u % (rw / per)) * per;
            const int gy = (comp ? cry0 : ry0) + r, gx = (comp ? crx0 : rx0) + xq;
            if (gy < 0 || gy >= PH || gx < 0 || gx >= PW) return;
            const Pel *src = comp ? gY + (size_t)W * H + (size_t)(comp - 1) * cw * ch : gY;
            Pel *dst = comp ? sC[comp - 1] : sY;
            *reinterpret_cast<uint32_t *>(dst + r * rw + xq) =
                *reinterpret_cast<const uint32_t *>(src + (size_t)gy * PW + gx);
        });
    }
    __syncthreads();

    // 2-3. deblocking: vertical edges on every halo row, then horizontal edges on every halo column
    if (!pd.dbk_disabled) {
        const int ne_y = kLfT / 8 + 1, ns_y = (kLfT + 8) / 4;  // edges x0 .. x0+64, segments y0-4 .. y0+68
        const int ne_cx = ctw / 8 + 1, ne_cy = cth / 8 + 1;
        for (int dir = 0; dir < 2; ++dir) {
            const bool vert = dir == 0;
            const int lc = vert ? 4 >> sy : 4 >> sx;                       // chroma lines per segment
            const int ne_c = vert ? ne_cx : ne_cy;
            const int ns_c = cf ? ((vert ? cth : ctw) + 2 * kLfHaloC) / lc : 0;
            const int nl = ne_y * ns_y, nc = cf ? ne_c * ns_c : 0;
            lf_for(nl + 2 * nc, [&](int t) {
                if (t < nl) {
                    const int e = t % ne_y, sgm = t / ne_y;
                    const int x = vert ? x0 + 8 * e : x0 - 4 + 4 * sgm, y = vert ? y0 - 4 + 4 * sgm : y0 + 8 * e;
                    if (vert ? (x <= 0 || x >= W || y < 0 || y >= H) : (y <= 0 || y >= H || x < 0 || x >= W)) return;
                    const int fq = flg[(y >> 2) * w4 + (x >> 2)];
                    if (!(fq & (vert ? MF_EDGE_V : MF_EDGE_H))) return;
                    const int xp = vert ? x - 1 : x, yp = vert ? y : y - 1;
                    const int fp = flg[(yp >> 2) * w4 + (xp >> 2)];
                    luma_segment<Pel>(sY + (y - ry0) * d.ly_w + (x - rx0), vert ? 1 : d.ly_w, vert ? d.ly_w : 1,
                                      qpy[(yp >> 2) * w4 + (xp >> 2)], qpy[(y >> 2) * w4 + (x >> 2)], fp & MF_NOFILT,
                                      fq & MF_NOFILT, pd.beta_off, pd.tc_off, sp.bit_depth_y);
                    return;
                }
                const int u = t - nl, cidx = 1 + u / nc, v = u % nc;
                const int e = v % ne_c, sgm = v / ne_c;
                const int xc = vert ? cx0 + 8 * e : crx0 + lc * sgm, yc = vert ? cry0 + lc * sgm : cy0 + 8 * e;
                if (vert ? (xc <= 0 || xc >= cw || yc < 0 || yc >= ch) : (yc <= 0 || yc >= ch || xc < 0 || xc >= cw))
                    return;
                const int xl = xc << sx, yl = yc << sy;
                const int fq = flg[(yl >> 2) * w4 + (xl >> 2)];
                if (!(fq & (vert ? MF_EDGE_V : MF_EDGE_H))) return;
                const int xlp = vert ? xl - 1 : xl, ylp = vert ? yl : yl - 1;
                const int fp = flg[(ylp >> 2) * w4 + (xlp >> 2)];
                const int qpP = qpy[(ylp >> 2) * w4 + (xlp >> 2)], qpQ = qpy[(yl >> 2) * w4 + (xl >> 2)];
                const int off = cidx == 1 ? sp.cb_qp_offset : sp.cr_qp_offset;
                const int qpc = chroma_qp_map(((qpQ + qpP + 1) >> 1) + off, cf);
                const int bd = sp.bit_depth_c;
                const int tc = c_tc[clip3(0, 53, qpc + 2 + (pd.tc_off << 1))] * (1 << (bd - 8));
                const int maxv = (1 << bd) - 1;
                Pel *q = sC[cidx - 1] + (yc - cry0) * d.lc_w + (xc - crx0);
                const int sa = vert ? 1 : d.lc_w, sk = vert ? d.lc_w : 1;  // across / along the edge
                for (int k = 0; k < lc; ++k) {
                    const int p0 = q[k * sk - sa], p1 = q[k * sk - 2 * sa], q0 = q[k * sk], q1 = q[k * sk + sa];
                    const int delta = clip3(-tc, tc, ((((q0 - p0) * 4) + p1 - q1 + 4) >> 3));
                    if (!(fp & MF_NOFILT)) q[k * sk - sa] = (Pel)clip3(0, maxv, p0 + delta);
                    if (!(fq & MF_NOFILT)) q[k * sk] = (Pel)clip3(0, maxv, q0 - delta);
                }
            });
            __syncthreads();
        }
    }

    // 4. SAO + crop + placement of the tile's visible samples, four output
    //    samples per task (one 4- or 8-byte store when whole and aligned)
    const bool on = pd.sao_luma || pd.sao_chroma;  // SaoTypeIdx is 0 for a component whose flag is off
    const SaoParams *sao = a.sao + pd.sao_off;
    int nq[3] = {0, 0, 0}, qlo[3] = {0, 0, 0}, rlo[3] = {0, 0, 0}, nr[3] = {0, 0, 0};
    for (int c = 0; c < ncomp; ++c) {
        const int subx = c ? sx : 0, suby = c ? sy : 0;
        const int tx0 = c ? cx0 : x0, ty0 = c ? cy0 : y0, tw = c ? ctw : kLfT, th = c ? cth : kLfT;
        const int cl = sp.conf_l >> subx, ct = sp.conf_t >> suby;
        const int vwc = c ? (vw + (1 << sx) - 1) >> sx : vw, vhc = c ? (vh + (1 << sy) - 1) >> sy : vh;
        // window rows / quads whose samples lie in the tile
        const int ya = max(ty0 - ct, 0), yb = min(ty0 + th - ct, vhc);
        const int xa = max(tx0 - cl, 0), xb = min(tx0 + tw - cl, vwc);
        if (ya >= yb || xa >= xb) continue;
        rlo[c] = ya;
        nr[c] = yb - ya;
        qlo[c] = xa >> 2;
        nq[c] = ((xb + 3) >> 2) - qlo[c];
    }
    const int n0 = nr[0] * nq[0], n1 = nr[1] * nq[1], n2 = nr[2] * nq[2];
    lf_for(n0 + n1 + n2, [&](int t) {
        const int c = t < n0 ? 0 : (t < n0 + n1 ? 1 : 2);
        const int u = c == 0 ? t : (c == 1 ? t - n0 : t - n0 - n1);
        const int subx = c ? sx : 0, suby = c ? sy : 0;
        const int tx0 = c ? cx0 : x0, tw = c ? ctw : kLfT;
        const int cl = sp.conf_l >> subx, ct = sp.conf_t >> suby;
        const int vwc = c ? (vw + (1 << sx) - 1) >> sx : vw;
        const int y = rlo[c] + u / nq[c], xw = (qlo[c] + u % nq[c]) * 4;  // window coordinates
        const int ys = y + ct;
        const Pel *R = c ? sC[c - 1] : sY;
        const int RW = c ? d.lc_w : d.ly_w, rxo = c ? crx0 : rx0, ryo = c ? cry0 : ry0;
        const int PW = c ? cw : W, PH = c ? ch : H, bd = c ? sp.bit_depth_c : sp.bit_depth_y;
        int v[4];
        bool own[4];
        int n_own = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int xs = xw + j + cl;
            own[j] = xw + j < vwc && xs >= tx0 && xs < tx0 + tw;
            v[j] = 0;
            if (!own[j]) continue;
            ++n_own;
            const Pel *pp = R + (ys - ryo) * RW + (xs - rxo);
            int s = *pp;
            if (on) {
                const SaoParams &sv = sao[(ys >> (log2ctb - suby)) * wctb + (xs >> (log2ctb - subx))];
                const int type = sv.type[c];
                if (type && !(flg[((ys << suby) >> 2) * w4 + ((xs << subx) >> 2)] & MF_NOFILT)) {
                    int o = 0;
                    if (type == 2) {
                        const int cls = sv.band_eo[c];
                        const int hx = cls == 0 ? 1 : (cls == 1 ? 0 : (cls == 2 ? 1 : -1));
                        const int vy = cls == 0 ? 0 : 1;
                        const int ax = xs - hx, ay = ys - vy, bx = xs + hx, by = ys + vy;
                        if (ax >= 0 && ay >= 0 && ax < PW && ay < PH && bx >= 0 && by >= 0 && bx < PW && by < PH) {
                            const int na = pp[-vy * RW - hx], nb = pp[vy * RW + hx];
                            int e = 2 + (s > na) - (s < na) + (s > nb) - (s < nb);
                            if (e <= 2) e = e == 2 ? 0 : e + 1;
                            o = e ? sv.off[c][e - 1] : 0;
                        }
                    } else {
                        const int k = ((s >> (bd - 5)) - sv.band_eo[c]) & 31;
                        o = k < 4 ? sv.off[c][k] : 0;
                    }
                    s = clip3(0, (1 << bd) - 1, s + o);
                }
            }
            v[j] = s;
        }
        const uint64_t plane = c == 0 ? oi.plane[0] : (c == 1 ? oi.plane[1] : oi.plane[2]);
        const int pitch = c == 0 ? oi.pitch[0] : (c == 1 ? oi.pitch[1] : oi.pitch[2]);
        const int ox = (pd.out_x >> subx) + xw, oy = (pd.out_y >> suby) + y;
        Pel *dst = reinterpret_cast<Pel *>(plane + (size_t)oy * pitch) + ox;
        if (n_own == 4 && (reinterpret_cast<uintptr_t>(dst) & (4 * sizeof(Pel) - 1)) == 0) {
            if (sizeof(Pel) == 1)
                *reinterpret_cast<uint32_t *>(dst) = (uint32_t)v[0] | (uint32_t)v[1] << 8 | (uint32_t)v[2] << 16 |
                                                     (uint32_t)v[3] << 24;
            else
                *reinterpret_cast<uint64_t *>(dst) = (uint64_t)v[0] | (uint64_t)v[1] << 16 | (uint64_t)v[2] << 32 |
                                                     (uint64_t)v[3] << 48;
        } else {
            for (int j = 0; j < 4; ++j)
                if (own[j]) dst[j] = (Pel)v[j];
        }
    });
}

// The fused loop filter only with HEIFGPU_LF=fused.  r04 A/B (same box, 128
// images): alone 9.2 ms against 2.9 + 4.1 for the three split kernels, and
// beside the next decode's parse 53 ms against ~33, with k_transform (on its
// own stream) 60 ms against 29.  Its 9.6 KB of LDS per workgroup competes with
// the parse waves and k_transform for the LDS the parse leaves free, which is
// what decides the reconstruction kernels' residency in the pipeline (a parse
// padded by 4 KB of LDS per wave took 129 ms instead of 81 beside them).
// (read at every launch, so a test can switch it within one process)
inline bool lf_fused() {
    const char *e = std::getenv("HEIFGPU_LF");
    return e && std::string(e) == "fused";
}
inline int lf_tiles(const BatchArgs &a) { return a.lf_tiles; }

#if defined(HG_HOST_EMU)
void emu_deblock(const BatchArgs &a) {
    if (a.has_assembly) {
        if (a.bytes_per_sample == 1) emu_launch(k_assemble<uint8_t>, 1, a.n_pics, 1, a, true);
        else emu_launch(k_assemble<uint16_t>, 1, a.n_pics, 1, a, true);
    }
    if (lf_fused()) return;  // deblocking runs inside k_loopfilter (emu_sao_out)
    if (a.bytes_per_sample == 1) {
        emu_launch(k_deblock<uint8_t, true>, 1, a.n_pics, 1, a, true);
        emu_launch(k_deblock<uint8_t, false>, 1, a.n_pics, 1, a, true);
    } else {
        emu_launch(k_deblock<uint16_t, true>, 1, a.n_pics, 1, a, true);
        emu_launch(k_deblock<uint16_t, false>, 1, a.n_pics, 1, a, true);
    }
}
void emu_sao_out(const BatchArgs &a) {
    if (lf_fused()) {
        const size_t lds = lf_lds_bytes(a.bytes_per_sample, a.chroma_format);
        if (a.bytes_per_sample == 1) emu_launch(k_loopfilter<uint8_t>, lf_tiles(a), a.n_pics, kLfWaves, a, false, lds);
        else emu_launch(k_loopfilter<uint16_t>, lf_tiles(a), a.n_pics, kLfWaves, a, false, lds);
        return;
    }
    if (a.bytes_per_sample == 1) emu_launch(k_sao_out<uint8_t>, 1, a.n_pics, 1, a, true);
    else emu_launch(k_sao_out<uint16_t>, 1, a.n_pics, 1, a, true);
}
#else
// Workgroups per picture of the grid-stride loop filter kernels: about
// `total` workgroups for the batch, within [lo, hi] per picture.  A full batch
// (128 images) gets few long-lived workgroups per picture: beside the next
// decode's parse, 2 / 4 instead of 64 / 256 took deblocking 21 -> 7.7 ms and
// the step 85.9 -> 85.6 ms (r04 A/B); small batches keep many, for latency.
// HEIFGPU_DBK_BLOCKS / HEIFGPU_SAO_BLOCKS force a count.
static int lf_blocks(const char *var, int n_pics, int total, int lo, int hi) {
    const char *e = std::getenv(var);
    int v = e ? std::atoi(e) : total / (n_pics > 0 ? n_pics : 1);
    if (!e) v = v < lo ? lo : (v > hi ? hi : v);
    return v < 1 ? 1 : (v > 1024 ? 1024 : v);
}

hipError_t launch_deblock(const BatchArgs &a, hipStream_t s) {
    dim3 grid(lf_blocks("HEIFGPU_DBK_BLOCKS", a.n_pics, 8192, 2, 64), a.n_pics), block(256);
    if (a.has_assembly) {  // the assemblies' children are reconstructed: put them together first
        if (a.bytes_per_sample == 1) hipLaunchKernelGGL(k_assemble<uint8_t>, grid, block, 0, s, a);
        else hipLaunchKernelGGL(k_assemble<uint16_t>, grid, block, 0, s, a);
    }
    if (lf_fused()) return hipGetLastError();  // deblocking runs inside k_loopfilter (launch_sao_out)
    if (a.bytes_per_sample == 1) {
        hipLaunchKernelGGL((k_deblock<uint8_t, true>), grid, block, 0, s, a);
        hipLaunchKernelGGL((k_deblock<uint8_t, false>), grid, block, 0, s, a);
    } else {
        hipLaunchKernelGGL((k_deblock<uint16_t, true>), grid, block, 0, s, a);
        hipLaunchKernelGGL((k_deblock<uint16_t, false>), grid, block, 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_sao_out(const BatchArgs &a, hipStream_t s) {
    if (lf_fused()) {
        const size_t lds = lf_lds_bytes(a.bytes_per_sample, a.chroma_format);
        const dim3 g(lf_tiles(a), a.n_pics), b(kLfWaves * 64);
        if (a.bytes_per_sample == 1) hipLaunchKernelGGL(k_loopfilter<uint8_t>, g, b, lds, s, a);
        else hipLaunchKernelGGL(k_loopfilter<uint16_t>, g, b, lds, s, a);
        return hipGetLastError();
    }
    dim3 grid(lf_blocks("HEIFGPU_SAO_BLOCKS", a.n_pics, 24576, 4, 256), a.n_pics), block(256);
    if (a.bytes_per_sample == 1) hipLaunchKernelGGL(k_sao_out<uint8_t>, grid, block, 0, s, a);
    else hipLaunchKernelGGL(k_sao_out<uint16_t>, grid, block, 0, s, a);
    return hipGetLastError();
}

// the batch's sticky status: every decode's per-picture status words ORed
// into one array that heifgpu_batch_status reads and clears, so damage seen
// by any of the pipelined decodes (three parse-output sets) is reported
__global__ void __launch_bounds__(256) k_status_fold(const uint32_t *__restrict__ st, uint32_t *__restrict__ sticky,
                                                     int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        const uint32_t v = st[i];
        if (v) sticky[i] |= v;
    }
}

hipError_t launch_status_fold(const uint32_t *status, uint32_t *sticky, int n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_status_fold, dim3((n + 255) / 256), dim3(256), 0, s, status, sticky, n);
    return hipGetLastError();
}
#endif

int lf_tiles_for(const PicDesc *pics, int n, const SeqParams *seqs) {
    int t = 0;
    for (int i = 0; i < n; ++i) {
        const SeqParams &sp = seqs[pics[i].seq];
        t = std::max(t, ((sp.width + kLfT - 1) / kLfT) * ((sp.height + kLfT - 1) / kLfT));
    }
    return t;
}

}  // namespace hg
