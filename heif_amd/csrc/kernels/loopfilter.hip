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

// t / d and t % d for 0 <= t < 2^24 and a divisor d >= 1 the wave shares, through
// its f32 reciprocal (computed once by the caller) and one correction each way:
// a handful of VALU instead of the ~40 of an integer division
struct FastDiv {
    int d;
    float r;
    __device__ __forceinline__ explicit FastDiv(int d_) : d(d_ > 0 ? d_ : 1), r(1.0f / (float)(d_ > 0 ? d_ : 1)) {}
    __device__ __forceinline__ int div(int t, int &rem) const {
        int q = (int)((float)t * r);
        rem = t - q * d;
        if (rem < 0) {
            --q;
            rem += d;
        } else if (rem >= d) {
            ++q;
            rem -= d;
        }
        return q;
    }
};

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
    const FastDiv dl(VERT ? ne_l : ns_l), dc(nc), dce(VERT ? ne_c : ns_c);
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        if (t < nl) {
            int x, y, tr;
            const int tq = dl.div(t, tr);
            if (VERT) {
                x = 8 * (tr + 1);
                y = 4 * tq;
            } else {
                x = 4 * tr;
                y = 8 * (tq + 1);
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
            int v, vr;
            const int cidx = 1 + dc.div(u, v);
            const int vq = dce.div(v, vr);
            int xc, yc;
            if (VERT) {
                xc = 8 * (vr + 1);
                yc = lc * vq;
            } else {
                xc = lc * vr;
                yc = 8 * (vq + 1);
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

// Four samples in one load: 4 x 8 bits in a dword, 4 x 16 bits in a qword
template <typename Pel>
struct QuadLoad;
template <>
struct QuadLoad<uint8_t> {
    using W = uint32_t;
    static __device__ __forceinline__ int at(W w, int j) { return (int)((w >> (8 * j)) & 0xffu); }
};
template <>
struct QuadLoad<uint16_t> {
    using W = uint64_t;
    static __device__ __forceinline__ int at(W w, int j) { return (int)((w >> (16 * j)) & 0xffffu); }
};

// SAO (8.7.3) of the four samples (xs0 .. xs0 + 3, ys) of component cidx when
// xs0 is a multiple of 4 and the four are one aligned load (then they share a
// CTB, and the neighbour rows are aligned loads too): the CTB's parameters
// read once, the neighbours of every edge class from two quads and two
// samples, no per-sample branches.  False: not applicable (sao_sample per
// sample).
template <typename Pel>
__device__ __forceinline__ bool sao_quad(const Pel *P, int PW, int PH, int xs0, int ys, int cidx, int subx, int suby,
                                         const SaoParams *sao, int wctb, int log2ctb, const uint8_t *flg, int w4,
                                         int bd, int v[4]) {
    using Q = QuadLoad<Pel>;
    using W = typename Q::W;
    const Pel *row = P + (size_t)ys * PW;
    if ((xs0 & 3) || (PW & 3) || (reinterpret_cast<uintptr_t>(row + xs0) & (sizeof(W) - 1))) return false;
    const W c = *reinterpret_cast<const W *>(row + xs0);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = Q::at(c, j);
    const SaoParams &s = sao[(ys >> (log2ctb - suby)) * wctb + (xs0 >> (log2ctb - subx))];
    const int type = s.type[cidx];
    if (!type) return true;
    // MF_NOFILT of each sample's 4x4 luma block: at most two blocks per quad
    const uint8_t *fr = flg + (size_t)((ys << suby) >> 2) * w4;
    const int b0 = (xs0 << subx) >> 2, b3 = ((xs0 + 3) << subx) >> 2;
    const int f0 = fr[b0], f3 = fr[b3];
    const int cl = s.band_eo[cidx];
    const int maxv = (1 << bd) - 1;
    int o[4] = {0, 0, 0, 0};
    if (type == 2) {
        const int hx = cl == 0 ? 1 : (cl == 1 ? 0 : (cl == 2 ? 1 : -1)), vy = cl == 0 ? 0 : 1;
        const int ya = ys - vy, yb = ys + vy;
        const bool va = ya >= 0, vb = yb < PH;
        const Pel *ra = P + (size_t)(va ? ya : ys) * PW, *rb = P + (size_t)(vb ? yb : ys) * PW;
        const W qa = *reinterpret_cast<const W *>(ra + xs0), qb = *reinterpret_cast<const W *>(rb + xs0);
        // the one sample of each neighbour row outside the quad: a at x - hx, b at x + hx
        const int xa_out = hx > 0 ? xs0 - 1 : xs0 + 4, xb_out = hx > 0 ? xs0 + 4 : xs0 - 1;
        const int ea = hx != 0 && xa_out >= 0 && xa_out < PW ? (int)ra[xa_out] : 0;
        const int eb = hx != 0 && xb_out >= 0 && xb_out < PW ? (int)rb[xb_out] : 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int ja = j - hx, jb = j + hx;  // quad positions of the neighbours (-1 or 4: outside)
            const int na = ja < 0 || ja > 3 ? ea : Q::at(qa, ja < 0 ? 0 : (ja > 3 ? 3 : ja));
            const int nb = jb < 0 || jb > 3 ? eb : Q::at(qb, jb < 0 ? 0 : (jb > 3 ? 3 : jb));
            const bool in = va && vb && xs0 + ja >= 0 && xs0 + ja < PW && xs0 + jb >= 0 && xs0 + jb < PW;
            int e = 2 + (v[j] > na) - (v[j] < na) + (v[j] > nb) - (v[j] < nb);
            e = e <= 2 ? (e == 2 ? 0 : e + 1) : e;
            o[j] = in && e ? s.off[cidx][e - 1] : 0;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = ((v[j] >> (bd - 5)) - cl) & 31;
            o[j] = k < 4 ? s.off[cidx][k] : 0;
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool nf = ((((xs0 + j) << subx) >> 2) == b0 ? f0 : f3) & MF_NOFILT;
        if (!nf) v[j] = clip3(0, maxv, v[j] + o[j]);
    }
    return true;
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
    const FastDiv dq(qw), dn(nc), dqc(qcw);
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        int cidx, q, y;
        if (t < nl) {
            cidx = 0;
            y = dq.div(t, q);
        } else {
            const int u = t - nl;
            int v;
            cidx = 1 + dn.div(u, v);
            y = dqc.div(v, q);
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
        if (!(n == 4 && on && sao_quad(P, PW, PH, xs0, ys, cidx, subx, suby, sao, wctb, log2ctb, flg, w4, bd, v))) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[j] = 0;
                if (j < n)
                    v[j] = on ? sao_sample(P, PW, PH, xs0 + j, ys, cidx, subx, suby, sao, wctb, log2ctb, flg, w4, bd)
                              : (int)P[(size_t)ys * PW + xs0 + j];
            }
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

// (r04 also had k_loopfilter: both deblocking directions, SAO and output per
// 64x64 tile in LDS, bit-exact, but 9.2 ms alone against 7.0 for the three
// kernels here and 53 against ~33 ms beside the next parse, whose residency its
// 9.6 KB of LDS per workgroup took; removed in r05)

#if defined(HG_HOST_EMU)
void emu_deblock(const BatchArgs &a) {
    if (a.has_assembly) {
        if (a.bytes_per_sample == 1) emu_launch(k_assemble<uint8_t>, 1, a.n_pics, 1, a, true);
        else emu_launch(k_assemble<uint16_t>, 1, a.n_pics, 1, a, true);
    }
    if (a.bytes_per_sample == 1) {
        emu_launch(k_deblock<uint8_t, true>, 1, a.n_pics, 1, a, true);
        emu_launch(k_deblock<uint8_t, false>, 1, a.n_pics, 1, a, true);
    } else {
        emu_launch(k_deblock<uint16_t, true>, 1, a.n_pics, 1, a, true);
        emu_launch(k_deblock<uint16_t, false>, 1, a.n_pics, 1, a, true);
    }
}
void emu_sao_out(const BatchArgs &a) {
    if (a.bytes_per_sample == 1) emu_launch(k_sao_out<uint8_t>, 1, a.n_pics, 1, a, true);
    else emu_launch(k_sao_out<uint16_t>, 1, a.n_pics, 1, a, true);
}
#else
// Workgroups per picture of the grid-stride loop filter kernels: about
// `total` workgroups for the batch, within [lo, hi] per picture.  A full batch
// (128 images) gets few long-lived workgroups per picture: beside the next
// decode's parse, 2 / 4 instead of 64 / 256 took deblocking 21 -> 7.7 ms and
// the step 85.9 -> 85.6 ms (r04 A/B); small batches keep many, for latency.
// HEIFGPU_DBK_BLOCKS / HEIFGPU_SAO_BLOCKS force a count (read once).
static int lf_blocks(int forced, int n_pics, int total, int lo, int hi) {
    int v = forced > 0 ? forced : total / (n_pics > 0 ? n_pics : 1);
    if (forced <= 0) v = v < lo ? lo : (v > hi ? hi : v);
    return v < 1 ? 1 : (v > 1024 ? 1024 : v);
}
static int env_int(const char *var) {
    const char *e = std::getenv(var);
    return e ? std::atoi(e) : 0;
}

hipError_t launch_deblock(const BatchArgs &a, hipStream_t s) {
    static const int forced = env_int("HEIFGPU_DBK_BLOCKS");
    dim3 grid(lf_blocks(forced, a.n_pics, 8192, 2, 64), a.n_pics), block(256);
    if (a.has_assembly) {  // the assemblies' children are reconstructed: put them together first
        if (a.bytes_per_sample == 1) hipLaunchKernelGGL(k_assemble<uint8_t>, grid, block, 0, s, a);
        else hipLaunchKernelGGL(k_assemble<uint16_t>, grid, block, 0, s, a);
    }
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
    static const int forced = env_int("HEIFGPU_SAO_BLOCKS");
    dim3 grid(lf_blocks(forced, a.n_pics, 24576, 4, 256), a.n_pics), block(256);
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

}  // namespace hg
