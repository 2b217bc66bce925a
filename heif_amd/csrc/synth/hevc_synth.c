/*
 * hevc_synth.c — synthetic HEVC intra picture generator (SURVEY.md §8(f)
 * row 3: Main-10 / 8K grid inputs; no 10-bit sample ships with the
 * reference, tests/ there hold only halfmoonbay.heic).
 *
 * This is a *syntax-driven* encoder: it walks the H.265 I-slice syntax
 * (7.3.8.1-7.3.8.12) exactly as a decoder would, but instead of decoding
 * each bin it draws the syntax element from a seeded RNG and CABAC-encodes it
 * with the same context selection (9.3.4.2).  No pixels are ever computed —
 * the only state it tracks is what context selection and the syntax itself
 * depend on (IntraPredModeY for MPM derivation and scanIdx, CtDepth for
 * split_cu_flag, IsCuQpDeltaCoded, coded_sub_block_flag, greater1 state).
 * The result is a conforming bitstream whose reconstruction exercises every
 * intra mode, TU size, transform-skip / bypass / sign hiding / scaling list /
 * cu_qp_delta path at any bit depth, chroma format 4:0:0 or 4:2:0, CTB size
 * and picture size, with WPP or tile substreams and entry points.
 *
 * Arithmetic coder: the standard low/range encoder with carry propagation
 * through buffered 0xff bytes (the inverse of 9.3.4.3), flushed at every
 * end_of_slice_segment_flag / end_of_subset_one_bit.
 *
 * Not part of the decode path: nothing in libheifgpu.so links this.  It is a
 * data generator used by tests/ and by bench.py's optional config-5 workload.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "hevc_synth.h"

/* ------------------------------------------------------------------ */
/* bit writer                                                          */
/* ------------------------------------------------------------------ */
typedef struct {
    uint8_t *d;
    size_t n, cap;   /* bytes complete */
    uint32_t acc;    /* pending bits */
    int nacc;
    int err;
} bw_t;

static void bw_byte(bw_t *w, uint32_t b) {
    if (w->n >= w->cap) {
        size_t nc = w->cap ? w->cap * 2 : 4096;
        uint8_t *nd = (uint8_t *)realloc(w->d, nc);
        if (!nd) { w->err = 1; return; }
        w->d = nd;
        w->cap = nc;
    }
    w->d[w->n++] = (uint8_t)b;
}
static void bw_bits(bw_t *w, uint32_t v, int n) {
    for (int i = n - 1; i >= 0; i--) {
        w->acc = (w->acc << 1) | ((v >> i) & 1);
        if (++w->nacc == 8) { bw_byte(w, w->acc & 0xff); w->acc = 0; w->nacc = 0; }
    }
}
static void bw_ue(bw_t *w, uint32_t v) {
    uint64_t x = (uint64_t)v + 1;
    int len = 0;
    while ((x >> len) > 1) len++;
    bw_bits(w, 0, len);
    bw_bits(w, (uint32_t)x, len + 1);
}
static void bw_se(bw_t *w, int32_t v) { bw_ue(w, v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * v)); }
static void bw_align1(bw_t *w) { /* rbsp_trailing_bits / byte_alignment(): 1 then zeros */
    bw_bits(w, 1, 1);
    while (w->nacc) bw_bits(w, 0, 1);
}

/* ------------------------------------------------------------------ */
/* RNG (splitmix64)                                                     */
/* ------------------------------------------------------------------ */
static uint64_t rng_next(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static int rnd(uint64_t *s, int n) { return (int)(rng_next(s) % (uint64_t)n); }
static int pct(uint64_t *s, int p) { return rnd(s, 100) < p; }

/* ------------------------------------------------------------------ */
/* CABAC tables (H.265 Tables 9-5..9-37 initType 0, 9-52, 9-53)         */
/* ------------------------------------------------------------------ */
enum {
    C_SAO_MERGE = 0, C_SAO_TYPE = 1, C_SPLIT_CU = 2, C_TQ_BYPASS = 5, C_PART_MODE = 6,
    C_PREV_INTRA = 7, C_CHROMA_MODE = 8, C_SPLIT_TF = 9, C_CBF_LUMA = 12, C_CBF_CHROMA = 14,
    C_CU_QP_DELTA = 19, C_TS_FLAG = 21, C_LAST_X = 23, C_LAST_Y = 41, C_CSBF = 59,
    C_SIG = 63, C_GT1 = 107, C_GT2 = 131, C_NUM = 137
};
static const uint8_t k_init[C_NUM] = {
    153, 200, 139, 141, 157, 154, 184, 184, 63, 153, 138, 138, 111, 141, 94, 138, 182, 154, 154, 154, 154,
    139, 139,
    110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,
    110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,
    91, 171, 134, 141,
    111, 111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107, 125, 141,
    179, 153, 125, 107, 125, 141, 179, 153, 125, 140, 139, 182, 182, 152, 136, 152, 136, 153,
    136, 139, 111, 136, 139, 111, 141, 111,
    140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152, 140, 179, 166,
    182, 140, 227, 122, 197,
    138, 153, 136, 167, 152, 152,
};
static const uint8_t k_lps[64][4] = {
    {128, 176, 208, 240}, {128, 167, 197, 227}, {128, 158, 187, 216}, {123, 150, 178, 205}, {116, 142, 169, 195},
    {111, 135, 160, 185}, {105, 128, 152, 175}, {100, 122, 144, 166}, {95, 116, 137, 158}, {90, 110, 130, 150},
    {85, 104, 123, 142}, {81, 99, 117, 135}, {77, 94, 111, 128}, {73, 89, 105, 122}, {69, 85, 100, 116},
    {66, 80, 95, 110}, {62, 76, 90, 104}, {59, 72, 86, 99}, {56, 69, 81, 94}, {53, 65, 77, 89},
    {51, 62, 73, 85}, {48, 59, 69, 80}, {46, 56, 66, 76}, {43, 53, 63, 72}, {41, 50, 59, 69},
    {39, 48, 56, 65}, {37, 45, 54, 62}, {35, 43, 51, 59}, {33, 41, 48, 56}, {32, 39, 46, 53},
    {30, 37, 43, 50}, {29, 35, 41, 48}, {27, 33, 39, 45}, {26, 31, 37, 43}, {24, 30, 35, 41},
    {23, 28, 33, 39}, {22, 27, 32, 37}, {21, 26, 30, 35}, {20, 24, 29, 33}, {19, 23, 27, 31},
    {18, 22, 26, 30}, {17, 21, 25, 28}, {16, 20, 23, 27}, {15, 19, 22, 25}, {14, 18, 21, 24},
    {14, 17, 20, 23}, {13, 16, 19, 22}, {12, 15, 18, 21}, {12, 14, 17, 20}, {11, 14, 16, 19},
    {11, 13, 15, 18}, {10, 12, 15, 17}, {10, 12, 14, 16}, {9, 11, 13, 15}, {9, 11, 12, 14},
    {8, 10, 12, 14}, {8, 9, 11, 13}, {7, 9, 11, 12}, {7, 9, 10, 12}, {7, 8, 10, 11},
    {6, 8, 9, 11}, {6, 7, 9, 10}, {6, 7, 8, 9}, {2, 2, 2, 2}};
static const uint8_t k_trans_lps[64] = {
    0, 0, 1, 2, 2, 4, 4, 5, 6, 7, 8, 9, 9, 11, 11, 12, 13, 13, 15, 15, 16, 16,
    18, 18, 19, 19, 21, 21, 22, 22, 23, 24, 24, 25, 26, 26, 27, 27, 28, 29, 29, 30,
    30, 30, 31, 32, 32, 33, 33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63};

/* ------------------------------------------------------------------ */
/* arithmetic encoder                                                   */
/* ------------------------------------------------------------------ */
typedef struct {
    bw_t *w;
    uint32_t low, range;
    int bits_left, nbuf;
    uint32_t buf_byte;
    uint8_t st[C_NUM], mps[C_NUM];
} cabe_t;

static void ce_init_ctx(cabe_t *c, int qp) {
    int q = qp < 0 ? 0 : qp > 51 ? 51 : qp;
    for (int i = 0; i < C_NUM; i++) {
        int v = k_init[i];
        int m = (v >> 4) * 5 - 45, nn = ((v & 15) << 3) - 16;
        int pre = ((m * q) >> 4) + nn;
        pre = pre < 1 ? 1 : pre > 126 ? 126 : pre;
        c->mps[i] = pre > 63;
        c->st[i] = (uint8_t)(c->mps[i] ? pre - 64 : 63 - pre);
    }
}
static void ce_start(cabe_t *c, bw_t *w) {
    c->w = w;
    c->low = 0;
    c->range = 510;
    c->bits_left = 23;
    c->nbuf = 0;
    c->buf_byte = 0xff;
}
static void ce_write_out(cabe_t *c) {
    uint32_t lead = c->low >> (24 - c->bits_left);
    c->bits_left += 8;
    c->low &= 0xffffffffu >> c->bits_left;
    if (lead == 0xff) {
        c->nbuf++;
    } else if (c->nbuf > 0) {
        uint32_t carry = lead >> 8;
        bw_bits(c->w, (c->buf_byte + carry) & 0xff, 8);
        c->buf_byte = lead & 0xff;
        uint32_t fill = (0xff + carry) & 0xff;
        while (c->nbuf > 1) { bw_bits(c->w, fill, 8); c->nbuf--; }
    } else {
        c->nbuf = 1;
        c->buf_byte = lead;
    }
}
static void ce_test(cabe_t *c) { if (c->bits_left < 12) ce_write_out(c); }
static void ce_bin(cabe_t *c, int ci, int bin) {
    uint32_t s = c->st[ci];
    uint32_t lps = k_lps[s][(c->range >> 6) & 3];
    c->range -= lps;
    if (bin != c->mps[ci]) {
        int nb = 0;
        while ((lps << nb) < 256) nb++;
        c->low = (c->low + c->range) << nb;
        c->range = lps << nb;
        if (s == 0) c->mps[ci] = (uint8_t)(1 - c->mps[ci]);
        c->st[ci] = k_trans_lps[s];
        c->bits_left -= nb;
    } else {
        c->st[ci] = (uint8_t)(s < 62 ? s + 1 : s);
        if (c->range >= 256) return;
        c->low <<= 1;
        c->range <<= 1;
        c->bits_left--;
    }
    ce_test(c);
}
static void ce_bypass(cabe_t *c, int bin) {
    c->low <<= 1;
    if (bin) c->low += c->range;
    c->bits_left--;
    ce_test(c);
}
static void ce_term(cabe_t *c, int bin) {
    c->range -= 2;
    if (bin) {
        c->low += c->range;
        c->low <<= 7;
        c->range = 2 << 7;
        c->bits_left -= 7;
    } else if (c->range >= 256) {
        return;
    } else {
        c->low <<= 1;
        c->range <<= 1;
        c->bits_left--;
    }
    ce_test(c);
}
static void ce_finish(cabe_t *c) {
    if (c->low >> (32 - c->bits_left)) {
        bw_bits(c->w, (c->buf_byte + 1) & 0xff, 8);
        while (c->nbuf > 1) { bw_bits(c->w, 0x00, 8); c->nbuf--; }
        c->low -= 1u << (32 - c->bits_left);
    } else {
        if (c->nbuf > 0) bw_bits(c->w, c->buf_byte, 8);
        while (c->nbuf > 1) { bw_bits(c->w, 0xff, 8); c->nbuf--; }
    }
    bw_bits(c->w, c->low >> 8, 24 - c->bits_left);
}
static void ce_fl(cabe_t *c, uint32_t v, int n) {
    for (int i = n - 1; i >= 0; i--) ce_bypass(c, (v >> i) & 1);
}
static void ce_egk(cabe_t *c, uint32_t v, int k) {
    for (;;) {
        if (v >= (1u << k)) { ce_bypass(c, 1); v -= 1u << k; k++; }
        else { ce_bypass(c, 0); ce_fl(c, v, k); break; }
    }
}
/* TR (9.3.3.2) with bypass bins */
static void ce_tr_bypass(cabe_t *c, int v, int cmax, int crice) {
    int p = v >> crice, pmax = cmax >> crice;
    for (int i = 0; i < p; i++) ce_bypass(c, 1);
    if (p < pmax) ce_bypass(c, 0);
    if (crice > 0 && p < pmax) ce_fl(c, (uint32_t)v & ((1u << crice) - 1), crice);
}
/* coeff_abs_level_remaining (9.3.3.11) */
static void ce_calr(cabe_t *c, int v, int k) {
    int cmax = 4 << k;
    if (v < cmax) ce_tr_bypass(c, v, cmax, k);
    else {
        for (int i = 0; i < 4; i++) ce_bypass(c, 1);
        ce_egk(c, (uint32_t)(v - cmax), k + 1);
    }
}

/* ------------------------------------------------------------------ */
/* scans (6.5.3-6.5.5), entries (y << 4) | x                            */
/* ------------------------------------------------------------------ */
static uint8_t g_scan[4][3][64];
static void init_scans(void) {
    static int ready = 0;
    if (ready) return;
    for (int l = 0; l < 4; l++) {
        int n = 1 << l, i = 0, x = 0, y = 0;
        while (i < n * n) {
            while (y >= 0) {
                if (x < n && y < n) g_scan[l][0][i++] = (uint8_t)((y << 4) | x);
                y--;
                x++;
            }
            y = x;
            x = 0;
        }
        i = 0;
        for (y = 0; y < n; y++)
            for (x = 0; x < n; x++) g_scan[l][1][i++] = (uint8_t)((y << 4) | x);
        i = 0;
        for (x = 0; x < n; x++)
            for (y = 0; y < n; y++) g_scan[l][2][i++] = (uint8_t)((y << 4) | x);
    }
    ready = 1;
}

/* ------------------------------------------------------------------ */
/* picture state                                                        */
/* ------------------------------------------------------------------ */
typedef struct {
    const synth_params *P;
    uint64_t rng;
    cabe_t c;
    int W, H, log2ctb, ctb, wctb, hctb, w4, h4, qpbdY;
    uint8_t *ipm, *depth;
    int *ts2rs, *tile_rs; /* 6.5.1 tile scan; tile of each CTB by raster address */
    int *slice_rs;        /* slice of each CTB by raster address */
    /* current CU */
    int cu_bypass, intra_split, max_trafo_depth;
    int cu_x, cu_y, cu_pb, chroma_mode[4];  /* IntraPredModeC per PB (4:4:4 NxN: four) */
    int is_qp_coded;
} pic_t;

static void set_map(pic_t *p, uint8_t *m, int x0, int y0, int n, uint8_t v) {
    for (int y = y0 >> 2; y < (y0 + n) >> 2 && y < p->h4; y++)
        for (int x = x0 >> 2; x < (x0 + n) >> 2 && x < p->w4; x++) m[y * p->w4 + x] = v;
}

static int tiles_on(const synth_params *P) { return P->tile_cols * P->tile_rows > 1; }

/* the neighbour (xn,yn) of (x,y) lies in the same tile and slice (availability
 * 6.4.1; in the picture and earlier in decoding order is the caller's check) */
static int same_tile(const pic_t *p, int x, int y, int xn, int yn) {
    const int a = (yn >> p->log2ctb) * p->wctb + (xn >> p->log2ctb), b = (y >> p->log2ctb) * p->wctb + (x >> p->log2ctb);
    return p->tile_rs[a] == p->tile_rs[b] && p->slice_rs[a] == p->slice_rs[b];
}

/* 6.5.1 column / row boundaries (6-3..6-6) → CtbAddrTsToRs, TileId */
static int tile_layout(pic_t *p) {
    const synth_params *P = p->P;
    int nc = tiles_on(P) ? P->tile_cols : 1, nr = tiles_on(P) ? P->tile_rows : 1;
    int colBd[SYNTH_MAX_TILES + 1], rowBd[SYNTH_MAX_TILES + 1];
    for (int pass = 0; pass < 2; pass++) {
        int n = pass ? nr : nc, tot = pass ? p->hctb : p->wctb, *bd = pass ? rowBd : colBd;
        const int32_t *ex = pass ? P->tile_row_h : P->tile_col_w;
        bd[0] = 0;
        for (int i = 0; i < n; i++) {
            int sz = (!tiles_on(P) || P->tile_uniform) ? ((i + 1) * tot) / n - (i * tot) / n
                                                       : (i + 1 < n ? ex[i] : tot - bd[i]);
            if (sz <= 0) return -1;
            bd[i + 1] = bd[i] + sz;
        }
    }
    int nctb = p->wctb * p->hctb, ts = 0;
    p->ts2rs = (int *)malloc(sizeof(int) * (size_t)nctb);
    p->tile_rs = (int *)malloc(sizeof(int) * (size_t)nctb);
    if (!p->ts2rs || !p->tile_rs) return -1;
    for (int ty = 0; ty < nr; ty++)
        for (int tx = 0; tx < nc; tx++)
            for (int y = rowBd[ty]; y < rowBd[ty + 1]; y++)
                for (int x = colBd[tx]; x < colBd[tx + 1]; x++) {
                    p->ts2rs[ts++] = y * p->wctb + x;
                    p->tile_rs[y * p->wctb + x] = ty * nc + tx;
                }
    return 0;
}

static int scan_idx_for(const pic_t *p, int log2n, int cIdx, int mode) {
    if (log2n == 2 || (log2n == 3 && (cIdx == 0 || p->P->chroma_format == 3))) {
        if (mode >= 6 && mode <= 14) return 2;
        if (mode >= 22 && mode <= 30) return 1;
    }
    return 0;
}

/* a small non-negative level with a long tail */
static int draw_remaining(pic_t *p) {
    int r = rnd(&p->rng, 100);
    if (r < 60) return rnd(&p->rng, 3);
    if (r < 90) return rnd(&p->rng, 16);
    if (r < 99) return rnd(&p->rng, 200);
    return rnd(&p->rng, 3000);
}

/* 7.3.8.11 residual_coding, bins drawn at random */
static void residual_coding(pic_t *p, int log2n, int cIdx, int mode) {
    cabe_t *c = &p->c;
    const synth_params *P = p->P;
    int n = 1 << log2n;
    if (P->transform_skip && !p->cu_bypass && log2n <= 2) ce_bin(c, C_TS_FLAG + (cIdx ? 1 : 0), pct(&p->rng, 25));
    int scanIdx = scan_idx_for(p, log2n, cIdx, mode);
    /* last significant position: biased towards low frequencies */
    int lx, ly;
    if (pct(&p->rng, 70)) { lx = rnd(&p->rng, n < 8 ? n : 8); ly = rnd(&p->rng, n < 8 ? n : 8); }
    else { lx = rnd(&p->rng, n); ly = rnd(&p->rng, n); }
    if (P->density <= 10) { lx = lx < 4 ? lx : rnd(&p->rng, 4); ly = ly < 4 ? ly : rnd(&p->rng, 4); }
    int sx = lx, sy = ly;
    if (scanIdx == 2) { sx = ly; sy = lx; }
    int cmax = (log2n << 1) - 1, off, shift;
    if (cIdx == 0) { off = 3 * (log2n - 2) + ((log2n - 1) >> 2); shift = (log2n + 1) >> 2; }
    else { off = 15; shift = log2n - 2; }
    int pre[2], suf[2], sk[2];
    for (int a = 0; a < 2; a++) {
        int v = a ? sy : sx;
        if (v < 4) { pre[a] = v; sk[a] = 0; suf[a] = 0; }
        else {
            int pp = 4;
            for (;; pp++) {
                int k = (pp >> 1) - 1, base = (1 << k) * (2 + (pp & 1));
                if (v >= base && v < base + (1 << k)) { pre[a] = pp; sk[a] = k; suf[a] = v - base; break; }
            }
        }
    }
    for (int i = 0; i < pre[0]; i++) ce_bin(c, C_LAST_X + off + (i >> shift), 1);
    if (pre[0] < cmax) ce_bin(c, C_LAST_X + off + (pre[0] >> shift), 0);
    for (int i = 0; i < pre[1]; i++) ce_bin(c, C_LAST_Y + off + (i >> shift), 1);
    if (pre[1] < cmax) ce_bin(c, C_LAST_Y + off + (pre[1] >> shift), 0);
    if (pre[0] > 3) ce_fl(c, (uint32_t)suf[0], sk[0]);
    if (pre[1] > 3) ce_fl(c, (uint32_t)suf[1], sk[1]);

    int sbl = log2n - 2, sbw = 1 << sbl;
    const uint8_t *sbscan = g_scan[sbl][scanIdx], *scan4 = g_scan[2][scanIdx];
    int lastSub = sbw * sbw - 1, lastPos = 16;
    for (;;) {
        if (lastPos == 0) { lastPos = 16; lastSub--; }
        lastPos--;
        int xS = sbscan[lastSub] & 15, yS = sbscan[lastSub] >> 4;
        int xC = (xS << 2) + (scan4[lastPos] & 15), yC = (yS << 2) + (scan4[lastPos] >> 4);
        if (xC == lx && yC == ly) break;
    }
    int dens = P->density;
    uint8_t csbf[8][8];
    memset(csbf, 0, sizeof(csbf));
    int g1prev = 1, first_sb_done = 0;
    static const uint8_t ctxIdxMap[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
    for (int i = lastSub; i >= 0; i--) {
        int xS = sbscan[i] & 15, yS = sbscan[i] >> 4;
        int infer_dc = 0, coded;
        if (i < lastSub && i > 0) {
            int r = (xS + 1 < sbw) ? csbf[yS][xS + 1] : 0;
            int b = (yS + 1 < sbw) ? csbf[yS + 1][xS] : 0;
            coded = pct(&p->rng, 55);
            ce_bin(c, C_CSBF + ((r + b) ? 1 : 0) + (cIdx ? 2 : 0), coded);
            infer_dc = 1;
        } else {
            coded = 1;
        }
        csbf[yS][xS] = (uint8_t)coded;
        int sig[16] = {0};
        int prevCsbf = 0;
        if (xS < sbw - 1) prevCsbf += csbf[yS][xS + 1];
        if (yS < sbw - 1) prevCsbf += csbf[yS + 1][xS] << 1;
        int nstart = (i == lastSub) ? lastPos - 1 : 15;
        if (i == lastSub) sig[lastPos] = 1;
        for (int nn = nstart; nn >= 0; nn--) {
            int xP = scan4[nn] & 15, yP = scan4[nn] >> 4;
            int xC = (xS << 2) + xP, yC = (yS << 2) + yP;
            if (coded && (nn > 0 || !infer_dc)) {
                int sigCtx;
                if (log2n == 2) sigCtx = ctxIdxMap[(yC << 2) + xC];
                else if (xC + yC == 0) sigCtx = 0;
                else {
                    if (prevCsbf == 0) sigCtx = (xP + yP == 0) ? 2 : (xP + yP < 3) ? 1 : 0;
                    else if (prevCsbf == 1) sigCtx = (yP == 0) ? 2 : (yP == 1) ? 1 : 0;
                    else if (prevCsbf == 2) sigCtx = (xP == 0) ? 2 : (xP == 1) ? 1 : 0;
                    else sigCtx = 2;
                    if (cIdx == 0) {
                        if (xS > 0 || yS > 0) sigCtx += 3;
                        sigCtx += (log2n == 3) ? ((scanIdx == 0) ? 9 : 15) : 21;
                    } else {
                        sigCtx += (log2n == 3) ? 9 : 12;
                    }
                }
                sig[nn] = pct(&p->rng, dens);
                ce_bin(c, C_SIG + (cIdx == 0 ? sigCtx : 27 + sigCtx), sig[nn]);
                if (sig[nn]) infer_dc = 0;
            } else if (coded && nn == 0 && infer_dc) {
                sig[0] = 1;
            }
        }
        int any = 0;
        for (int nn = 0; nn < 16; nn++) any |= sig[nn];
        if (!any) continue;
        int ctxSet = (i == 0 || cIdx > 0) ? 0 : 2;
        if (first_sb_done && g1prev == 0) ctxSet++;
        first_sb_done = 1;
        int g1c = 1, firstSig = 16, lastSig = -1, numG1 = 0, lastG1Pos = -1;
        int g1[16] = {0}, g2[16] = {0};
        for (int nn = 15; nn >= 0; nn--) {
            if (!sig[nn]) continue;
            if (numG1 < 8) {
                g1[nn] = pct(&p->rng, 35);
                ce_bin(c, C_GT1 + ctxSet * 4 + (g1c < 3 ? g1c : 3) + (cIdx ? 16 : 0), g1[nn]);
                numG1++;
                if (g1[nn] && lastG1Pos == -1) lastG1Pos = nn;
                if (g1c > 0) g1c = g1[nn] ? 0 : g1c + 1;
            }
            if (lastSig == -1) lastSig = nn;
            firstSig = nn;
        }
        g1prev = g1c;
        int hidden = p->cu_bypass ? 0 : (lastSig - firstSig > 3);
        if (lastG1Pos != -1) {
            g2[lastG1Pos] = pct(&p->rng, 40);
            ce_bin(c, C_GT2 + ctxSet + (cIdx ? 4 : 0), g2[lastG1Pos]);
        }
        for (int nn = 15; nn >= 0; nn--)
            if (sig[nn] && (!P->sign_hiding || !hidden || nn != firstSig)) ce_bypass(c, pct(&p->rng, 50));
        int numSig = 0, cLastAbs = 0, cLastRice = 0, firstRem = 1;
        for (int nn = 15; nn >= 0; nn--) {
            if (!sig[nn]) continue;
            int base = 1 + g1[nn] + g2[nn];
            if (base == ((numSig < 8) ? ((nn == lastG1Pos) ? 3 : 2) : 1)) {
                int k;
                if (firstRem) { k = 0; firstRem = 0; }
                else k = cLastRice + (cLastAbs > 3 * (1 << cLastRice) ? 1 : 0) < 4
                             ? cLastRice + (cLastAbs > 3 * (1 << cLastRice) ? 1 : 0) : 4;
                int rem = draw_remaining(p);
                ce_calr(c, rem, k);
                cLastAbs = base + rem;
                cLastRice = k;
            }
            numSig++;
        }
    }
}

static void transform_unit(pic_t *p, int x0, int y0, int log2n, int blk, int cbf_l, int cbf_cb, int cbf_cr,
                           int pcb, int pcr) {
    const synth_params *P = p->P;
    int chroma4 = log2n == 2 && P->chroma_format != 3;
    int cbfChroma = P->chroma_format == 0 ? 0 : (chroma4 ? (pcb || pcr) : (cbf_cb || cbf_cr));
    if ((cbf_l || cbfChroma) && P->cu_qp_delta && !p->is_qp_coded) {
        int lim = 26 + p->qpbdY / 2;
        int v = pct(&p->rng, 70) ? rnd(&p->rng, 5) - 2 : rnd(&p->rng, 2 * lim) - lim;
        int a = v < 0 ? -v : v;
        for (int i = 0; i < (a < 5 ? a : 5); i++) ce_bin(&p->c, C_CU_QP_DELTA + (i == 0 ? 0 : 1), 1);
        if (a < 5) ce_bin(&p->c, C_CU_QP_DELTA + (a == 0 ? 0 : 1), 0);
        else ce_egk(&p->c, (uint32_t)(a - 5), 0);
        if (a) ce_bypass(&p->c, v < 0);
        p->is_qp_coded = 1;
    }
    int lmode = p->ipm[(y0 >> 2) * p->w4 + (x0 >> 2)];
    if (cbf_l) residual_coding(p, log2n, 0, lmode);
    if (P->chroma_format == 0) return;
    /* chroma TBs (7.3.8.10): log2TrafoSizeC, two per component with 4:2:2
     * (cbf bits 0 / 1); 4x4 luma TBs (not 4:4:4): the 8x8 parent's chroma */
    const int k = ((y0 - p->cu_y) >= p->cu_pb ? 2 : 0) + ((x0 - p->cu_x) >= p->cu_pb ? 1 : 0);
    const int cm = p->chroma_mode[P->chroma_format == 3 && p->intra_split ? k : 0];
    const int l2c = chroma4 ? 2 : (P->chroma_format == 3 ? log2n : log2n - 1);
    if (!chroma4 || blk == 3)
        for (int ci = 1; ci < 3; ci++)
            for (int h = 0; h < (P->chroma_format == 2 ? 2 : 1); h++) {
                const int cbf = chroma4 ? (ci == 1 ? pcb : pcr) : (ci == 1 ? cbf_cb : cbf_cr);
                if ((cbf >> h) & 1) residual_coding(p, l2c, ci, cm);
            }
}

static void transform_tree(pic_t *p, int x0, int y0, int log2n, int depth, int blk, int pcb, int pcr) {
    const synth_params *P = p->P;
    int split;
    if (log2n <= P->log2_max_tb && log2n > P->log2_min_tb && depth < p->max_trafo_depth &&
        !(p->intra_split && depth == 0)) {
        split = pct(&p->rng, 40);
        ce_bin(&p->c, C_SPLIT_TF + 5 - log2n, split);
    } else {
        split = (log2n > P->log2_max_tb || (p->intra_split && depth == 0));
    }
    int cbf_cb = 0, cbf_cr = 0;  /* bit 1: 4:2:2 lower chroma TB (coded when not split or 8x8) */
    if ((log2n > 2 && P->chroma_format != 0) || P->chroma_format == 3) {
        const int two = P->chroma_format == 2 && (!split || log2n == 3);
        for (int ci = 0; ci < 2; ci++) {
            if (!(depth == 0 || ((ci ? pcr : pcb) & 1))) continue;
            int v = 0;
            for (int h = 0; h < (two ? 2 : 1); h++) {
                const int b = pct(&p->rng, 50);
                ce_bin(&p->c, C_CBF_CHROMA + depth, b);
                v |= b << h;
            }
            if (ci) cbf_cr = v;
            else cbf_cb = v;
        }
    }
    if (split) {
        int h = 1 << (log2n - 1);
        transform_tree(p, x0, y0, log2n - 1, depth + 1, 0, cbf_cb, cbf_cr);
        transform_tree(p, x0 + h, y0, log2n - 1, depth + 1, 1, cbf_cb, cbf_cr);
        transform_tree(p, x0, y0 + h, log2n - 1, depth + 1, 2, cbf_cb, cbf_cr);
        transform_tree(p, x0 + h, y0 + h, log2n - 1, depth + 1, 3, cbf_cb, cbf_cr);
        return;
    }
    int cbf_l = pct(&p->rng, 60);
    ce_bin(&p->c, C_CBF_LUMA + (depth == 0 ? 1 : 0), cbf_l);
    transform_unit(p, x0, y0, log2n, blk, cbf_l, cbf_cb, cbf_cr, pcb, pcr);
}

/* 8.4.2 candidate list */
static void mpm_list(pic_t *p, int xPb, int yPb, int l[3]) {
    int cand[2];
    for (int k = 0; k < 2; k++) {
        int xn = k == 0 ? xPb - 1 : xPb, yn = k == 0 ? yPb : yPb - 1;
        if (xn < 0 || yn < 0 || !same_tile(p, xPb, yPb, xn, yn)) cand[k] = 1;
        else if (k == 1 && yPb - 1 < ((yPb >> p->log2ctb) << p->log2ctb)) cand[k] = 1;
        else cand[k] = p->ipm[(yn >> 2) * p->w4 + (xn >> 2)];
    }
    if (cand[0] == cand[1]) {
        if (cand[0] < 2) { l[0] = 0; l[1] = 1; l[2] = 26; }
        else { l[0] = cand[0]; l[1] = 2 + ((cand[0] + 29) % 32); l[2] = 2 + ((cand[0] - 2 + 1) % 32); }
    } else {
        l[0] = cand[0];
        l[1] = cand[1];
        if (l[0] != 0 && l[1] != 0) l[2] = 0;
        else if (l[0] != 1 && l[1] != 1) l[2] = 1;
        else l[2] = 26;
    }
}

static void coding_unit(pic_t *p, int x0, int y0, int log2cb, int depth) {
    const synth_params *P = p->P;
    cabe_t *c = &p->c;
    int n = 1 << log2cb;
    p->cu_bypass = 0;
    if (P->tq_bypass) { p->cu_bypass = pct(&p->rng, 15); ce_bin(c, C_TQ_BYPASS, p->cu_bypass); }
    int nxn = 0;
    if (log2cb == P->log2_min_cb) {
        nxn = log2cb > P->log2_min_tb ? pct(&p->rng, 35) : 0;
        ce_bin(c, C_PART_MODE, !nxn);
    }
    set_map(p, p->depth, x0, y0, n, (uint8_t)depth);
    if (!nxn && P->pcm && log2cb >= P->pcm_log2_min && log2cb <= P->pcm_log2_max) {
        const int pcm = pct(&p->rng, P->pcm_pct);
        ce_term(c, pcm); /* pcm_flag */
        if (pcm) {       /* 7.3.8.7: flush + 1 + alignment zeros, raw samples, engine restart */
            set_map(p, p->ipm, x0, y0, n, 1);
            ce_finish(c);
            bw_align1(c->w);
            for (int ci = 0; ci < (P->chroma_format ? 3 : 1); ci++) {
                const int sw = P->chroma_format == 3 ? 1 : 2, sh = P->chroma_format == 1 ? 2 : 1;
                const int ns = ci ? (n / sw) * (n / sh) : n * n, bd = ci ? P->pcm_bd_c : P->pcm_bd_y;
                for (int k = 0; k < ns; k++) bw_bits(c->w, (uint32_t)rnd(&p->rng, 1 << bd), bd);
            }
            ce_start(c, c->w);
            return;
        }
    }
    int np = nxn ? 4 : 1, pb = nxn ? n / 2 : n;
    int prev[4], mpm[4] = {0}, rem[4] = {0};
    for (int i = 0; i < np; i++) {
        prev[i] = pct(&p->rng, 45);
        ce_bin(c, C_PREV_INTRA, prev[i]);
    }
    for (int i = 0; i < np; i++) {
        if (prev[i]) {
            mpm[i] = rnd(&p->rng, 3);
            ce_bypass(c, mpm[i] > 0);
            if (mpm[i] > 0) ce_bypass(c, mpm[i] > 1);
        } else {
            rem[i] = rnd(&p->rng, 32);
            ce_fl(c, (uint32_t)rem[i], 5);
        }
        int xPb = x0 + (i & 1) * pb, yPb = y0 + (i >> 1) * pb;
        int l[3], m;
        mpm_list(p, xPb, yPb, l);
        if (prev[i]) m = l[mpm[i]];
        else {
            if (l[0] > l[1]) { int t = l[0]; l[0] = l[1]; l[1] = t; }
            if (l[0] > l[2]) { int t = l[0]; l[0] = l[2]; l[2] = t; }
            if (l[1] > l[2]) { int t = l[1]; l[1] = l[2]; l[2] = t; }
            m = rem[i];
            for (int k = 0; k < 3; k++)
                if (m >= l[k]) m++;
        }
        set_map(p, p->ipm, xPb, yPb, pb, (uint8_t)m);
    }
    /* intra_chroma_pred_mode per PB with 4:4:4, else per CU; 8.4.3 (Table 8-3 with 4:2:2) */
    static const uint8_t k_mode422[35] = {0,  1,  2,  2,  2,  2,  3,  5,  7,  8,  10, 11, 13, 15, 16, 18, 19, 20,
                                          21, 22, 23, 23, 24, 24, 25, 25, 26, 27, 27, 28, 28, 29, 29, 30, 31};
    p->cu_x = x0;
    p->cu_y = y0;
    p->cu_pb = pb;
    for (int i = 0; P->chroma_format != 0 && i < (P->chroma_format == 3 ? np : 1); i++) {
        int icpm = rnd(&p->rng, 5);
        ce_bin(c, C_CHROMA_MODE, icpm != 4);
        if (icpm != 4) ce_fl(c, (uint32_t)icpm, 2);
        const int xPb = x0 + (i & 1) * pb, yPb = y0 + (i >> 1) * pb;
        int lm = p->ipm[(yPb >> 2) * p->w4 + (xPb >> 2)];
        static const int base[4] = {0, 26, 10, 1};
        const int cm = icpm == 4 ? lm : (base[icpm] == lm ? 34 : base[icpm]);
        p->chroma_mode[i] = P->chroma_format == 2 ? k_mode422[cm] : cm;
    }
    p->intra_split = nxn;
    p->max_trafo_depth = P->max_th_depth_intra + nxn;
    transform_tree(p, x0, y0, log2cb, 0, 0, 0, 0);
}

static void coding_quadtree(pic_t *p, int x0, int y0, int log2cb, int depth) {
    const synth_params *P = p->P;
    int n = 1 << log2cb, split;
    if (x0 + n <= p->W && y0 + n <= p->H && log2cb > P->log2_min_cb) {
        int cond = 0;
        if (x0 > 0 && same_tile(p, x0, y0, x0 - 1, y0) && p->depth[(y0 >> 2) * p->w4 + ((x0 - 1) >> 2)] > depth)
            cond++;
        if (y0 > 0 && same_tile(p, x0, y0, x0, y0 - 1) && p->depth[((y0 - 1) >> 2) * p->w4 + (x0 >> 2)] > depth)
            cond++;
        split = pct(&p->rng, log2cb >= 5 ? 60 : 45);
        ce_bin(&p->c, C_SPLIT_CU + cond, split);
    } else {
        split = log2cb > P->log2_min_cb;
    }
    if (P->cu_qp_delta && log2cb >= p->log2ctb - P->diff_cu_qp_delta_depth) p->is_qp_coded = 0;
    if (split) {
        int h = n >> 1;
        coding_quadtree(p, x0, y0, log2cb - 1, depth + 1);
        if (x0 + h < p->W) coding_quadtree(p, x0 + h, y0, log2cb - 1, depth + 1);
        if (y0 + h < p->H) coding_quadtree(p, x0, y0 + h, log2cb - 1, depth + 1);
        if (x0 + h < p->W && y0 + h < p->H) coding_quadtree(p, x0 + h, y0 + h, log2cb - 1, depth + 1);
        return;
    }
    coding_unit(p, x0, y0, log2cb, depth);
}

/* 7.3.8.3 */
static void sao_syntax(pic_t *p, int rx, int ry, int sao_l, int sao_c) {
    const synth_params *P = p->P;
    cabe_t *c = &p->c;
    if (rx > 0 && same_tile(p, rx << p->log2ctb, ry << p->log2ctb, (rx - 1) << p->log2ctb, ry << p->log2ctb)) {
        int ml = pct(&p->rng, 25);
        ce_bin(c, C_SAO_MERGE, ml);
        if (ml) return;
    }
    if (ry > 0 && same_tile(p, rx << p->log2ctb, ry << p->log2ctb, rx << p->log2ctb, (ry - 1) << p->log2ctb)) {
        int mu = pct(&p->rng, 25);
        ce_bin(c, C_SAO_MERGE, mu);
        if (mu) return;
    }
    int ncomp = P->chroma_format ? 3 : 1, type1 = 0;
    for (int ci = 0; ci < ncomp; ci++) {
        if (!((sao_l && ci == 0) || (sao_c && ci > 0))) continue;
        int t;
        if (ci < 2) {
            t = rnd(&p->rng, 3);
            ce_bin(c, C_SAO_TYPE, t != 0);
            if (t) ce_bypass(c, t == 2);
            if (ci == 1) type1 = t;
        } else {
            t = type1;
        }
        if (!t) continue;
        int bd = P->bit_depth, cmax = (1 << ((bd < 10 ? bd : 10) - 5)) - 1;
        int a[4];
        for (int i = 0; i < 4; i++) {
            a[i] = pct(&p->rng, 30) ? 0 : rnd(&p->rng, cmax + 1);
            ce_tr_bypass(c, a[i], cmax, 0);
        }
        if (t == 1) {
            for (int i = 0; i < 4; i++)
                if (a[i]) ce_bypass(c, pct(&p->rng, 50));
            ce_fl(c, (uint32_t)rnd(&p->rng, 32), 5);
        } else if (ci < 2) {
            ce_fl(c, (uint32_t)rnd(&p->rng, 4), 2);
        }
    }
}

/* ------------------------------------------------------------------ */
/* NAL assembly                                                         */
/* ------------------------------------------------------------------ */
static void nal_header(bw_t *w, int type) {
    bw_bits(w, 0, 1);
    bw_bits(w, (uint32_t)type, 6);
    bw_bits(w, 0, 6);
    bw_bits(w, 1, 3);
}

/* copy rbsp[hdr..) with emulation prevention (7.4.2); returns bytes written */
static size_t ep_insert(const uint8_t *in, size_t n, uint8_t *out, size_t cap, int *zeros_io) {
    size_t o = 0;
    int z = zeros_io ? *zeros_io : 0;
    for (size_t i = 0; i < n; i++) {
        if (z >= 2 && in[i] <= 3) {
            if (o >= cap) return (size_t)-1;
            out[o++] = 3;
            z = 0;
        }
        if (o >= cap) return (size_t)-1;
        out[o++] = in[i];
        z = in[i] == 0 ? z + 1 : 0;
    }
    if (zeros_io) *zeros_io = z;
    return o;
}

static int profile_idc(const synth_params *P) {
    if (P->chroma_format != 1 || P->bit_depth > 10) return 4; /* format range extensions */
    return P->bit_depth > 8 ? 2 : 1;
}

static void ptl(bw_t *w, const synth_params *P) {
    int pi = profile_idc(P);
    bw_bits(w, 0, 2);
    bw_bits(w, 0, 1);
    bw_bits(w, (uint32_t)pi, 5);
    uint32_t compat = 1u << (31 - pi);
    if (pi == 1) compat |= 1u << (31 - 2);
    bw_bits(w, compat, 32);
    bw_bits(w, 1, 1); /* progressive */
    bw_bits(w, 0, 1);
    bw_bits(w, 0, 1);
    bw_bits(w, 1, 1); /* frame only */
    bw_bits(w, 0, 32);
    bw_bits(w, 0, 11);
    bw_bits(w, 0, 1);
    bw_bits(w, 183, 8); /* level 6.1 */
}

static long finish_nal(bw_t *w, uint8_t *out, size_t cap) {
    if (w->err) { free(w->d); return -1; }
    if (cap < 2) { free(w->d); return -1; }
    out[0] = w->d[0];
    out[1] = w->d[1];
    size_t m = ep_insert(w->d + 2, w->n - 2, out + 2, cap - 2, NULL);
    free(w->d);
    if (m == (size_t)-1) return -1;
    return (long)(m + 2);
}

long synth_vps(const synth_params *P, uint8_t *out, size_t cap) {
    bw_t w = {0};
    nal_header(&w, 32);
    bw_bits(&w, 0, 4);
    bw_bits(&w, 1, 1);
    bw_bits(&w, 1, 1);
    bw_bits(&w, 0, 6);
    bw_bits(&w, 0, 3);
    bw_bits(&w, 1, 1);
    bw_bits(&w, 0xffff, 16);
    ptl(&w, P);
    bw_bits(&w, 1, 1);
    bw_ue(&w, 0);
    bw_ue(&w, 0);
    bw_ue(&w, 0);
    bw_bits(&w, 0, 6);
    bw_ue(&w, 0);
    bw_bits(&w, 0, 1);
    bw_bits(&w, 0, 1);
    bw_align1(&w);
    return finish_nal(&w, out, cap);
}

long synth_sps(const synth_params *P, uint8_t *out, size_t cap) {
    bw_t w = {0};
    nal_header(&w, 33);
    bw_bits(&w, 0, 4);
    bw_bits(&w, 0, 3);
    bw_bits(&w, 1, 1);
    ptl(&w, P);
    bw_ue(&w, 0);
    bw_ue(&w, (uint32_t)P->chroma_format);
    if (P->chroma_format == 3) bw_bits(&w, 0, 1); /* separate_colour_plane_flag */
    bw_ue(&w, (uint32_t)P->width);
    bw_ue(&w, (uint32_t)P->height);
    const int subw = (P->chroma_format == 1 || P->chroma_format == 2) ? 2 : 1, subh = P->chroma_format == 1 ? 2 : 1;
    if (P->conf_right || P->conf_bottom) {
        bw_bits(&w, 1, 1);
        bw_ue(&w, 0);
        bw_ue(&w, (uint32_t)(P->conf_right / subw));
        bw_ue(&w, 0);
        bw_ue(&w, (uint32_t)(P->conf_bottom / subh));
    } else {
        bw_bits(&w, 0, 1);
    }
    bw_ue(&w, (uint32_t)(P->bit_depth - 8));
    bw_ue(&w, (uint32_t)(P->bit_depth - 8));
    bw_ue(&w, 4);
    bw_bits(&w, 1, 1);
    bw_ue(&w, 0);
    bw_ue(&w, 0);
    bw_ue(&w, 0);
    bw_ue(&w, (uint32_t)(P->log2_min_cb - 3));
    bw_ue(&w, (uint32_t)(P->log2_ctb - P->log2_min_cb));
    bw_ue(&w, (uint32_t)(P->log2_min_tb - 2));
    bw_ue(&w, (uint32_t)(P->log2_max_tb - P->log2_min_tb));
    bw_ue(&w, 0);
    bw_ue(&w, (uint32_t)P->max_th_depth_intra);
    bw_bits(&w, P->scaling_list ? 1 : 0, 1);
    if (P->scaling_list) bw_bits(&w, 0, 1); /* default lists (Tables 7-5 / 7-6) */
    bw_bits(&w, 0, 1);                      /* amp */
    bw_bits(&w, P->sao ? 1 : 0, 1);
    bw_bits(&w, P->pcm ? 1 : 0, 1); /* pcm_enabled_flag */
    if (P->pcm) {
        bw_bits(&w, (uint32_t)(P->pcm_bd_y - 1), 4);
        bw_bits(&w, (uint32_t)(P->pcm_bd_c - 1), 4);
        bw_ue(&w, (uint32_t)(P->pcm_log2_min - 3));
        bw_ue(&w, (uint32_t)(P->pcm_log2_max - P->pcm_log2_min));
        bw_bits(&w, P->pcm_lf_disabled ? 1 : 0, 1);
    }
    bw_ue(&w, 0);
    bw_bits(&w, 0, 1);
    bw_bits(&w, 0, 1);
    bw_bits(&w, P->strong_intra ? 1 : 0, 1);
    bw_bits(&w, 0, 1); /* vui */
    bw_bits(&w, 0, 1); /* extensions */
    bw_align1(&w);
    return finish_nal(&w, out, cap);
}

long synth_pps(const synth_params *P, uint8_t *out, size_t cap) {
    bw_t w = {0};
    nal_header(&w, 34);
    bw_ue(&w, 0);
    bw_ue(&w, 0);
    bw_bits(&w, P->slice_dependent ? 1 : 0, 1); /* dependent_slice_segments_enabled_flag */
    bw_bits(&w, 0, 1);
    bw_bits(&w, 0, 3);
    bw_bits(&w, P->sign_hiding ? 1 : 0, 1);
    bw_bits(&w, 0, 1);
    bw_ue(&w, 0);
    bw_ue(&w, 0);
    bw_se(&w, P->init_qp - 26);
    bw_bits(&w, 0, 1);
    bw_bits(&w, P->transform_skip ? 1 : 0, 1);
    bw_bits(&w, P->cu_qp_delta ? 1 : 0, 1);
    if (P->cu_qp_delta) bw_ue(&w, (uint32_t)P->diff_cu_qp_delta_depth);
    bw_se(&w, P->cb_qp_offset);
    bw_se(&w, P->cr_qp_offset);
    bw_bits(&w, 0, 1);
    bw_bits(&w, 0, 1);
    bw_bits(&w, 0, 1);
    bw_bits(&w, P->tq_bypass ? 1 : 0, 1);
    bw_bits(&w, tiles_on(P) ? 1 : 0, 1); /* tiles_enabled_flag */
    bw_bits(&w, P->wpp ? 1 : 0, 1); /* entropy_coding_sync */
    if (tiles_on(P)) {
        bw_ue(&w, (uint32_t)(P->tile_cols - 1));
        bw_ue(&w, (uint32_t)(P->tile_rows - 1));
        bw_bits(&w, P->tile_uniform ? 1 : 0, 1);
        if (!P->tile_uniform) {
            for (int i = 0; i + 1 < P->tile_cols; i++) bw_ue(&w, (uint32_t)(P->tile_col_w[i] - 1));
            for (int i = 0; i + 1 < P->tile_rows; i++) bw_ue(&w, (uint32_t)(P->tile_row_h[i] - 1));
        }
        bw_bits(&w, P->tile_lf_across ? 1 : 0, 1);
    }
    bw_bits(&w, P->slice_lf_across ? 1 : 0, 1); /* pps_loop_filter_across_slices_enabled_flag */
    bw_bits(&w, 1, 1); /* deblocking control present */
    bw_bits(&w, P->slice_dbk_vary ? 1 : 0, 1); /* deblocking_filter_override_enabled_flag */
    bw_bits(&w, P->deblock_disabled ? 1 : 0, 1);
    if (!P->deblock_disabled) {
        bw_se(&w, P->beta_offset_div2);
        bw_se(&w, P->tc_offset_div2);
    }
    bw_bits(&w, 0, 1);
    bw_bits(&w, 0, 1);
    bw_ue(&w, 0);
    bw_bits(&w, 0, 1);
    bw_bits(&w, 0, 1);
    bw_align1(&w);
    return finish_nal(&w, out, cap);
}

int synth_check_params(const synth_params *P) {
    if (P->chroma_format < 0 || P->chroma_format > 3) return -1;
    if (P->bit_depth < 8 || P->bit_depth > 12) return -1;
    if (P->log2_min_cb < 3 || P->log2_ctb < 4 || P->log2_ctb > 6 || P->log2_min_cb > P->log2_ctb) return -1;
    if (P->log2_min_tb != 2 || P->log2_max_tb < P->log2_min_tb || P->log2_max_tb > 5 ||
        P->log2_max_tb > P->log2_ctb || P->log2_min_tb >= P->log2_min_cb)
        return -1;
    if (P->max_th_depth_intra < 0 || P->max_th_depth_intra > P->log2_ctb - P->log2_min_tb) return -1;
    if (P->width <= 0 || P->height <= 0 || (P->width & ((1 << P->log2_min_cb) - 1)) ||
        (P->height & ((1 << P->log2_min_cb) - 1)))
        return -1;
    if (P->diff_cu_qp_delta_depth < 0 || P->diff_cu_qp_delta_depth > P->log2_ctb - P->log2_min_cb) return -1;
    if (P->density < 0 || P->density > 100) return -1;
    if (P->wpp != 0 && P->wpp != 1) return -1;
    if (P->tile_cols < 0 || P->tile_rows < 0 || P->tile_cols > SYNTH_MAX_TILES || P->tile_rows > SYNTH_MAX_TILES)
        return -1;
    if (P->pcm && (P->pcm_bd_y < 1 || P->pcm_bd_y > P->bit_depth || P->pcm_bd_c < 1 || P->pcm_bd_c > P->bit_depth ||
                   P->pcm_log2_min < 3 || P->pcm_log2_min < P->log2_min_cb || P->pcm_log2_max > 5 ||
                   P->pcm_log2_max > P->log2_ctb || P->pcm_log2_max < P->pcm_log2_min || P->pcm_pct < 0 ||
                   P->pcm_pct > 100))
        return -1;
    if (P->slice_ctus < 0 || P->slice_dependent < 0 || P->slice_dependent > 2 || P->slice_lf_across < 0 ||
        P->slice_lf_across > 2)
        return -1;
    if (tiles_on(P)) {
        int ctb = 1 << P->log2_ctb, wctb = (P->width + ctb - 1) / ctb, hctb = (P->height + ctb - 1) / ctb;
        if (P->tile_cols < 1 || P->tile_rows < 1 || P->tile_cols > wctb || P->tile_rows > hctb) return -1;
        if (!P->tile_uniform) {
            int sw = 0, sh = 0;
            for (int i = 0; i + 1 < P->tile_cols; i++) { if (P->tile_col_w[i] < 1) return -1; sw += P->tile_col_w[i]; }
            for (int i = 0; i + 1 < P->tile_rows; i++) { if (P->tile_row_h[i] < 1) return -1; sh += P->tile_row_h[i]; }
            if (sw >= wctb || sh >= hctb) return -1;
        }
    }
    return 0;
}

/* one slice segment of the picture being written */
typedef struct {
    int ts0, first_sub, nsub, dependent;
    int qp_delta, sao_l, sao_c, dbk_override, dbk_disabled, beta, tc, lf_across;
} seg_t;

static int n_segments(const synth_params *P, int nctb) {
    return P->slice_ctus > 0 ? (nctb + P->slice_ctus - 1) / P->slice_ctus : 1;
}

/* Writes the picture's slice segments: item = 0 one NAL unit (a single
 * segment only), item = 1 every segment as a 4-byte-length-prefixed NAL unit
 * (the layout of a HEIF item). */
static long synth_impl(const synth_params *P, uint64_t seed, uint8_t *out, size_t cap, int item) {
    if (synth_check_params(P)) return -2;
    init_scans();
    pic_t pic;
    memset(&pic, 0, sizeof(pic));
    pic_t *p = &pic;
    p->P = P;
    p->rng = seed * 0x2545F4914F6CDD1Dull + 0x1234567ull;
    p->W = P->width;
    p->H = P->height;
    p->log2ctb = P->log2_ctb;
    p->ctb = 1 << P->log2_ctb;
    p->wctb = (p->W + p->ctb - 1) >> p->log2ctb;
    p->hctb = (p->H + p->ctb - 1) >> p->log2ctb;
    p->w4 = (p->W + 3) >> 2;
    p->h4 = (p->H + 3) >> 2;
    p->qpbdY = 6 * (P->bit_depth - 8);
    const int nctb = p->wctb * p->hctb, nseg = n_segments(P, nctb);
    if (!item && nseg > 1) return -2;
    const int seg_ctus = P->slice_ctus > 0 ? P->slice_ctus : nctb;
    p->ipm = (uint8_t *)calloc((size_t)p->w4 * p->h4, 1);
    p->depth = (uint8_t *)calloc((size_t)p->w4 * p->h4, 1);
    p->slice_rs = (int *)calloc((size_t)nctb, sizeof(int));
    bw_t *subs = (bw_t *)calloc((size_t)nctb + 1, sizeof(bw_t)); /* every substream holds a CTU at least */
    seg_t *segs = (seg_t *)calloc((size_t)nseg, sizeof(seg_t));
    if (!p->ipm || !p->depth || !p->slice_rs || !subs || !segs || tile_layout(p)) {
        free(p->ipm); free(p->depth); free(p->slice_rs); free(subs); free(segs); free(p->ts2rs); free(p->tile_rs);
        return -1;
    }
    int slice_qp = P->init_qp + P->slice_qp_delta;
    int sao_l = P->sao ? !pct(&p->rng, 10) : 0;
    int sao_c = (P->sao && P->chroma_format) ? !pct(&p->rng, 10) : 0;
    uint8_t wst[C_NUM], wmps[C_NUM], dst_[C_NUM], dmps[C_NUM];
    int saved = 0, nsub = 0, cur_slice = -1;
    seg_t *sg = NULL;
    ce_init_ctx(&p->c, slice_qp);
    /* CTUs in tile scan (7.3.8.1), cut into slice segments of slice_ctus CTUs.
     * A substream starts at a segment start, a WPP row start (9.3.1: contexts
     * after CTU 1 of the row above when the above-right CTB is available, else
     * initialised) or a tile start (initialised); a dependent segment starts
     * from the previous segment's final contexts.  Each substream but a
     * segment's last ends in end_of_subset_one_bit and byte_alignment();
     * without WPP or tiles a segment is one substream whose engine and
     * contexts run on across rows (slice.rs:206-231). */
    for (int ts = 0; ts < nctb; ts++) {
        const int rs = p->ts2rs[ts], rx = rs % p->wctb, ry = rs / p->wctb;
        const int tile_start = ts > 0 && p->tile_rs[rs] != p->tile_rs[p->ts2rs[ts - 1]];
        const int seg_start = ts % seg_ctus == 0;
        if (seg_start) {
            const int k = ts / seg_ctus;
            sg = &segs[k];
            sg->ts0 = ts;
            sg->first_sub = nsub;
            sg->dependent = k > 0 && (P->slice_dependent == 1 || (P->slice_dependent == 2 && (k & 1)));
            if (!sg->dependent) {
                ++cur_slice;
                if (k > 0) { /* a new slice: its own QP, SAO flags, deblocking and filter-across flags */
                    int q = P->init_qp + P->slice_qp_delta + (k * 7) % 5 - 2;
                    q = q < -p->qpbdY ? -p->qpbdY : q > 51 ? 51 : q;
                    slice_qp = q;
                    sao_l = P->sao ? !pct(&p->rng, 20) : 0;
                    sao_c = (P->sao && P->chroma_format) ? !pct(&p->rng, 20) : 0;
                }
                sg->qp_delta = slice_qp - P->init_qp;
                sg->sao_l = sao_l;
                sg->sao_c = sao_c;
                sg->dbk_disabled = P->deblock_disabled;
                sg->beta = P->beta_offset_div2;
                sg->tc = P->tc_offset_div2;
                if (P->slice_dbk_vary && k > 0) {
                    sg->dbk_override = 1;
                    sg->dbk_disabled = k % 3 == 2;
                    sg->beta = k % 3 - 1;
                    sg->tc = 1 - k % 3;
                }
                sg->lf_across = P->slice_lf_across == 1 || (P->slice_lf_across == 2 && !(cur_slice & 1));
            } else {
                *sg = segs[k - 1];
                sg->ts0 = ts;
                sg->first_sub = nsub;
                sg->nsub = 0;
                sg->dependent = 1;
            }
        }
        p->slice_rs[rs] = cur_slice;
        /* WPP: each CTB row of a tile is a substream (9.3.1: the CTB to its left is in another tile) */
        const int wpp_row = P->wpp && (rx == 0 || p->tile_rs[rs] != p->tile_rs[rs - 1]);
        if (seg_start || wpp_row || tile_start) {
            ce_start(&p->c, &subs[nsub]);
            sg->nsub++;
            if (ts == 0 || tile_start) {
                ce_init_ctx(&p->c, slice_qp);
            } else if (wpp_row) {
                /* T = the CTB above-right: in the picture, the same tile and the same slice */
                const int t_ok = saved && rx + 1 < p->wctb && p->slice_rs[rs - p->wctb + 1] == cur_slice &&
                                 p->tile_rs[rs - p->wctb + 1] == p->tile_rs[rs];
                if (t_ok) { memcpy(p->c.st, wst, C_NUM); memcpy(p->c.mps, wmps, C_NUM); }
                else ce_init_ctx(&p->c, slice_qp);
            } else if (sg->dependent && seg_start) {
                memcpy(p->c.st, dst_, C_NUM);
                memcpy(p->c.mps, dmps, C_NUM);
            } else {
                ce_init_ctx(&p->c, slice_qp);
            }
        }
        if (sao_l || sao_c) sao_syntax(p, rx, ry, sao_l, sao_c);
        coding_quadtree(p, rx << p->log2ctb, ry << p->log2ctb, p->log2ctb, 0);
        /* 9.3.2.2 storage: CtbAddrInRs % PicWidthInCtbs == 1, or its tile differs from CtbAddrInRs - 2's */
        if (P->wpp && (rs % p->wctb == 1 || (rs > 1 && p->tile_rs[rs] != p->tile_rs[rs - 2]))) {
            memcpy(wst, p->c.st, C_NUM);
            memcpy(wmps, p->c.mps, C_NUM);
            saved = 1;
        }
        const int seg_end = ts == nctb - 1 || (ts + 1) % seg_ctus == 0;
        ce_term(&p->c, seg_end); /* end_of_slice_segment_flag */
        if (seg_end || (P->wpp && p->ts2rs[ts + 1] / p->wctb != ry) || p->tile_rs[p->ts2rs[ts + 1]] != p->tile_rs[rs]) {
            if (!seg_end) ce_term(&p->c, 1); /* end_of_subset_one_bit */
            ce_finish(&p->c);
            bw_align1(&subs[nsub++]); /* byte_alignment() / rbsp_slice_segment_trailing_bits() */
            if (seg_end) { memcpy(dst_, p->c.st, C_NUM); memcpy(dmps, p->c.mps, C_NUM); } /* 9.3.2.4 */
        }
    }
    /* NAL units: slice header + the segment's substreams with emulation
     * prevention (the entry points are their sizes) */
    long ret = -1;
    size_t o = 0;
    int err = 0, addr_bits = 0;
    while ((1 << addr_bits) < nctb) addr_bits++;
    for (int r = 0; r < nsub; r++) err |= subs[r].err;
    for (int k = 0; k < nseg && !err; k++) {
        seg_t *g = &segs[k];
        size_t total = 0;
        for (int r = 0; r < g->nsub; r++) total += subs[g->first_sub + r].n;
        uint8_t *data = (uint8_t *)malloc(total * 3 / 2 + 16);
        size_t *sub_len = (size_t *)calloc((size_t)g->nsub, sizeof(size_t));
        if (!data || !sub_len) { free(data); free(sub_len); err = 1; break; }
        size_t dn = 0;
        int z = 0; /* the slice header ends in a nonzero byte (its alignment bit) */
        for (int r = 0; r < g->nsub; r++) {
            const bw_t *b = &subs[g->first_sub + r];
            size_t m = ep_insert(b->d, b->n, data + dn, total * 3 / 2 + 16 - dn, &z);
            sub_len[r] = m;
            dn += m;
        }
        bw_t w = {0};
        nal_header(&w, 19);
        bw_bits(&w, k == 0, 1); /* first_slice_segment_in_pic_flag */
        bw_bits(&w, 0, 1);      /* no_output_of_prior_pics_flag */
        bw_ue(&w, 0);
        if (k > 0) {
            if (P->slice_dependent) bw_bits(&w, (uint32_t)g->dependent, 1);
            bw_bits(&w, (uint32_t)p->ts2rs[g->ts0], addr_bits); /* slice_segment_address (raster) */
        }
        if (!g->dependent) {
            bw_ue(&w, 2); /* I slice */
            if (P->sao) {
                bw_bits(&w, (uint32_t)g->sao_l, 1);
                if (P->chroma_format) bw_bits(&w, (uint32_t)g->sao_c, 1);
            }
            bw_se(&w, g->qp_delta); /* slice_qp_delta: SliceQpY - (26 + init_qp_minus26) */
            if (P->slice_dbk_vary) {
                bw_bits(&w, (uint32_t)g->dbk_override, 1);
                if (g->dbk_override) {
                    bw_bits(&w, (uint32_t)g->dbk_disabled, 1);
                    if (!g->dbk_disabled) { bw_se(&w, g->beta); bw_se(&w, g->tc); }
                }
            }
            if (P->slice_lf_across && (g->sao_l || g->sao_c || !g->dbk_disabled))
                bw_bits(&w, (uint32_t)g->lf_across, 1);
        }
        if (P->wpp || tiles_on(P)) { /* num_entry_point_offsets: present only with tiles or WPP (7.3.6.1) */
            bw_ue(&w, (uint32_t)(g->nsub - 1));
            if (g->nsub > 1) {
                size_t mx = 1;
                for (int r = 0; r < g->nsub - 1; r++) mx = sub_len[r] > mx ? sub_len[r] : mx;
                int len = 1;
                while (((size_t)1 << len) < mx) len++;
                bw_ue(&w, (uint32_t)(len - 1));
                for (int r = 0; r < g->nsub - 1; r++) bw_bits(&w, (uint32_t)(sub_len[r] - 1), len);
            }
        }
        bw_align1(&w);
        if (w.err) err = 1;
        uint8_t *hdr = err ? NULL : (uint8_t *)malloc(w.n * 3 / 2 + 4);
        size_t hm = hdr ? ep_insert(w.d + 2, w.n - 2, hdr, w.n * 3 / 2 + 4, NULL) : (size_t)-1;
        if (hm == (size_t)-1) {
            err = 1;
        } else {
            const size_t nl = 2 + hm + dn, pre = item ? 4 : 0;
            if (o + pre + nl > cap) {
                ret = -3; /* capacity */
                err = 2;
            } else {
                if (item) {
                    out[o] = (uint8_t)(nl >> 24);
                    out[o + 1] = (uint8_t)(nl >> 16);
                    out[o + 2] = (uint8_t)(nl >> 8);
                    out[o + 3] = (uint8_t)nl;
                }
                out[o + pre] = w.d[0];
                out[o + pre + 1] = w.d[1];
                memcpy(out + o + pre + 2, hdr, hm);
                memcpy(out + o + pre + 2 + hm, data, dn);
                o += pre + nl;
            }
        }
        free(hdr);
        free(w.d);
        free(data);
        free(sub_len);
    }
    if (!err) ret = (long)o;
    for (int r = 0; r < nsub; r++) free(subs[r].d);
    free(subs);
    free(segs);
    free(p->ipm);
    free(p->depth);
    free(p->slice_rs);
    free(p->ts2rs);
    free(p->tile_rs);
    return ret;
}

long synth_picture(const synth_params *P, uint64_t seed, uint8_t *out, size_t cap) {
    return synth_impl(P, seed, out, cap, 0);
}

long synth_picture_item(const synth_params *P, uint64_t seed, uint8_t *out, size_t cap) {
    return synth_impl(P, seed, out, cap, 1);
}
