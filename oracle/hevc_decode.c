/*
 * hevc_decode.c — CPU oracle: HEVC intra-still decode (TEST INFRASTRUCTURE ONLY).
 *
 * Restates, single-threaded and spec-literally:
 *   - EP removal / RBSP bit reads:     src/hevc/rbsp_reader.rs:11-136
 *   - VPS/SPS/PPS parse:               src/hevc/parameter_set_reader.rs:7-551
 *                                       (+ scaling lists, st_ref_pic_set, HRD,
 *                                        range-extension flags: H.265 7.3.2.2,
 *                                        7.3.4, 7.3.7, E.2)
 *   - I-slice header:                  src/hevc/slice.rs:44-204 (+ POC/RPS for
 *                                       non-IDR, H.265 7.3.6.1)
 *   - CABAC engine + contexts:         src/cabac/arithmetic.rs:23-255,
 *                                       src/cabac/syntax_element.rs:90-242
 *   - binarizations:                   src/cabac/decoder.rs:152-284
 *   - slice-data CTU loop:             src/hevc/slice.rs:206-247, with WPP
 *                                       storage/sync (H.265 9.3.1, 9.3.2.4)
 *                                       and engine re-init (9.3.2.5)
 *   - everything the reference leaves todo!() (slice.rs:249-255), from
 *     H.265: SAO syntax 7.3.8.3, coding_quadtree/unit 7.3.8.4-5,
 *     transform_tree/unit 7.3.8.8-10, residual_coding 7.3.8.11, QP 8.6.1,
 *     scaling 8.6.2-3, transforms 8.6.4, intra 8.4.2-8.4.4, deblocking
 *     8.7.2, SAO 8.7.3.
 */
#include "oracle_internal.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static __thread char g_err[256];
/* bit0: skip deblocking, bit1: skip SAO (bring-up only); bit2: a picture may
 * end in end_of_slice_segment_flag 0 + end_of_subset_one_bit 1 — a tile cut
 * out of a tiled picture as a stand-alone picture (tests/hevc_tiles.py) */
static __thread int g_debug_flags;
void oracle_set_debug_flags(int flags) { g_debug_flags = flags; }
/* test coverage (debug flag 8): chroma TBs of 4:2:0 pictures by [log2 - 2][mode][cbf] */
static __thread uint32_t g_chroma_tb_hist[2][35][2];
void oracle_chroma_tb_hist(uint32_t *out, int reset) {
    memcpy(out, g_chroma_tb_hist, sizeof(g_chroma_tb_hist));
    if (reset) memset(g_chroma_tb_hist, 0, sizeof(g_chroma_tb_hist));
}
int oracle_fail(const char *msg) {
    snprintf(g_err, sizeof(g_err), "%s", msg);
    return -1;
}
const char *oracle_last_error(void) { return g_err; }

#define CLIP3(lo, hi, v) ((v) < (lo) ? (lo) : ((v) > (hi) ? (hi) : (v)))
static int imin(int a, int b) { return a < b ? a : b; }
static int iabs(int a) { return a < 0 ? -a : a; }

/* ===================================================================== */
/* EP removal — rbsp_reader.rs:11-39 (identical rule)                      */
/* ===================================================================== */
static size_t ep_remove(const uint8_t *in, size_t n, uint8_t *out, uint32_t *ep_pos, int *n_ep, int max_ep) {
    size_t i = 0, w = 0;
    int ne = 0;
    while (i < n) {
        size_t z = i;
        while (z < n && in[z] != 0) z++;
        if (z >= n) {
            memcpy(out + w, in + i, n - i);
            w += n - i;
            break;
        }
        memcpy(out + w, in + i, z - i);
        w += z - i;
        out[w++] = 0;
        if (z + 2 < n && in[z + 1] == 0 && in[z + 2] == 3 && (z + 3 >= n || in[z + 3] <= 3)) {
            out[w++] = 0;
            if (ep_pos && ne < max_ep) ep_pos[ne] = (uint32_t)(z + 2);
            ne++;
            i = z + 3;
        } else {
            i = z + 1;
        }
    }
    if (n_ep) *n_ep = ne;
    return w;
}

size_t oracle_remove_emulation_prevention(const uint8_t *in, size_t n, uint8_t *out) {
    return ep_remove(in, n, out, NULL, NULL, 0);
}

/* ===================================================================== */
/* Bit reader — rbsp_reader.rs:73-136                                     */
/* ===================================================================== */
typedef struct {
    const uint8_t *d;
    size_t n;
    size_t bit; /* absolute bit position */
    int err;
} br_t;

static uint32_t br_bit(br_t *b) {
    if ((b->bit >> 3) >= b->n) { b->err = 1; b->bit++; return 0; }
    uint32_t v = (b->d[b->bit >> 3] >> (7 - (b->bit & 7))) & 1;
    b->bit++;
    return v;
}
static uint32_t br_u(br_t *b, int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 1) | br_bit(b);
    return v;
}
static uint32_t br_ue(br_t *b) {
    int lz = 0;
    while (!br_bit(b)) {
        if (++lz > 31) { b->err = 1; return 0; }
    }
    if (lz == 0) return 0;
    return ((1u << lz) - 1) + br_u(b, lz);
}
static int32_t br_se(br_t *b) {
    uint32_t k = br_ue(b);
    if (k == 0) return 0;
    if (k & 1) return (int32_t)((k + 1) / 2);
    return -(int32_t)(k / 2);
}

int oracle_read_ue(const uint8_t *buf, size_t n, uint32_t *val) {
    br_t b = {buf, n, 0, 0};
    *val = br_ue(&b);
    return b.err ? -1 : 0;
}
int oracle_read_se(const uint8_t *buf, size_t n, int32_t *val) {
    br_t b = {buf, n, 0, 0};
    *val = br_se(&b);
    return b.err ? -1 : 0;
}

/* ===================================================================== */
/* Scan orders — H.265 6.5.3-6.5.5                                        */
/* ===================================================================== */
/* scan[log2blk 0..3][scanIdx 0..2][pos] = (x | y<<4) */
static uint8_t g_scan[4][3][64];
static int g_tables_ready = 0;
static void init_tables(void) {
    if (g_tables_ready) return;
    for (int l = 0; l < 4; l++) {
        int s = 1 << l;
        /* up-right diagonal */
        int i = 0, x = 0, y = 0;
        while (i < s * s) {
            while (y >= 0) {
                if (x < s && y < s) g_scan[l][0][i++] = (uint8_t)(x | (y << 4));
                y--;
                x++;
            }
            y = x;
            x = 0;
        }
        /* horizontal, vertical */
        for (int k = 0; k < s * s; k++) {
            g_scan[l][1][k] = (uint8_t)((k % s) | ((k / s) << 4));
            g_scan[l][2][k] = (uint8_t)((k / s) | ((k % s) << 4));
        }
    }
    g_tables_ready = 1;
}

/* Table 7-6 default 8x8 lists, raster (symmetric) */
static const uint8_t k_default_intra8[64] = {
    16, 16, 16, 16, 17, 18, 21, 24, 16, 16, 16, 16, 17, 19, 22, 25, 16, 16, 17, 18, 20, 22, 25, 29,
    16, 16, 18, 21, 24, 27, 31, 36, 17, 17, 20, 24, 30, 35, 41, 47, 18, 19, 22, 27, 35, 44, 54, 65,
    21, 22, 25, 31, 41, 54, 70, 88, 24, 25, 29, 36, 47, 65, 88, 115};
static const uint8_t k_default_inter8[64] = {
    16, 16, 16, 16, 17, 18, 20, 24, 16, 16, 16, 17, 18, 20, 24, 25, 16, 16, 17, 18, 20, 24, 25, 28,
    16, 17, 18, 20, 24, 25, 28, 33, 17, 18, 20, 24, 25, 28, 33, 41, 18, 20, 24, 25, 28, 33, 41, 54,
    20, 24, 25, 28, 33, 41, 54, 71, 24, 25, 28, 33, 41, 54, 71, 91};

static void default_list(int sizeId, int matrixId, uint8_t *out, int *dc) {
    init_tables();
    if (sizeId == 0) {
        for (int i = 0; i < 16; i++) out[i] = 16;
    } else {
        const uint8_t *m = matrixId < 3 ? k_default_intra8 : k_default_inter8;
        for (int i = 0; i < 64; i++) {
            int x = g_scan[3][0][i] & 15, y = g_scan[3][0][i] >> 4;
            out[i] = m[y * 8 + x];
        }
    }
    *dc = 16;
}

static void set_default_lists(uint8_t sl[4][6][64], int dc[4][6]) {
    for (int s = 0; s < 4; s++)
        for (int m = 0; m < 6; m++) default_list(s, m, sl[s][m], &dc[s][m]);
}

/* 7.3.4 scaling_list_data */
static int parse_scaling_list(br_t *b, uint8_t sl[4][6][64], int dc[4][6]) {
    for (int sizeId = 0; sizeId < 4; sizeId++) {
        int step = sizeId == 3 ? 3 : 1;
        for (int matrixId = 0; matrixId < 6; matrixId += step) {
            int pred_mode = (int)br_u(b, 1);
            int coefNum = imin(64, 1 << (4 + (sizeId << 1)));
            if (!pred_mode) {
                int delta = (int)br_ue(b);
                if (delta == 0) {
                    default_list(sizeId, matrixId, sl[sizeId][matrixId], &dc[sizeId][matrixId]);
                } else {
                    int ref = matrixId - delta * step;
                    if (ref < 0) return oracle_fail("bad scaling_list_pred_matrix_id_delta");
                    memcpy(sl[sizeId][matrixId], sl[sizeId][ref], 64);
                    dc[sizeId][matrixId] = dc[sizeId][ref];
                }
            } else {
                int next = 8;
                if (sizeId > 1) {
                    int d = br_se(b);
                    next = d + 8;
                    dc[sizeId][matrixId] = next;
                }
                for (int i = 0; i < coefNum; i++) {
                    int delta = br_se(b);
                    next = (next + delta + 256) % 256;
                    sl[sizeId][matrixId][i] = (uint8_t)next;
                }
                if (sizeId <= 1) dc[sizeId][matrixId] = 16;
            }
        }
    }
    /* 32x32 chroma (only used for 4:4:4): copy from 16x16 */
    for (int m = 1; m < 6; m++) {
        if (m == 3) continue;
        memcpy(sl[3][m], sl[2][m], 64);
        dc[3][m] = dc[2][m];
    }
    return b->err ? oracle_fail("scaling list overrun") : 0;
}

/* 7.3.3 profile_tier_level */
static void parse_ptl(br_t *b, int max_sub_layers_minus1) {
    br_u(b, 8);  /* profile_space, tier, profile_idc */
    br_u(b, 32); /* compat flags */
    br_u(b, 4);  /* progressive..frame_only */
    br_u(b, 32);
    br_u(b, 12); /* 43 + 1 bits total with above 32 → 44 */
    br_u(b, 8);  /* level */
    int spp[8] = {0}, slp[8] = {0};
    for (int i = 0; i < max_sub_layers_minus1; i++) {
        spp[i] = (int)br_u(b, 1);
        slp[i] = (int)br_u(b, 1);
    }
    if (max_sub_layers_minus1 > 0)
        for (int i = max_sub_layers_minus1; i < 8; i++) br_u(b, 2);
    for (int i = 0; i < max_sub_layers_minus1; i++) {
        if (spp[i]) { br_u(b, 32); br_u(b, 32); br_u(b, 24); }
        if (slp[i]) br_u(b, 8);
    }
}

/* E.2.3 sub_layer_hrd_parameters / E.2.2 hrd_parameters */
static void parse_sub_hrd(br_t *b, int cpb_cnt, int sub_pic) {
    for (int j = 0; j <= cpb_cnt; j++) {
        br_ue(b);
        br_ue(b);
        if (sub_pic) { br_ue(b); br_ue(b); }
        br_u(b, 1);
    }
}
static void parse_hrd(br_t *b, int common, int max_sub_layers_minus1) {
    int nal = 0, vcl = 0, sub_pic = 0;
    if (common) {
        nal = (int)br_u(b, 1);
        vcl = (int)br_u(b, 1);
        if (nal || vcl) {
            sub_pic = (int)br_u(b, 1);
            if (sub_pic) { br_u(b, 8); br_u(b, 5); br_u(b, 1); br_u(b, 5); }
            br_u(b, 4);
            br_u(b, 4);
            if (sub_pic) br_u(b, 4);
            br_u(b, 5); br_u(b, 5); br_u(b, 5);
        }
    }
    for (int i = 0; i <= max_sub_layers_minus1; i++) {
        int fixed_general = (int)br_u(b, 1);
        int fixed_cvs = 1;
        if (!fixed_general) fixed_cvs = (int)br_u(b, 1);
        int low_delay = 0;
        if (fixed_cvs) br_ue(b);
        else low_delay = (int)br_u(b, 1);
        int cpb_cnt = 0;
        if (!low_delay) cpb_cnt = (int)br_ue(b);
        if (nal) parse_sub_hrd(b, cpb_cnt, sub_pic);
        if (vcl) parse_sub_hrd(b, cpb_cnt, sub_pic);
    }
}

/* E.2.1 vui_parameters */
static void parse_vui(br_t *b, int max_sub_layers_minus1) {
    if (br_u(b, 1)) { if (br_u(b, 8) == 255) { br_u(b, 16); br_u(b, 16); } }
    if (br_u(b, 1)) br_u(b, 1);
    if (br_u(b, 1)) { br_u(b, 3); br_u(b, 1); if (br_u(b, 1)) { br_u(b, 8); br_u(b, 8); br_u(b, 8); } }
    if (br_u(b, 1)) { br_ue(b); br_ue(b); }
    br_u(b, 1); br_u(b, 1); br_u(b, 1);
    if (br_u(b, 1)) { br_ue(b); br_ue(b); br_ue(b); br_ue(b); }
    if (br_u(b, 1)) {
        br_u(b, 32); br_u(b, 32);
        if (br_u(b, 1)) br_ue(b);
        if (br_u(b, 1)) parse_hrd(b, 1, max_sub_layers_minus1);
    }
    if (br_u(b, 1)) { br_u(b, 1); br_u(b, 1); br_u(b, 1); br_ue(b); br_ue(b); br_ue(b); br_ue(b); br_ue(b); }
}

/* 7.3.7 st_ref_pic_set — only NumDeltaPocs is retained */
static int parse_st_rps(br_t *b, int idx, int num_sets, int *num_delta) {
    int inter = 0;
    if (idx != 0) inter = (int)br_u(b, 1);
    if (inter) {
        int delta_idx = 1;
        if (idx == num_sets) delta_idx = (int)br_ue(b) + 1;
        int ref = idx - delta_idx;
        if (ref < 0) return oracle_fail("bad st_rps ref");
        br_u(b, 1);
        br_ue(b);
        int cnt = 0;
        for (int j = 0; j <= num_delta[ref]; j++) {
            int used = (int)br_u(b, 1);
            int use_delta = 1;
            if (!used) use_delta = (int)br_u(b, 1);
            if (used || use_delta) cnt++;
        }
        num_delta[idx] = cnt;
    } else {
        int neg = (int)br_ue(b), pos = (int)br_ue(b);
        if (neg > 16 || pos > 16) return oracle_fail("bad st_rps");
        for (int i = 0; i < neg; i++) { br_ue(b); br_u(b, 1); }
        for (int i = 0; i < pos; i++) { br_ue(b); br_u(b, 1); }
        num_delta[idx] = neg + pos;
    }
    return 0;
}

/* 7.3.2.2 seq_parameter_set_rbsp — parameter_set_reader.rs:36-201 */
static int parse_sps(const uint8_t *rbsp, size_t n, hevc_sps *s) {
    br_t b = {rbsp, n, 0, 0};
    memset(s, 0, sizeof(*s));
    br_u(&b, 4);
    int msl = (int)br_u(&b, 3);
    br_u(&b, 1);
    parse_ptl(&b, msl);
    br_ue(&b); /* sps id */
    s->chroma_format_idc = (int)br_ue(&b);
    if (s->chroma_format_idc == 3) s->separate_colour_plane = (int)br_u(&b, 1);
    s->width = (int)br_ue(&b);
    s->height = (int)br_ue(&b);
    int sw = (s->chroma_format_idc == 1 || s->chroma_format_idc == 2) ? 2 : 1;
    int sh = s->chroma_format_idc == 1 ? 2 : 1;
    if (br_u(&b, 1)) {
        s->conf_l = (int)br_ue(&b) * sw;
        s->conf_r = (int)br_ue(&b) * sw;
        s->conf_t = (int)br_ue(&b) * sh;
        s->conf_b = (int)br_ue(&b) * sh;
    }
    s->out_w = s->width - s->conf_l - s->conf_r;
    s->out_h = s->height - s->conf_t - s->conf_b;
    s->bit_depth_y = (int)br_ue(&b) + 8;
    s->bit_depth_c = (int)br_ue(&b) + 8;
    s->log2_max_poc_lsb = (int)br_ue(&b) + 4;
    int ordering = (int)br_u(&b, 1);
    for (int i = ordering ? 0 : msl; i <= msl; i++) { br_ue(&b); br_ue(&b); br_ue(&b); }
    s->log2_min_cb = (int)br_ue(&b) + 3;
    s->log2_ctb = s->log2_min_cb + (int)br_ue(&b);
    s->log2_min_tb = (int)br_ue(&b) + 2;
    s->log2_max_tb = s->log2_min_tb + (int)br_ue(&b);
    s->max_th_depth_inter = (int)br_ue(&b);
    s->max_th_depth_intra = (int)br_ue(&b);
    s->scaling_list_enabled = (int)br_u(&b, 1);
    set_default_lists(s->sl, s->sl_dc);
    if (s->scaling_list_enabled) {
        if (br_u(&b, 1))
            if (parse_scaling_list(&b, s->sl, s->sl_dc)) return -1;
    }
    s->amp = (int)br_u(&b, 1);
    s->sao = (int)br_u(&b, 1);
    s->pcm = (int)br_u(&b, 1);
    if (s->pcm) {
        s->pcm_bd_y = (int)br_u(&b, 4) + 1;
        s->pcm_bd_c = (int)br_u(&b, 4) + 1;
        s->log2_min_pcm = (int)br_ue(&b) + 3;
        s->log2_max_pcm = s->log2_min_pcm + (int)br_ue(&b);
        s->pcm_loop_filter_disabled = (int)br_u(&b, 1);
    }
    s->num_st_rps = (int)br_ue(&b);
    if (s->num_st_rps > 64) return oracle_fail("too many st_rps");
    for (int i = 0; i < s->num_st_rps; i++)
        if (parse_st_rps(&b, i, s->num_st_rps, s->st_rps_num_delta)) return -1;
    s->long_term_refs_present = (int)br_u(&b, 1);
    if (s->long_term_refs_present) {
        s->num_lt_sps = (int)br_ue(&b);
        for (int i = 0; i < s->num_lt_sps; i++) { br_u(&b, s->log2_max_poc_lsb); br_u(&b, 1); }
    }
    s->temporal_mvp = (int)br_u(&b, 1);
    s->strong_intra_smoothing = (int)br_u(&b, 1);
    if (br_u(&b, 1)) parse_vui(&b, msl);
    if (br_u(&b, 1)) {
        int range = (int)br_u(&b, 1);
        br_u(&b, 1); br_u(&b, 1); br_u(&b, 1);
        br_u(&b, 4);
        if (range) {
            /* 7.3.2.2.2: nine flags; any set ⇒ unsupported here */
            s->range_ext_any = (int)br_u(&b, 9);
        }
    }
    if (b.err) return oracle_fail("SPS overrun");
    return 0;
}

/* 7.3.2.3 pic_parameter_set_rbsp — parameter_set_reader.rs:351-491 */
static int parse_pps(const uint8_t *rbsp, size_t n, const hevc_sps *sps, hevc_pps *p) {
    br_t b = {rbsp, n, 0, 0};
    memset(p, 0, sizeof(*p));
    br_ue(&b);
    br_ue(&b);
    p->dependent_slices = (int)br_u(&b, 1);
    p->output_flag_present = (int)br_u(&b, 1);
    p->num_extra_bits = (int)br_u(&b, 3);
    p->sign_hiding = (int)br_u(&b, 1);
    p->cabac_init_present = (int)br_u(&b, 1);
    br_ue(&b);
    br_ue(&b);
    p->init_qp = 26 + br_se(&b);
    p->constrained_intra = (int)br_u(&b, 1);
    p->transform_skip = (int)br_u(&b, 1);
    p->cu_qp_delta = (int)br_u(&b, 1);
    if (p->cu_qp_delta) p->diff_cu_qp_delta_depth = (int)br_ue(&b);
    p->cb_qp_offset = br_se(&b);
    p->cr_qp_offset = br_se(&b);
    p->slice_chroma_qp_offsets_present = (int)br_u(&b, 1);
    br_u(&b, 1);
    br_u(&b, 1);
    p->transquant_bypass = (int)br_u(&b, 1);
    p->tiles = (int)br_u(&b, 1);
    p->wpp = (int)br_u(&b, 1);
    p->tile_cols = p->tile_rows = p->tile_uniform = 1;
    p->lf_across_tiles = 1;
    if (p->tiles) {
        /* num_tile_columns/rows_minus1, uniform_spacing_flag, column_width /
         * row_height_minus1[], loop_filter_across_tiles_enabled_flag
         * (parameter_set_reader.rs:380-408) */
        uint32_t nc = br_ue(&b) + 1, nr = br_ue(&b) + 1;
        if (nc > HEVC_MAX_TILE_DIM || nr > HEVC_MAX_TILE_DIM || nc * nr < 2) return oracle_fail("tile count");
        p->tile_cols = (int)nc;
        p->tile_rows = (int)nr;
        p->tile_uniform = (int)br_u(&b, 1);
        if (!p->tile_uniform) {
            for (int i = 0; i + 1 < p->tile_cols; i++) p->tile_col_w[i] = (int)br_ue(&b) + 1;
            for (int i = 0; i + 1 < p->tile_rows; i++) p->tile_row_h[i] = (int)br_ue(&b) + 1;
        }
        p->lf_across_tiles = (int)br_u(&b, 1);
    }
    p->loop_filter_across_slices = (int)br_u(&b, 1);
    if (br_u(&b, 1)) {
        p->deblock_override_enabled = (int)br_u(&b, 1);
        p->deblock_disabled = (int)br_u(&b, 1);
        if (!p->deblock_disabled) {
            p->beta_offset_div2 = br_se(&b);
            p->tc_offset_div2 = br_se(&b);
        }
    }
    p->scaling_list_present = (int)br_u(&b, 1);
    memcpy(p->sl, sps->sl, sizeof(p->sl));
    memcpy(p->sl_dc, sps->sl_dc, sizeof(p->sl_dc));
    if (p->scaling_list_present) {
        set_default_lists(p->sl, p->sl_dc);
        if (parse_scaling_list(&b, p->sl, p->sl_dc)) return -1;
    }
    p->lists_mod = (int)br_u(&b, 1);
    p->log2_parallel_merge = (int)br_ue(&b) + 2;
    p->slice_header_ext = (int)br_u(&b, 1);
    if (br_u(&b, 1)) {
        int range = (int)br_u(&b, 1);
        br_u(&b, 1); br_u(&b, 1); br_u(&b, 1);
        br_u(&b, 4);
        if (range) {
            if (p->transform_skip) { if (br_ue(&b) != 0) p->range_ext_any = 1; }
            if (br_u(&b, 1)) p->range_ext_any = 1;
            if (br_u(&b, 1)) p->range_ext_any = 1;
            if (br_ue(&b)) p->range_ext_any = 1;
            if (br_ue(&b)) p->range_ext_any = 1;
        }
    }
    if (b.err) return oracle_fail("PPS overrun");
    return 0;
}

/* hvcC → VPS/SPS/PPS (heif/reader.rs:570-630, heic/decoder.rs:24-71) */
int hevc_parse_hvcc(const uint8_t *p, size_t n, hevc_ps *ps) {
    if (n < 23) return oracle_fail("short hvcC");
    size_t pos = 22;
    int narr = p[pos++];
    const uint8_t *sps = NULL, *pps = NULL;
    size_t sps_n = 0, pps_n = 0;
    for (int a = 0; a < narr; a++) {
        if (pos + 3 > n) return oracle_fail("hvcC overrun");
        int type = p[pos] & 0x3f;
        int cnt = (p[pos + 1] << 8) | p[pos + 2];
        pos += 3;
        for (int k = 0; k < cnt; k++) {
            if (pos + 2 > n) return oracle_fail("hvcC overrun");
            size_t len = ((size_t)p[pos] << 8) | p[pos + 1];
            pos += 2;
            if (pos + len > n) return oracle_fail("hvcC overrun");
            if (type == 33 && !sps) { sps = p + pos; sps_n = len; }
            if (type == 34 && !pps) { pps = p + pos; pps_n = len; }
            pos += len;
        }
    }
    if (!sps || !pps || sps_n < 3 || pps_n < 3) return oracle_fail("missing SPS/PPS");
    uint8_t *buf = (uint8_t *)malloc(sps_n + pps_n);
    size_t m = ep_remove(sps + 2, sps_n - 2, buf, NULL, NULL, 0);
    int r = parse_sps(buf, m, &ps->sps);
    if (!r) {
        m = ep_remove(pps + 2, pps_n - 2, buf, NULL, NULL, 0);
        r = parse_pps(buf, m, &ps->sps, &ps->pps);
    }
    free(buf);
    return r;
}

/* ===================================================================== */
/* CABAC — arithmetic.rs:23-174, syntax_element.rs:90-242                 */
/* ===================================================================== */
enum {
    CTX_SAO_MERGE = 0, CTX_SAO_TYPE = 1, CTX_SPLIT_CU = 2, CTX_TQ_BYPASS = 5, CTX_PART_MODE = 6,
    CTX_PREV_INTRA = 7, CTX_CHROMA_MODE = 8, CTX_SPLIT_TF = 9, CTX_CBF_LUMA = 12, CTX_CBF_CHROMA = 14,
    CTX_CU_QP_DELTA = 19, CTX_TS_FLAG = 21, CTX_LAST_X = 23, CTX_LAST_Y = 41, CTX_CSBF = 59,
    CTX_SIG = 63, CTX_GT1 = 107, CTX_GT2 = 131, CTX_NUM = 137
};
static const uint8_t k_init_i[CTX_NUM] = {
    153,                                                                   /* sao_merge */
    200,                                                                   /* sao_type */
    139, 141, 157,                                                         /* split_cu */
    154,                                                                   /* tq_bypass */
    184,                                                                   /* part_mode */
    184,                                                                   /* prev_intra */
    63,                                                                    /* chroma mode */
    153, 138, 138,                                                         /* split_tf */
    111, 141,                                                              /* cbf_luma */
    94, 138, 182, 154, 154,                                                /* cbf_chroma */
    154, 154,                                                              /* cu_qp_delta */
    139, 139,                                                              /* transform_skip */
    110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63, /* last_x */
    110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63, /* last_y */
    91, 171, 134, 141,                                                     /* csbf */
    111, 111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107, 125, 141,
    179, 153, 125, 107, 125, 141, 179, 153, 125, 140, 139, 182, 182, 152, 136, 152, 136, 153,
    136, 139, 111, 136, 139, 111, 141, 111,                                /* sig (42 + 2) */
    140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152, 140, 179, 166,
    182, 140, 227, 122, 197,                                               /* gt1 */
    138, 153, 136, 167, 152, 152,                                          /* gt2 */
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

typedef struct {
    br_t b;           /* over the slice RBSP */
    uint32_t range, offset;
    uint8_t st[CTX_NUM];  /* pStateIdx */
    uint8_t mps[CTX_NUM]; /* valMps */
    uint32_t bins;
} cabac_t;

/* 9.3.2.2 context init — arithmetic.rs:51-78 */
static void cabac_init_ctx(cabac_t *c, int qp) {
    int q = CLIP3(0, 51, qp);
    for (int i = 0; i < CTX_NUM; i++) {
        int v = k_init_i[i];
        int m = (v >> 4) * 5 - 45, nn = ((v & 15) << 3) - 16;
        int pre = CLIP3(1, 126, ((m * q) >> 4) + nn);
        c->mps[i] = pre > 63;
        c->st[i] = (uint8_t)(c->mps[i] ? pre - 64 : 63 - pre);
    }
}
/* 9.3.2.5 — arithmetic.rs:23-38 */
static int cabac_init_engine(cabac_t *c) {
    c->range = 510;
    c->offset = br_u(&c->b, 9);
    if (c->offset >= 510) return oracle_fail("ivlOffset 510/511");
    return 0;
}
/* 9.3.4.3.2 — arithmetic.rs:97-144 */
static int dec_bin(cabac_t *c, int ci) {
    c->bins++;
    uint32_t s = c->st[ci];
    uint32_t lps = k_lps[s][(c->range >> 6) & 3];
    int bin;
    c->range -= lps;
    if (c->offset >= c->range) {
        bin = !c->mps[ci];
        c->offset -= c->range;
        c->range = lps;
        if (s == 0) c->mps[ci] = (uint8_t)(1 - c->mps[ci]);
        c->st[ci] = k_trans_lps[s];
    } else {
        bin = c->mps[ci];
        c->st[ci] = (uint8_t)(s < 62 ? s + 1 : s);
    }
    while (c->range < 256) {
        c->range <<= 1;
        c->offset = (c->offset << 1) | br_bit(&c->b);
    }
    return bin;
}
/* 9.3.4.3.4 — arithmetic.rs:146-157 */
static int dec_bypass(cabac_t *c) {
    c->bins++;
    c->offset = (c->offset << 1) | br_bit(&c->b);
    if (c->offset >= c->range) { c->offset -= c->range; return 1; }
    return 0;
}
/* 9.3.4.3.5 — arithmetic.rs:159-169 */
static int dec_term(cabac_t *c) {
    c->bins++;
    c->range -= 2;
    if (c->offset >= c->range) return 1;
    while (c->range < 256) {
        c->range <<= 1;
        c->offset = (c->offset << 1) | br_bit(&c->b);
    }
    return 0;
}

/* ---- binarizations over an abstract bin source (decoder.rs:152-261) ---- */
typedef int (*binsrc_fn)(void *ctx);
static int bz_fl(binsrc_fn f, void *ctx, int nbits) {
    int v = 0;
    for (int i = 0; i < nbits; i++) v = (v << 1) | f(ctx);
    return v;
}
static int bz_tr(binsrc_fn f, void *ctx, int cmax, int crice) {
    int pmax = cmax >> crice, p = 0;
    while (p < pmax && f(ctx)) p++;
    int suf = 0;
    if (crice > 0 && p < pmax) suf = bz_fl(f, ctx, crice);
    return (p << crice) + suf;
}
static int bz_egk(binsrc_fn f, void *ctx, int k) {
    int ones = 0;
    while (f(ctx)) {
        if (++ones > 31) return -1;
    }
    int v = ((1 << ones) - 1) << k;
    return v + bz_fl(f, ctx, ones + k);
}
/* coeff_abs_level_remaining prefix TR(cMax=4<<k, k) + EG(k+1) suffix */
static int bz_calr(binsrc_fn f, void *ctx, int k) {
    int cmax = 4 << k;
    int pre = bz_tr(f, ctx, cmax, k);
    if (pre == cmax) {
        int s = bz_egk(f, ctx, k + 1);
        if (s < 0) return -1;
        return cmax + s;
    }
    return pre;
}
static int bypass_src(void *ctx) { return dec_bypass((cabac_t *)ctx); }

typedef struct { const uint8_t *b; int n, i, under; } vecsrc;
static int vec_src(void *ctx) {
    vecsrc *v = (vecsrc *)ctx;
    if (v->i >= v->n) { v->under = 1; return 0; }
    return v->b[v->i++] ? 1 : 0;
}
int oracle_decode_tr_bins(const uint8_t *bins, int nbins, int c_max, int c_rice, int *used) {
    vecsrc v = {bins, nbins, 0, 0};
    int r = bz_tr(vec_src, &v, c_max, c_rice);
    *used = v.i;
    return v.under ? -1 : r;
}
int oracle_decode_chroma_mode_bins(const uint8_t *bins, int nbins, int *used) {
    vecsrc v = {bins, nbins, 0, 0};
    int r = vec_src(&v) ? bz_fl(vec_src, &v, 2) : 4;
    *used = v.i;
    return v.under ? -1 : r;
}
int oracle_decode_coeff_abs_level_remaining_bins(const uint8_t *bins, int nbins, int c_rice, int *used) {
    vecsrc v = {bins, nbins, 0, 0};
    int r = bz_calr(vec_src, &v, c_rice);
    *used = v.i;
    return v.under ? -1 : r;
}

/* ===================================================================== */
/* Picture decode state                                                   */
/* ===================================================================== */
typedef struct {
    int type[3], band[3], eo[3];
    int off[3][5];
} sao_ctb;

/* per-slice values the loop filters need after parsing (7.4.7.1) */
typedef struct {
    int qp, sao_l, sao_c, dbk_disabled, beta, tc, cb_off, cr_off, lf_across;
    int addr_rs; /* SliceAddrRs */
} slice_par;

typedef struct {
    const hevc_sps *sps;
    const hevc_pps *pps;
    /* the slice being parsed */
    int slice_qp, sao_luma, sao_chroma, dbk_disabled, beta_off, tc_off, cb_qp_off, cr_qp_off;
    /* geometry */
    int W, H, log2ctb, ctb, wctb, hctb, minTb, minCb;
    int chroma, sw, sh, cw, chh;
    int bdY, bdC, qpbdY, qpbdC;
    uint16_t *pl[3];
    int ps[3];
    int w4, h4;
    uint8_t *ipm, *depth, *flg;
    int8_t *qpy;
    sao_ctb *sao;
    /* ScalingFactor m[sizeId][matrixId][y*n+x] */
    uint8_t *sf[4][6];
    cabac_t c;
    uint8_t wpp_st[CTX_NUM], wpp_mps[CTX_NUM];
    int wpp_saved;
    /* QP state */
    int cu_qp_delta_val, is_cu_qp_delta_coded, qg_new, qg_x, qg_y, qp_prev_last, qp_pred, qpy_cur;
    int ctb_x, ctb_y, first_qg_in_ctb_row_pending, first_qg_in_slice;
    /* 6.5.1 tiles: column / row boundaries in CTBs, CtbAddrRsToTs / TsToRs and
     * the tile of each CTB by raster address (one tile when tiles is 0) */
    int colBd[HEVC_MAX_TILE_DIM + 1], rowBd[HEVC_MAX_TILE_DIM + 1];
    int *rs2ts, *ts2rs, *tile_rs;
    /* slices: index of the slice holding each CTB (raster address), their values */
    int *slice_rs;
    slice_par *slices;
    uint8_t ds_st[CTX_NUM], ds_mps[CTX_NUM]; /* 9.3.2.4 storage at a slice segment's end */
    /* current CU */
    int cu_bypass, cu_intra_split, cu_max_trafo_depth;
    int cu_x, cu_y, cu_pb;        /* the CU and its prediction block size */
    int cu_chroma_mode_c[4];      /* IntraPredModeC per PB (4:4:4 NxN: four; else PB 0) */
} pic_t;

#define F_EDGE_V 1
#define F_EDGE_H 2
#define F_NOFILT 4

static int zscan_addr(const pic_t *p, int x, int y) {
    /* MinTbAddrZs (6-10) for luma sample (x,y): CtbAddrRsToTs of its CTB, then
     * the z-order inside the CTB */
    int tbx = x >> p->minTb, tby = y >> p->minTb;
    int sh = p->log2ctb - p->minTb;
    int ctbAddr = p->rs2ts[(tbx >> sh) + (tby >> sh) * p->wctb];
    int v = ctbAddr << (sh * 2);
    for (int i = 0; i < sh; i++) {
        int m = 1 << i;
        v += (m & tbx ? m * m : 0) + (m & tby ? 2 * m * m : 0);
    }
    return v;
}
/* tile of the CTB holding luma sample (x,y) (TileId by raster CTB address) */
static int tile_at(const pic_t *p, int x, int y) {
    return p->tile_rs[(y >> p->log2ctb) * p->wctb + (x >> p->log2ctb)];
}
/* slice of the CTB holding luma sample (x,y) (-1: not decoded yet) */
static int slice_at(const pic_t *p, int x, int y) {
    return p->slice_rs[(y >> p->log2ctb) * p->wctb + (x >> p->log2ctb)];
}
/* 6.4.1 z-scan availability: outside the picture, later in decoding order,
 * in another tile or in another slice ⇒ unavailable */
static int avail_zs(const pic_t *p, int xc, int yc, int xn, int yn) {
    if (xn < 0 || yn < 0 || xn >= p->W || yn >= p->H) return 0;
    if (tile_at(p, xn, yn) != tile_at(p, xc, yc)) return 0;
    if (zscan_addr(p, xn, yn) > zscan_addr(p, xc, yc)) return 0;
    return slice_at(p, xn, yn) == slice_at(p, xc, yc);
}

/* 6.5.1 (6-3..6-10): colBd / rowBd, CtbAddrRsToTs, CtbAddrTsToRs, TileId */
static int tile_scan_init(pic_t *p) {
    const hevc_pps *pp = p->pps;
    int nc = pp->tiles ? pp->tile_cols : 1, nr = pp->tiles ? pp->tile_rows : 1;
    int colW[HEVC_MAX_TILE_DIM], rowH[HEVC_MAX_TILE_DIM];
    for (int pass = 0; pass < 2; pass++) {
        int n = pass ? nr : nc, tot = pass ? p->hctb : p->wctb, *sz = pass ? rowH : colW;
        const int *ex = pass ? pp->tile_row_h : pp->tile_col_w;
        int used = 0;
        for (int i = 0; i < n; i++) {
            if (!pp->tiles || pp->tile_uniform) sz[i] = ((i + 1) * tot) / n - (i * tot) / n;
            else sz[i] = i + 1 < n ? ex[i] : tot - used;
            if (sz[i] <= 0) return oracle_fail("tile sizes exceed the picture");
            used += sz[i];
        }
        int *bd = pass ? p->rowBd : p->colBd;
        bd[0] = 0;
        for (int i = 0; i < n; i++) bd[i + 1] = bd[i] + sz[i];
    }
    int nctb = p->wctb * p->hctb;
    p->rs2ts = (int *)malloc(sizeof(int) * (size_t)nctb);
    p->ts2rs = (int *)malloc(sizeof(int) * (size_t)nctb);
    p->tile_rs = (int *)malloc(sizeof(int) * (size_t)nctb);
    for (int rs = 0; rs < nctb; rs++) {
        int tbX = rs % p->wctb, tbY = rs / p->wctb, tx = 0, ty = 0;
        for (int i = 0; i < nc; i++)
            if (tbX >= p->colBd[i]) tx = i;
        for (int j = 0; j < nr; j++)
            if (tbY >= p->rowBd[j]) ty = j;
        int v = 0;
        for (int i = 0; i < tx; i++) v += rowH[ty] * colW[i];
        for (int j = 0; j < ty; j++) v += p->wctb * rowH[j];
        v += (tbY - p->rowBd[ty]) * colW[tx] + tbX - p->colBd[tx];
        p->rs2ts[rs] = v;
        p->ts2rs[v] = rs;
        p->tile_rs[rs] = ty * nc + tx;
    }
    return 0;
}

static void build_scaling(pic_t *p) {
    const hevc_pps *pp = p->pps;
    for (int s = 0; s < 4; s++) {
        int n = 4 << s;
        for (int m = 0; m < 6; m++) {
            uint8_t *f = (uint8_t *)malloc((size_t)n * n);
            p->sf[s][m] = f;
            if (s == 0) {
                for (int i = 0; i < 16; i++) {
                    int x = g_scan[2][0][i] & 15, y = g_scan[2][0][i] >> 4;
                    f[y * 4 + x] = pp->sl[0][m][i];
                }
            } else {
                int rep = n / 8;
                for (int i = 0; i < 64; i++) {
                    int x = g_scan[3][0][i] & 15, y = g_scan[3][0][i] >> 4;
                    for (int j = 0; j < rep; j++)
                        for (int k = 0; k < rep; k++) f[(y * rep + j) * n + x * rep + k] = pp->sl[s][m][i];
                }
                if (s >= 2) f[0] = (uint8_t)pp->sl_dc[s][m];
            }
        }
    }
}

/* ---- maps ---- */
static void set_map(pic_t *p, uint8_t *map, int x0, int y0, int size, uint8_t v) {
    for (int y = y0 >> 2; y < (y0 + size) >> 2 && y < p->h4; y++)
        for (int x = x0 >> 2; x < (x0 + size) >> 2 && x < p->w4; x++) map[y * p->w4 + x] = v;
}

/* ===================================================================== */
/* Intra sample prediction — H.265 8.4.4.2                                */
/* ===================================================================== */
static const int k_angle[35] = {0, 0, 32, 26, 21, 17, 13, 9, 5, 2, 0, -2, -5, -9, -13, -17, -21, -26,
                                -32, -26, -21, -17, -13, -9, -5, -2, 0, 2, 5, 9, 13, 17, 21, 26, 32};
static const int k_inv_angle[35] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, -4096, -1638, -910, -630, -482, -390, -315,
                                    -256, -315, -390, -482, -630, -910, -1638, -4096, 0, 0, 0, 0, 0, 0, 0, 0, 0};

static void intra_predict(pic_t *p, int cIdx, int xTb, int yTb, int log2n, int mode) {
    int n = 1 << log2n;
    int sw = cIdx ? p->sw : 1, sh = cIdx ? p->sh : 1;
    int bd = cIdx ? p->bdC : p->bdY;
    uint16_t *pl = p->pl[cIdx];
    int ps = p->ps[cIdx];
    int PW = cIdx ? p->cw : p->W, PH = cIdx ? p->chh : p->H;
    /* ref arrays: left[0] = p[-1][-1], left[1+y] = p[-1][y]; top[1+x] = p[x][-1] */
    int left[129], top[129], av_l[129], av_t[129];
    left[0] = top[0] = 0;
    int xc = xTb * sw, yc = yTb * sh;
    int any = 0;
    for (int i = -1; i < 2 * n; i++) {
        /* left column p[-1][i] */
        int xn = xTb - 1, yn = yTb + i;
        int a = xn >= 0 && yn >= 0 && xn < PW && yn < PH && avail_zs(p, xc, yc, xn * sw, yn * sh);
        av_l[i + 1] = a;
        left[i + 1] = a ? pl[yn * ps + xn] : 0;
        any |= a;
    }
    for (int i = 0; i < 2 * n; i++) {
        int xn = xTb + i, yn = yTb - 1;
        int a = xn >= 0 && yn >= 0 && xn < PW && yn < PH && avail_zs(p, xc, yc, xn * sw, yn * sh);
        av_t[i + 1] = a;
        top[i + 1] = a ? pl[yn * ps + xn] : 0;
        any |= a;
    }
    /* 8.4.4.2.2 substitution */
    if (!any) {
        for (int i = 0; i <= 2 * n; i++) left[i] = top[i] = 1 << (bd - 1);
    } else {
        /* search order: p[-1][2n-1] ... p[-1][-1], p[0][-1] ... p[2n-1][-1] */
        if (!av_l[2 * n]) {
            int v = 0, found = 0;
            for (int i = 2 * n - 1; i >= 0 && !found; i--)
                if (av_l[i]) { v = left[i]; found = 1; }
            for (int i = 1; i <= 2 * n && !found; i++)
                if (av_t[i]) { v = top[i]; found = 1; }
            left[2 * n] = v;
            av_l[2 * n] = 1;
        }
        for (int i = 2 * n - 1; i >= 0; i--)
            if (!av_l[i]) left[i] = left[i + 1];
        top[0] = left[0];
        for (int i = 1; i <= 2 * n; i++)
            if (!av_t[i]) top[i] = top[i - 1];
    }
    top[0] = left[0];
    /* 8.4.4.2.3 filtering (cIdx == 0 or 4:4:4) */
    if (cIdx == 0 || p->chroma == 3) {
        int filter = 0;
        if (mode != 1 && n != 4) {
            int d = imin(iabs(mode - 26), iabs(mode - 10));
            int thr = n == 8 ? 7 : (n == 16 ? 1 : 0);
            filter = d > thr;
        }
        if (filter) {
            int fl[129], ft[129];
            int bi = p->sps->strong_intra_smoothing && cIdx == 0 && n == 32 &&
                     iabs(left[0] + top[2 * n] - 2 * top[n]) < (1 << (bd - 5)) &&
                     iabs(left[0] + left[2 * n] - 2 * left[n]) < (1 << (bd - 5));
            if (bi) {
                fl[0] = ft[0] = left[0];
                for (int i = 0; i < 63; i++) {
                    fl[i + 1] = ((63 - i) * left[0] + (i + 1) * left[64] + 32) >> 6;
                    ft[i + 1] = ((63 - i) * top[0] + (i + 1) * top[64] + 32) >> 6;
                }
                fl[64] = left[64];
                ft[64] = top[64];
            } else {
                fl[0] = ft[0] = (left[1] + 2 * left[0] + top[1] + 2) >> 2;
                for (int i = 1; i < 2 * n; i++) {
                    fl[i] = (left[i + 1] + 2 * left[i] + left[i - 1] + 2) >> 2;
                    ft[i] = (top[i + 1] + 2 * top[i] + top[i - 1] + 2) >> 2;
                }
                fl[2 * n] = left[2 * n];
                ft[2 * n] = top[2 * n];
            }
            memcpy(left, fl, sizeof(int) * (2 * n + 1));
            memcpy(top, ft, sizeof(int) * (2 * n + 1));
        }
    }
    uint16_t *dst = pl + yTb * ps + xTb;
    int maxv = (1 << bd) - 1;
#define P_L(y) left[(y) + 1]
#define P_T(x) top[(x) + 1]
    if (mode == 0) { /* planar 8.4.4.2.5 */
        for (int y = 0; y < n; y++)
            for (int x = 0; x < n; x++)
                dst[y * ps + x] = (uint16_t)(((n - 1 - x) * P_L(y) + (x + 1) * P_T(n) + (n - 1 - y) * P_T(x) +
                                              (y + 1) * P_L(n) + n) >> (log2n + 1));
    } else if (mode == 1) { /* DC 8.4.4.2.6 */
        int sum = n;
        for (int i = 0; i < n; i++) sum += P_T(i) + P_L(i);
        int dc = sum >> (log2n + 1);
        for (int y = 0; y < n; y++)
            for (int x = 0; x < n; x++) dst[y * ps + x] = (uint16_t)dc;
        if (cIdx == 0 && n < 32) {
            dst[0] = (uint16_t)((P_L(0) + 2 * dc + P_T(0) + 2) >> 2);
            for (int x = 1; x < n; x++) dst[x] = (uint16_t)((P_T(x) + 3 * dc + 2) >> 2);
            for (int y = 1; y < n; y++) dst[y * ps] = (uint16_t)((P_L(y) + 3 * dc + 2) >> 2);
        }
    } else { /* angular 8.4.4.2.6 */
        int ang = k_angle[mode];
        int refbuf[3 * 64 + 2];
        int *ref = refbuf + 64 + 1;
        if (mode >= 18) {
            for (int x = 0; x <= n; x++) ref[x] = top[x]; /* p[-1+x][-1] */
            if (ang < 0) {
                if (((n * ang) >> 5) < -1)
                    for (int x = (n * ang) >> 5; x <= -1; x++) ref[x] = left[((x * k_inv_angle[mode] + 128) >> 8)];
            } else {
                for (int x = n + 1; x <= 2 * n; x++) ref[x] = top[x];
            }
            for (int y = 0; y < n; y++) {
                int idx = ((y + 1) * ang) >> 5, fact = ((y + 1) * ang) & 31;
                for (int x = 0; x < n; x++) {
                    int v = fact ? ((32 - fact) * ref[x + idx + 1] + fact * ref[x + idx + 2] + 16) >> 5
                                 : ref[x + idx + 1];
                    dst[y * ps + x] = (uint16_t)v;
                }
            }
            if (mode == 26 && cIdx == 0 && n < 32)
                for (int y = 0; y < n; y++)
                    dst[y * ps] = (uint16_t)CLIP3(0, maxv, P_T(0) + ((P_L(y) - left[0]) >> 1));
        } else {
            for (int x = 0; x <= n; x++) ref[x] = left[x]; /* p[-1][-1+x] */
            if (ang < 0) {
                if (((n * ang) >> 5) < -1)
                    for (int x = (n * ang) >> 5; x <= -1; x++) ref[x] = top[((x * k_inv_angle[mode] + 128) >> 8)];
            } else {
                for (int x = n + 1; x <= 2 * n; x++) ref[x] = left[x];
            }
            for (int x = 0; x < n; x++) {
                int idx = ((x + 1) * ang) >> 5, fact = ((x + 1) * ang) & 31;
                for (int y = 0; y < n; y++) {
                    int v = fact ? ((32 - fact) * ref[y + idx + 1] + fact * ref[y + idx + 2] + 16) >> 5
                                 : ref[y + idx + 1];
                    dst[y * ps + x] = (uint16_t)v;
                }
            }
            if (mode == 10 && cIdx == 0 && n < 32)
                for (int x = 0; x < n; x++)
                    dst[x] = (uint16_t)CLIP3(0, maxv, P_L(0) + ((P_T(x) - top[0]) >> 1));
        }
    }
#undef P_L
#undef P_T
}

/* ===================================================================== */
/* Scaling + transform — H.265 8.6.2-8.6.4                                */
/* ===================================================================== */
static int8_t g_tm[32][32]; /* transMatrix[k][n] */
static int g_tm_ready = 0;
static void init_transform(void) {
    if (g_tm_ready) return;
    /* unique magnitudes of the HEVC core transform: c[j] for cos(j*pi/64) */
    static const int odd[16] = {90, 90, 88, 85, 82, 78, 73, 67, 61, 54, 46, 38, 31, 22, 13, 4};
    static const int e2[8] = {90, 87, 80, 70, 57, 43, 25, 9};
    static const int e4[4] = {89, 75, 50, 18};
    int cv[33];
    cv[0] = 64;
    cv[32] = 0;
    cv[16] = 64;
    for (int i = 0; i < 16; i++) cv[2 * i + 1] = odd[i];
    for (int i = 0; i < 8; i++) cv[2 * (2 * i + 1)] = e2[i];
    for (int i = 0; i < 4; i++) cv[4 * (2 * i + 1)] = e4[i];
    cv[8] = 83;
    cv[24] = 36;
    for (int k = 0; k < 32; k++)
        for (int n = 0; n < 32; n++) {
            int j = ((2 * n + 1) * k) % 128;
            int v;
            if (j <= 32) v = cv[j];
            else if (j <= 64) v = -cv[64 - j];
            else if (j <= 96) v = -cv[j - 64];
            else v = cv[128 - j];
            g_tm[k][n] = (int8_t)v;
        }
    g_tm_ready = 1;
}
static const int k_dst[4][4] = {{29, 55, 74, 84}, {74, 74, 0, -74}, {84, -29, -74, 55}, {55, -84, 74, -29}};

/* 8.6.4.2 one-dimensional transform: y[i] = sum_j M[j][i] * x[j] */
static void tr1d(const int *x, int *y, int n, int dst) {
    for (int i = 0; i < n; i++) {
        int64_t s = 0;
        for (int j = 0; j < n; j++) {
            int m = dst ? k_dst[j][i] : g_tm[j * (32 / n)][i];
            s += (int64_t)m * x[j];
        }
        y[i] = (int)s;
    }
}

/* coef[y*n+x] TransCoeffLevel → res[y*n+x] residual (8.6.2) */
static void residual_from_coeffs(pic_t *p, int cIdx, int log2n, const int *coef, int qp, int ts, int bypass,
                                 int dst, int *res) {
    int n = 1 << log2n;
    if (bypass) {
        for (int i = 0; i < n * n; i++) res[i] = coef[i];
        return;
    }
    int bd = cIdx ? p->bdC : p->bdY;
    static const int ls[6] = {40, 45, 51, 57, 64, 72};
    int bdShift = bd + log2n - 5;
    int d[32 * 32];
    const uint8_t *m = p->sf[log2n - 2][log2n == 5 ? (cIdx ? cIdx : 0) : cIdx];
    for (int i = 0; i < n * n; i++) {
        int mm = (!p->sps->scaling_list_enabled || (ts && n > 4)) ? 16 : m[i];
        int64_t v = (int64_t)coef[i] * mm * ls[qp % 6] * ((int64_t)1 << (qp / 6));
        v = (v + ((int64_t)1 << (bdShift - 1))) >> bdShift;
        d[i] = (int)CLIP3(-32768, 32767, v);
    }
    int r[32 * 32];
    if (ts) {
        int tsShift = 5 + log2n;
        for (int i = 0; i < n * n; i++) r[i] = d[i] * (1 << tsShift);
    } else {
        int col[32], out[32], g[32 * 32];
        for (int x = 0; x < n; x++) { /* vertical: each column */
            for (int y = 0; y < n; y++) col[y] = d[y * n + x];
            tr1d(col, out, n, dst);
            for (int y = 0; y < n; y++) g[y * n + x] = CLIP3(-32768, 32767, (out[y] + 64) >> 7);
        }
        for (int y = 0; y < n; y++) { /* horizontal: each row */
            tr1d(g + y * n, out, n, dst);
            for (int x = 0; x < n; x++) r[y * n + x] = out[x];
        }
    }
    int bdShift2 = 20 - bd;
    for (int i = 0; i < n * n; i++) res[i] = (r[i] + (1 << (bdShift2 - 1))) >> bdShift2;
}

/* ===================================================================== */
/* Parsing                                                                */
/* ===================================================================== */
static int chroma_qp_map(int qpi, int chroma) {
    static const int tab[14] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37};
    if (chroma != 1) return imin(qpi, 51);
    if (qpi < 30) return qpi;
    if (qpi > 43) return qpi - 6;
    return tab[qpi - 30];
}

static void update_qpy(pic_t *p) {
    p->qpy_cur = ((p->qp_pred + p->cu_qp_delta_val + 52 + 2 * p->qpbdY) % (52 + p->qpbdY)) - p->qpbdY;
}

/* 8.6.1 first part: qPY_PRED for the quantization group */
/* 9.3.1 / 8.6.1: the CTB (rx, ry) starts a CTB row within its tile (the CTB to
 * its left is outside the picture or in another tile) */
static int first_ctb_in_tile_row(const pic_t *p, int rx, int ry) {
    const int rs = ry * p->wctb + rx;
    return rx == 0 || p->tile_rs[rs] != p->tile_rs[rs - 1];
}

/* 9.3.2.2: the WPP storage process runs after the CTB at raster address rs when
 * CtbAddrInRs % PicWidthInCtbsY == 1, or CtbAddrInRs > 1 and its tile differs
 * from that of CtbAddrInRs - 2 (so the state kept is the one after the second
 * CTB of the tile's row; a one-CTB-wide tile never syncs: its T is unavailable) */
static int wpp_storage_point(const pic_t *p, int rs) {
    return rs % p->wctb == 1 || (rs > 1 && p->tile_rs[rs] != p->tile_rs[rs - 2]);
}

static void derive_qp_pred(pic_t *p) {
    int prev;
    int first_in_ctb = (p->qg_x == p->ctb_x && p->qg_y == p->ctb_y);
    if (p->first_qg_in_slice) { /* first QG in the slice or in a tile */
        prev = p->slice_qp;
        p->first_qg_in_slice = 0;
    } else if (p->pps->wpp && first_in_ctb && first_ctb_in_tile_row(p, p->ctb_x >> p->log2ctb, p->ctb_y >> p->log2ctb)) {
        prev = p->slice_qp; /* 8.6.1: first QG of a CTB row within a tile, WPP */
    } else {
        prev = p->qp_prev_last;
    }
    int mask = p->ctb - 1;
    int qa = (p->qg_x & mask) ? p->qpy[(p->qg_y >> 2) * p->w4 + ((p->qg_x - 1) >> 2)] : prev;
    int qb = (p->qg_y & mask) ? p->qpy[((p->qg_y - 1) >> 2) * p->w4 + (p->qg_x >> 2)] : prev;
    p->qp_pred = (qa + qb + 1) >> 1;
}

static int scan_idx_for(pic_t *p, int log2n, int cIdx, int mode) {
    if (log2n == 2 || (log2n == 3 && cIdx == 0) || (log2n == 3 && p->chroma == 3)) {
        if (mode >= 6 && mode <= 14) return 2;
        if (mode >= 22 && mode <= 30) return 1;
    }
    return 0;
}

/* 7.3.8.11 residual_coding; coef[y*n+x] */
static int residual_coding(pic_t *p, int x0, int y0, int log2n, int cIdx, int mode, int *coef, int *ts_out) {
    cabac_t *c = &p->c;
    int n = 1 << log2n;
    memset(coef, 0, sizeof(int) * n * n);
    int ts = 0;
    (void)x0;
    (void)y0;
    if (p->pps->transform_skip && !p->cu_bypass && log2n <= 2) ts = dec_bin(c, CTX_TS_FLAG + (cIdx ? 1 : 0));
    *ts_out = ts;
    /* last_sig_coeff prefix — decoder.rs:109-130 */
    int cmax = (log2n << 1) - 1;
    int off, shift;
    if (cIdx == 0) { off = 3 * (log2n - 2) + ((log2n - 1) >> 2); shift = (log2n + 1) >> 2; }
    else { off = 15; shift = log2n - 2; }
    int px = 0, py = 0;
    while (px < cmax && dec_bin(c, CTX_LAST_X + off + (px >> shift))) px++;
    while (py < cmax && dec_bin(c, CTX_LAST_Y + off + (py >> shift))) py++;
    int lx = px, ly = py;
    if (px > 3) { int k = (px >> 1) - 1; lx = (1 << k) * (2 + (px & 1)) + bz_fl(bypass_src, c, k); }
    if (py > 3) { int k = (py >> 1) - 1; ly = (1 << k) * (2 + (py & 1)) + bz_fl(bypass_src, c, k); }
    int scanIdx = scan_idx_for(p, log2n, cIdx, mode);
    if (scanIdx == 2) { int t = lx; lx = ly; ly = t; }
    if (lx >= n || ly >= n) return oracle_fail("last sig coeff out of range");
    int sbl = log2n - 2, sbw = 1 << sbl;
    const uint8_t *sbscan = g_scan[sbl][scanIdx];
    const uint8_t *scan4 = g_scan[2][scanIdx];
    /* locate last sub-block / position */
    int lastSub = sbw * sbw - 1, lastPos = 16;
    for (;;) {
        if (lastPos == 0) { lastPos = 16; lastSub--; }
        lastPos--;
        int xS = sbscan[lastSub] & 15, yS = sbscan[lastSub] >> 4;
        int xC = (xS << 2) + (scan4[lastPos] & 15), yC = (yS << 2) + (scan4[lastPos] >> 4);
        if (xC == lx && yC == ly) break;
        if (lastSub < 0) return oracle_fail("last pos search");
    }
    uint8_t csbf[8][8];
    memset(csbf, 0, sizeof(csbf));
    int greater1_state_prev = 1; /* c1 carried across sub-blocks (HM-style ≡ 9.3.4.2.6) */
    int first_sb_done = 0;
    static const uint8_t ctxIdxMap[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
    for (int i = lastSub; i >= 0; i--) {
        int xS = sbscan[i] & 15, yS = sbscan[i] >> 4;
        int infer_dc = 0;
        int coded;
        if (i < lastSub && i > 0) {
            int r = (xS + 1 < sbw) ? csbf[yS][xS + 1] : 0;
            int b = (yS + 1 < sbw) ? csbf[yS + 1][xS] : 0;
            int ctx = imin(1, r + b) + (cIdx ? 2 : 0);
            coded = dec_bin(c, CTX_CSBF + ctx);
            infer_dc = 1;
        } else {
            coded = 1;
        }
        csbf[yS][xS] = (uint8_t)coded;
        int sig[16];
        memset(sig, 0, sizeof(sig));
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
                        if (log2n == 3) sigCtx += (scanIdx == 0) ? 9 : 15;
                        else sigCtx += 21;
                    } else {
                        if (log2n == 3) sigCtx += 9;
                        else sigCtx += 12;
                    }
                }
                int ctxInc = cIdx == 0 ? sigCtx : 27 + sigCtx;
                sig[nn] = dec_bin(c, CTX_SIG + ctxInc);
                if (sig[nn]) infer_dc = 0;
            } else if (coded && nn == 0 && infer_dc) {
                sig[0] = 1;
            }
        }
        /* greater1 / greater2 */
        int g1[16], g2[16], sign[16];
        memset(g1, 0, sizeof(g1));
        memset(g2, 0, sizeof(g2));
        memset(sign, 0, sizeof(sign));
        int any = 0;
        for (int nn = 15; nn >= 0; nn--) any |= sig[nn];
        if (!any) continue;
        int ctxSet = (i == 0 || cIdx > 0) ? 0 : 2;
        if (first_sb_done && greater1_state_prev == 0) ctxSet++;
        first_sb_done = 1;
        int greater1Ctx = 1;
        int firstSig = 16, lastSig = -1, numG1 = 0, lastG1Pos = -1;
        for (int nn = 15; nn >= 0; nn--) {
            if (!sig[nn]) continue;
            if (numG1 < 8) {
                int ctxInc = ctxSet * 4 + imin(3, greater1Ctx) + (cIdx ? 16 : 0);
                g1[nn] = dec_bin(c, CTX_GT1 + ctxInc);
                numG1++;
                if (g1[nn]) { if (lastG1Pos == -1) lastG1Pos = nn; }
                if (greater1Ctx > 0) greater1Ctx = g1[nn] ? 0 : greater1Ctx + 1;
            }
            if (lastSig == -1) lastSig = nn;
            firstSig = nn;
        }
        greater1_state_prev = greater1Ctx;
        int signHidden = (p->cu_bypass) ? 0 : (lastSig - firstSig > 3);
        if (lastG1Pos != -1) g2[lastG1Pos] = dec_bin(c, CTX_GT2 + ctxSet + (cIdx ? 4 : 0));
        for (int nn = 15; nn >= 0; nn--)
            if (sig[nn] && (!p->pps->sign_hiding || !signHidden || nn != firstSig)) sign[nn] = dec_bypass(c);
        int numSig = 0, sumAbs = 0;
        int cLastAbs = 0, cLastRice = 0, firstRem = 1;
        for (int nn = 15; nn >= 0; nn--) {
            if (!sig[nn]) continue;
            int base = 1 + g1[nn] + g2[nn];
            int rem = 0;
            if (base == ((numSig < 8) ? ((nn == lastG1Pos) ? 3 : 2) : 1)) {
                int k;
                if (firstRem) { k = 0; firstRem = 0; }
                else k = imin(cLastRice + (cLastAbs > 3 * (1 << cLastRice) ? 1 : 0), 4);
                rem = bz_calr(bypass_src, c, k);
                if (rem < 0) return oracle_fail("bad coeff_abs_level_remaining");
                cLastAbs = base + rem;
                cLastRice = k;
            }
            int xC = (xS << 2) + (scan4[nn] & 15), yC = (yS << 2) + (scan4[nn] >> 4);
            int v = (rem + base) * (1 - 2 * sign[nn]);
            if (p->pps->sign_hiding && signHidden) {
                sumAbs += rem + base;
                if (nn == firstSig && (sumAbs & 1)) v = -v;
            }
            coef[yC * n + xC] = v;
            numSig++;
        }
    }
    return 0;
}

/* reconstruct one TB: predict + residual */
static int recon_tb(pic_t *p, int cIdx, int xTb, int yTb, int log2n, int mode, int cbf, int x0l, int y0l) {
    if ((g_debug_flags & 8) && cIdx && p->chroma == 1 && log2n <= 3 && mode >= 0 && mode < 35)
        g_chroma_tb_hist[log2n - 2][mode][cbf ? 1 : 0]++;
    intra_predict(p, cIdx, xTb, yTb, log2n, mode);
    if (!cbf) return 0;
    int n = 1 << log2n;
    int coef[32 * 32], res[32 * 32], ts = 0;
    if (residual_coding(p, x0l, y0l, log2n, cIdx, mode, coef, &ts)) return -1;
    int qp;
    if (cIdx == 0) qp = p->qpy_cur + p->qpbdY;
    else {
        int off = cIdx == 1 ? p->pps->cb_qp_offset + p->cb_qp_off : p->pps->cr_qp_offset + p->cr_qp_off;
        int qpi = CLIP3(-p->qpbdC, 57, p->qpy_cur + off);
        qp = chroma_qp_map(qpi, p->chroma) + p->qpbdC;
    }
    int dst = (cIdx == 0 && n == 4);
    residual_from_coeffs(p, cIdx, log2n, coef, qp, ts, p->cu_bypass, dst, res);
    int bd = cIdx ? p->bdC : p->bdY, maxv = (1 << bd) - 1;
    uint16_t *pl = p->pl[cIdx] + yTb * p->ps[cIdx] + xTb;
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) {
            int v = pl[y * p->ps[cIdx] + x] + res[y * n + x];
            pl[y * p->ps[cIdx] + x] = (uint16_t)CLIP3(0, maxv, v);
        }
    return 0;
}

/* IntraPredModeC of the PB holding luma location (x0, y0) */
static int chroma_mode_of(pic_t *p, int x0, int y0) {
    const int k = ((y0 - p->cu_y) >= p->cu_pb ? 2 : 0) + ((x0 - p->cu_x) >= p->cu_pb ? 1 : 0);
    return p->cu_chroma_mode_c[p->chroma == 3 && p->cu_intra_split ? k : 0];
}

static int transform_unit(pic_t *p, int x0, int y0, int xB, int yB, int log2n, int depth, int blk, int cbf_l,
                          int cbf_cb, int cbf_cr, int pcb, int pcr) {
    (void)depth;
    int chroma4 = (p->chroma != 3 && log2n == 2);
    int cbfChroma = p->chroma == 0 ? 0 : (chroma4 ? (pcb || pcr) : (cbf_cb || cbf_cr));  /* either 4:2:2 flag */
    if (cbf_l || cbfChroma) {
        if (p->pps->cu_qp_delta && !p->is_cu_qp_delta_coded) {
            cabac_t *c = &p->c;
            int v = 0;
            while (v < 5 && dec_bin(c, CTX_CU_QP_DELTA + (v == 0 ? 0 : 1))) v++;
            if (v == 5) {
                int s = bz_egk(bypass_src, c, 0);
                if (s < 0) return oracle_fail("bad cu_qp_delta");
                v += s;
            }
            if (v && dec_bypass(c)) v = -v;
            /* 7.4.9.14: CuQpDeltaVal in [-(26 + QpBdOffsetY / 2), 25 + QpBdOffsetY / 2] */
            if (v < -(26 + p->qpbdY / 2) || v > 25 + p->qpbdY / 2) return oracle_fail("CuQpDeltaVal out of range");
            p->is_cu_qp_delta_coded = 1;
            p->cu_qp_delta_val = v;
            update_qpy(p);
        }
    }
    /* mark transform edges */
    int n = 1 << log2n;
    for (int k = 0; k < n; k += 4) {
        if (((y0 + k) >> 2) < p->h4 && (x0 >> 2) < p->w4) p->flg[((y0 + k) >> 2) * p->w4 + (x0 >> 2)] |= F_EDGE_V;
        if ((y0 >> 2) < p->h4 && ((x0 + k) >> 2) < p->w4) p->flg[(y0 >> 2) * p->w4 + ((x0 + k) >> 2)] |= F_EDGE_H;
    }
    int lmode = p->ipm[(y0 >> 2) * p->w4 + (x0 >> 2)];
    if (recon_tb(p, 0, x0, y0, log2n, lmode, cbf_l, x0, y0)) return -1;
    if (p->chroma == 0) return 0;
    int cm = chroma_mode_of(p, x0, y0);
    /* the chroma TBs of the TU (7.3.8.10): log2TrafoSizeC, and for 4:2:2 a
     * second TB below the first; with 4x4 luma TBs (not 4:4:4) the chroma of
     * the 8x8 parent follows its 4th luma TB */
    const int cx = chroma4 ? xB : x0, cy = chroma4 ? yB : y0;
    const int l2c = chroma4 ? 2 : (p->chroma == 3 ? log2n : log2n - 1);
    const int cb = chroma4 ? pcb : cbf_cb, cr = chroma4 ? pcr : cbf_cr;
    if (!chroma4 || blk == 3) {
        for (int ci = 1; ci < 3; ci++)
            for (int h = 0; h < (p->chroma == 2 ? 2 : 1); h++) {
                const int yc = cy / p->sh + (h << l2c);
                if (recon_tb(p, ci, cx / p->sw, yc, l2c, cm, ((ci == 1 ? cb : cr) >> h) & 1, cx, yc * p->sh))
                    return -1;
            }
    }
    return 0;
}

static int transform_tree(pic_t *p, int x0, int y0, int xB, int yB, int log2n, int depth, int blk, int pcb,
                          int pcr) {
    cabac_t *c = &p->c;
    const hevc_sps *s = p->sps;
    int split;
    if (log2n <= s->log2_max_tb && log2n > s->log2_min_tb && depth < p->cu_max_trafo_depth &&
        !(p->cu_intra_split && depth == 0))
        split = dec_bin(c, CTX_SPLIT_TF + 5 - log2n);
    else
        split = (log2n > s->log2_max_tb || (p->cu_intra_split && depth == 0));
    /* cbf_cb / cbf_cr: bit 0, and for 4:2:2 bit 1 of the lower chroma TB
     * (coded when the node is not split or is 8x8: 7.3.8.8) */
    int cbf_cb = 0, cbf_cr = 0;
    if ((log2n > 2 && p->chroma != 0) || p->chroma == 3) {
        const int two = p->chroma == 2 && (!split || log2n == 3);
        if (depth == 0 || (pcb & 1)) {
            cbf_cb = dec_bin(c, CTX_CBF_CHROMA + depth);
            if (two) cbf_cb |= dec_bin(c, CTX_CBF_CHROMA + depth) << 1;
        }
        if (depth == 0 || (pcr & 1)) {
            cbf_cr = dec_bin(c, CTX_CBF_CHROMA + depth);
            if (two) cbf_cr |= dec_bin(c, CTX_CBF_CHROMA + depth) << 1;
        }
    }
    if (split) {
        int h = 1 << (log2n - 1);
        if (transform_tree(p, x0, y0, x0, y0, log2n - 1, depth + 1, 0, cbf_cb, cbf_cr)) return -1;
        if (transform_tree(p, x0 + h, y0, x0, y0, log2n - 1, depth + 1, 1, cbf_cb, cbf_cr)) return -1;
        if (transform_tree(p, x0, y0 + h, x0, y0, log2n - 1, depth + 1, 2, cbf_cb, cbf_cr)) return -1;
        if (transform_tree(p, x0 + h, y0 + h, x0, y0, log2n - 1, depth + 1, 3, cbf_cb, cbf_cr)) return -1;
        return 0;
    }
    int cbf_l = dec_bin(c, CTX_CBF_LUMA + (depth == 0 ? 1 : 0));
    return transform_unit(p, x0, y0, xB, yB, log2n, depth, blk, cbf_l, cbf_cb, cbf_cr, pcb, pcr);
}

/* 8.4.2 luma MPM */
static int derive_luma_mode(pic_t *p, int xPb, int yPb, int prev, int mpm_idx, int rem) {
    int cand[2];
    for (int k = 0; k < 2; k++) {
        int xn = k == 0 ? xPb - 1 : xPb, yn = k == 0 ? yPb : yPb - 1;
        int m;
        if (!avail_zs(p, xPb, yPb, xn, yn)) m = 1;
        else if (k == 1 && yPb - 1 < ((yPb >> p->log2ctb) << p->log2ctb)) m = 1;
        else m = p->ipm[(yn >> 2) * p->w4 + (xn >> 2)];
        cand[k] = m;
    }
    int l[3];
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
    if (prev) return l[mpm_idx];
    /* sort ascending */
    if (l[0] > l[1]) { int t = l[0]; l[0] = l[1]; l[1] = t; }
    if (l[0] > l[2]) { int t = l[0]; l[0] = l[2]; l[2] = t; }
    if (l[1] > l[2]) { int t = l[1]; l[1] = l[2]; l[2] = t; }
    int m = rem;
    for (int i = 0; i < 3; i++)
        if (m >= l[i]) m++;
    return m;
}

/* 7.3.8.7 pcm_sample() of a CU with pcm_flag = 1 (the reference parses the SPS
 * PCM fields, parameter_set_reader.rs:107-125, and stops at the CU): after the
 * terminating bin the decoder has consumed through the codeword's final 1 bit;
 * pcm_alignment_zero_bits up to a byte boundary, PcmBitDepth-bit samples
 * (luma, then Cb, Cr), then 9.3.2.5 re-initialises the engine.  8.4.4.1:
 * recSamples = pcm_sample << (BitDepth - PcmBitDepth); 8.4.2: a PCM neighbour
 * counts as INTRA_DC; the CU is one block for deblocking, left unfiltered (and
 * without SAO) when pcm_loop_filter_disabled_flag is 1. */
static int pcm_cu(pic_t *p, int x0, int y0, int log2cb) {
    cabac_t *c = &p->c;
    const hevc_sps *s = p->sps;
    const int n = 1 << log2cb;
    set_map(p, p->ipm, x0, y0, n, 1);
    while (c->b.bit & 7)
        if (br_bit(&c->b)) return oracle_fail("pcm_alignment_zero_bit is 1");
    for (int ci = 0; ci < (p->chroma ? 3 : 1); ci++) {
        const int w = ci ? n / p->sw : n, h = ci ? n / p->sh : n;
        const int xs = ci ? x0 / p->sw : x0, ys = ci ? y0 / p->sh : y0;
        const int bd = ci ? p->bdC : p->bdY, pbd = ci ? s->pcm_bd_c : s->pcm_bd_y;
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++)
                p->pl[ci][(size_t)(ys + y) * p->ps[ci] + xs + x] = (uint16_t)(br_u(&c->b, pbd) << (bd - pbd));
    }
    if (c->b.err) return oracle_fail("PCM samples overrun the slice data");
    if (cabac_init_engine(c)) return -1;
    for (int k = 0; k < n; k += 4) {
        if (((y0 + k) >> 2) < p->h4) p->flg[((y0 + k) >> 2) * p->w4 + (x0 >> 2)] |= F_EDGE_V;
        if (((x0 + k) >> 2) < p->w4) p->flg[(y0 >> 2) * p->w4 + ((x0 + k) >> 2)] |= F_EDGE_H;
    }
    set_map(p, (uint8_t *)p->qpy, x0, y0, n, (uint8_t)(int8_t)p->qpy_cur);
    if (p->cu_bypass || s->pcm_loop_filter_disabled)
        for (int y = y0 >> 2; y < (y0 + n) >> 2 && y < p->h4; y++)
            for (int x = x0 >> 2; x < (x0 + n) >> 2 && x < p->w4; x++) p->flg[y * p->w4 + x] |= F_NOFILT;
    p->qp_prev_last = p->qpy_cur;
    return 0;
}

static int coding_unit(pic_t *p, int x0, int y0, int log2cb, int depth) {
    cabac_t *c = &p->c;
    const hevc_sps *s = p->sps;
    int n = 1 << log2cb;
    if (p->qg_new) { derive_qp_pred(p); p->qg_new = 0; }
    update_qpy(p);
    p->cu_bypass = p->pps->transquant_bypass ? dec_bin(c, CTX_TQ_BYPASS) : 0;
    int nxn = 0;
    if (log2cb == s->log2_min_cb) nxn = !dec_bin(c, CTX_PART_MODE);
    if (nxn && log2cb == s->log2_min_tb) return oracle_fail("NxN at min TB size");
    int pcm = 0;
    if (!nxn && s->pcm && log2cb >= s->log2_min_pcm && log2cb <= s->log2_max_pcm) pcm = dec_term(c);
    set_map(p, p->depth, x0, y0, n, (uint8_t)depth);
    if (pcm) return pcm_cu(p, x0, y0, log2cb);
    int np = nxn ? 4 : 1, pb = nxn ? n / 2 : n;
    int prev[4], mpm[4] = {0}, rem[4] = {0};
    for (int i = 0; i < np; i++) prev[i] = dec_bin(c, CTX_PREV_INTRA);
    for (int i = 0; i < np; i++) {
        if (prev[i]) mpm[i] = dec_bypass(c) ? (dec_bypass(c) ? 2 : 1) : 0;
        else rem[i] = bz_fl(bypass_src, c, 5);
        int xPb = x0 + (i & 1) * pb, yPb = y0 + (i >> 1) * pb;
        int m = derive_luma_mode(p, xPb, yPb, prev[i], mpm[i], rem[i]);
        set_map(p, p->ipm, xPb, yPb, pb, (uint8_t)m);
    }
    p->cu_x = x0;
    p->cu_y = y0;
    p->cu_pb = pb;
    /* intra_chroma_pred_mode: one per PB with 4:4:4, else one per CU (7.3.8.5);
     * 8.4.3 IntraPredModeC from it and the PB's luma mode, through Table 8-3
     * with 4:2:2 */
    static const uint8_t k_mode422[35] = {0,  1,  2,  2,  2,  2,  3,  5,  7,  8,  10, 11, 13, 15, 16, 18, 19, 20,
                                          21, 22, 23, 23, 24, 24, 25, 25, 26, 27, 27, 28, 28, 29, 29, 30, 31};
    for (int i = 0; p->chroma != 0 && i < (p->chroma == 3 ? np : 1); i++) {
        int icpm = dec_bin(c, CTX_CHROMA_MODE) ? bz_fl(bypass_src, c, 2) : 4;
        int xPb = x0 + (i & 1) * pb, yPb = y0 + (i >> 1) * pb;
        int lm = p->ipm[(yPb >> 2) * p->w4 + (xPb >> 2)];
        int cm;
        if (icpm == 4) cm = lm;
        else {
            static const int base[4] = {0, 26, 10, 1};
            cm = base[icpm];
            if (cm == lm) cm = 34;
        }
        p->cu_chroma_mode_c[i] = p->chroma == 2 ? k_mode422[cm] : cm;
    }
    p->cu_intra_split = nxn;
    p->cu_max_trafo_depth = s->max_th_depth_intra + nxn;
    if (transform_tree(p, x0, y0, x0, y0, log2cb, 0, 0, 0, 0)) return -1;
    /* CU-level maps */
    set_map(p, (uint8_t *)p->qpy, x0, y0, n, (uint8_t)(int8_t)p->qpy_cur);
    if (p->cu_bypass)
        for (int y = y0 >> 2; y < (y0 + n) >> 2 && y < p->h4; y++)
            for (int x = x0 >> 2; x < (x0 + n) >> 2 && x < p->w4; x++) p->flg[y * p->w4 + x] |= F_NOFILT;
    p->qp_prev_last = p->qpy_cur;
    return 0;
}

static int coding_quadtree(pic_t *p, int x0, int y0, int log2cb, int depth) {
    const hevc_sps *s = p->sps;
    int n = 1 << log2cb;
    int split;
    if (x0 + n <= p->W && y0 + n <= p->H && log2cb > s->log2_min_cb) {
        int cond = 0;
        if (avail_zs(p, x0, y0, x0 - 1, y0) && p->depth[(y0 >> 2) * p->w4 + ((x0 - 1) >> 2)] > depth) cond++;
        if (avail_zs(p, x0, y0, x0, y0 - 1) && p->depth[((y0 - 1) >> 2) * p->w4 + (x0 >> 2)] > depth) cond++;
        split = dec_bin(&p->c, CTX_SPLIT_CU + cond);
    } else {
        split = log2cb > s->log2_min_cb;
    }
    int log2qg = p->log2ctb - p->pps->diff_cu_qp_delta_depth;
    if (log2cb >= log2qg) {
        p->is_cu_qp_delta_coded = 0;
        p->cu_qp_delta_val = 0;
        p->qg_new = 1;
        p->qg_x = x0;
        p->qg_y = y0;
    }
    if (split) {
        int h = n >> 1;
        if (coding_quadtree(p, x0, y0, log2cb - 1, depth + 1)) return -1;
        if (x0 + h < p->W && coding_quadtree(p, x0 + h, y0, log2cb - 1, depth + 1)) return -1;
        if (y0 + h < p->H && coding_quadtree(p, x0, y0 + h, log2cb - 1, depth + 1)) return -1;
        if (x0 + h < p->W && y0 + h < p->H && coding_quadtree(p, x0 + h, y0 + h, log2cb - 1, depth + 1)) return -1;
        return 0;
    }
    return coding_unit(p, x0, y0, log2cb, depth);
}

/* 7.3.8.3 sao syntax */
static void parse_sao(pic_t *p, int rx, int ry) {
    cabac_t *c = &p->c;
    sao_ctb *s = &p->sao[ry * p->wctb + rx];
    memset(s, 0, sizeof(*s));
    const int cr = ry * p->wctb + rx, t = p->tile_rs[cr], sl = p->slice_rs[cr];
    int ml = 0, mu = 0;
    /* merge candidates: left / above CTB in the same slice and tile */
    if (rx > 0 && p->tile_rs[cr - 1] == t && p->slice_rs[cr - 1] == sl) ml = dec_bin(c, CTX_SAO_MERGE);
    if (ry > 0 && !ml && p->tile_rs[cr - p->wctb] == t && p->slice_rs[cr - p->wctb] == sl)
        mu = dec_bin(c, CTX_SAO_MERGE);
    if (ml) { *s = p->sao[ry * p->wctb + rx - 1]; return; }
    if (mu) { *s = p->sao[(ry - 1) * p->wctb + rx]; return; }
    int ncomp = p->chroma ? 3 : 1;
    for (int ci = 0; ci < ncomp; ci++) {
        if (!((p->sao_luma && ci == 0) || (p->sao_chroma && ci > 0))) { s->type[ci] = 0; continue; }
        if (ci < 2) {
            int t = 0;
            if (dec_bin(c, CTX_SAO_TYPE)) t = dec_bypass(c) ? 2 : 1;
            s->type[ci] = t;
        } else {
            s->type[2] = s->type[1];
        }
        if (!s->type[ci]) continue;
        int bd = ci ? p->bdC : p->bdY;
        int cmax = (1 << (imin(bd, 10) - 5)) - 1;
        int a[4];
        for (int i = 0; i < 4; i++) a[i] = bz_tr(bypass_src, c, cmax, 0);
        int sh = bd - imin(bd, 10); /* log2OffsetScale = 0 without RExt; bitDepth-Min(bitDepth,10) per 8.7.3 */
        (void)sh;
        if (s->type[ci] == 1) {
            for (int i = 0; i < 4; i++)
                if (a[i] && dec_bypass(c)) a[i] = -a[i];
            s->band[ci] = bz_fl(bypass_src, c, 5);
            for (int i = 0; i < 4; i++) s->off[ci][i + 1] = a[i];
        } else {
            if (ci == 0) s->eo[0] = bz_fl(bypass_src, c, 2);
            if (ci == 1) s->eo[1] = bz_fl(bypass_src, c, 2);
            if (ci == 2) s->eo[2] = s->eo[1];
            s->off[ci][1] = a[0];
            s->off[ci][2] = a[1];
            s->off[ci][3] = -a[2];
            s->off[ci][4] = -a[3];
        }
    }
}

/* ===================================================================== */
/* Deblocking — H.265 8.7.2                                               */
/* ===================================================================== */
static const uint8_t k_beta[52] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15,
                                   16, 17, 18, 20, 22, 24, 26, 28, 30, 32, 34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};
static const uint8_t k_tc[54] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};

/* filter one luma edge segment of 4 lines; vertical=1: edge between columns x-1|x */
static void dbk_luma_seg(pic_t *p, int x, int y, int vertical) {
    uint16_t *pl = p->pl[0];
    int ps = p->ps[0];
    int xp = vertical ? x - 1 : x, yp = vertical ? y : y - 1;
    int fp = p->flg[(yp >> 2) * p->w4 + (xp >> 2)], fq = p->flg[(y >> 2) * p->w4 + (x >> 2)];
    int qP = p->qpy[(yp >> 2) * p->w4 + (xp >> 2)], qQ = p->qpy[(y >> 2) * p->w4 + (x >> 2)];
    int qpl = (qQ + qP + 1) >> 1;
    int bS = 2;
    int bd = p->bdY;
    int Q = CLIP3(0, 51, qpl + p->beta_off * 2);
    int beta = k_beta[Q] * (1 << (bd - 8));
    Q = CLIP3(0, 53, qpl + 2 * (bS - 1) + p->tc_off * 2);
    int tc = k_tc[Q] * (1 << (bd - 8));
    /* sample accessor: P(i,k) = p_i at line k, Qs(i,k) = q_i */
    int stepx = vertical ? 1 : ps, stepk = vertical ? ps : 1;
    uint16_t *q0p = pl + y * ps + x;
#define PS(i, k) q0p[(k)*stepk - ((i) + 1) * stepx]
#define QS(i, k) q0p[(k)*stepk + (i)*stepx]
    int dp0 = iabs(PS(2, 0) - 2 * PS(1, 0) + PS(0, 0));
    int dp3 = iabs(PS(2, 3) - 2 * PS(1, 3) + PS(0, 3));
    int dq0 = iabs(QS(2, 0) - 2 * QS(1, 0) + QS(0, 0));
    int dq3 = iabs(QS(2, 3) - 2 * QS(1, 3) + QS(0, 3));
    int dpq0 = dp0 + dq0, dpq3 = dp3 + dq3, dp = dp0 + dp3, dq = dq0 + dq3, d = dpq0 + dpq3;
    if (d >= beta) return;
    int dsam[2];
    for (int t = 0; t < 2; t++) {
        int k = t ? 3 : 0;
        int dpq = 2 * (t ? dpq3 : dpq0);
        dsam[t] = (dpq < (beta >> 2) && iabs(PS(3, k) - PS(0, k)) + iabs(QS(0, k) - QS(3, k)) < (beta >> 3) &&
                   iabs(PS(0, k) - QS(0, k)) < ((5 * tc + 1) >> 1));
    }
    int dE = (dsam[0] && dsam[1]) ? 2 : 1;
    int dEp = dp < ((beta + (beta >> 1)) >> 3);
    int dEq = dq < ((beta + (beta >> 1)) >> 3);
    int maxv = (1 << bd) - 1;
    int nofp = (fp & F_NOFILT) != 0, nofq = (fq & F_NOFILT) != 0;
    for (int k = 0; k < 4; k++) {
        int p0 = PS(0, k), p1 = PS(1, k), p2 = PS(2, k), p3 = PS(3, k);
        int q0 = QS(0, k), q1 = QS(1, k), q2 = QS(2, k), q3 = QS(3, k);
        if (dE == 2) {
            int np0 = CLIP3(p0 - 2 * tc, p0 + 2 * tc, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
            int np1 = CLIP3(p1 - 2 * tc, p1 + 2 * tc, (p2 + p1 + p0 + q0 + 2) >> 2);
            int np2 = CLIP3(p2 - 2 * tc, p2 + 2 * tc, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
            int nq0 = CLIP3(q0 - 2 * tc, q0 + 2 * tc, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
            int nq1 = CLIP3(q1 - 2 * tc, q1 + 2 * tc, (p0 + q0 + q1 + q2 + 2) >> 2);
            int nq2 = CLIP3(q2 - 2 * tc, q2 + 2 * tc, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3);
            if (!nofp) { PS(0, k) = (uint16_t)np0; PS(1, k) = (uint16_t)np1; PS(2, k) = (uint16_t)np2; }
            if (!nofq) { QS(0, k) = (uint16_t)nq0; QS(1, k) = (uint16_t)nq1; QS(2, k) = (uint16_t)nq2; }
        } else {
            int delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
            if (iabs(delta) < tc * 10) {
                delta = CLIP3(-tc, tc, delta);
                if (!nofp) PS(0, k) = (uint16_t)CLIP3(0, maxv, p0 + delta);
                if (!nofq) QS(0, k) = (uint16_t)CLIP3(0, maxv, q0 - delta);
                if (dEp && !nofp) {
                    int dl = CLIP3(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + delta) >> 1);
                    PS(1, k) = (uint16_t)CLIP3(0, maxv, p1 + dl);
                }
                if (dEq && !nofq) {
                    int dl = CLIP3(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - delta) >> 1);
                    QS(1, k) = (uint16_t)CLIP3(0, maxv, q1 + dl);
                }
            }
        }
    }
#undef PS
#undef QS
}

/* chroma edge segment: (xc,yc) chroma coords of q0 of first line; lines = 4/sub */
static void dbk_chroma_seg(pic_t *p, int cIdx, int xc, int yc, int vertical, int lines) {
    uint16_t *pl = p->pl[cIdx];
    int ps = p->ps[cIdx];
    int xl = xc * p->sw, yl = yc * p->sh;
    int xlp = vertical ? xl - 1 : xl, ylp = vertical ? yl : yl - 1;
    int fp = p->flg[(ylp >> 2) * p->w4 + (xlp >> 2)], fq = p->flg[(yl >> 2) * p->w4 + (xl >> 2)];
    int qP = p->qpy[(ylp >> 2) * p->w4 + (xlp >> 2)], qQ = p->qpy[(yl >> 2) * p->w4 + (xl >> 2)];
    int off = cIdx == 1 ? p->pps->cb_qp_offset : p->pps->cr_qp_offset;
    int qpi = ((qQ + qP + 1) >> 1) + off;
    int qpc = chroma_qp_map(qpi, p->chroma);
    int Q = CLIP3(0, 53, qpc + 2 + p->tc_off * 2);
    int tc = k_tc[Q] * (1 << (p->bdC - 8));
    int maxv = (1 << p->bdC) - 1;
    int stepx = vertical ? 1 : ps, stepk = vertical ? ps : 1;
    uint16_t *q0p = pl + yc * ps + xc;
    for (int k = 0; k < lines; k++) {
        int p0 = q0p[k * stepk - stepx], p1 = q0p[k * stepk - 2 * stepx];
        int q0 = q0p[k * stepk], q1 = q0p[k * stepk + stepx];
        int delta = CLIP3(-tc, tc, ((((q0 - p0) * 4) + p1 - q1 + 4) >> 3));
        if (!(fp & F_NOFILT)) q0p[k * stepk - stepx] = (uint16_t)CLIP3(0, maxv, p0 + delta);
        if (!(fq & F_NOFILT)) q0p[k * stepk] = (uint16_t)CLIP3(0, maxv, q0 - delta);
    }
}

/* 8.7.2: the edge whose q0 sample is (x,y) is not filtered when q0's slice
 * has slice_deblocking_filter_disabled_flag, or the edge is a tile boundary
 * with loop_filter_across_tiles_enabled_flag 0, or a boundary with an earlier
 * slice and q0's slice_loop_filter_across_slices_enabled_flag is 0.
 * Otherwise the filter takes q0's slice_beta / tc offsets. */
static int edge_off(pic_t *p, int x, int y, int vertical) {
    const int xp = vertical ? x - 1 : x, yp = vertical ? y : y - 1;
    const slice_par *sq = &p->slices[slice_at(p, x, y)];
    if (sq->dbk_disabled) return 1;
    if (!p->pps->lf_across_tiles && tile_at(p, xp, yp) != tile_at(p, x, y)) return 1;
    if (!sq->lf_across && slice_at(p, xp, yp) != slice_at(p, x, y)) return 1;
    p->beta_off = sq->beta;
    p->tc_off = sq->tc;
    return 0;
}

static void deblock_picture(pic_t *p) {
    for (int dir = 0; dir < 2; dir++) {
        int vertical = dir == 0;
        /* luma: edges on the 8x8 grid, 4-line segments */
        for (int y = 0; y < p->H; y += 4)
            for (int x = 0; x < p->W; x += 4) {
                int e = vertical ? x : y;
                if (e == 0 || (e & 7)) continue;
                if (!vertical && (x & 3)) continue;
                int f = p->flg[(y >> 2) * p->w4 + (x >> 2)];
                if (!(f & (vertical ? F_EDGE_V : F_EDGE_H))) continue;
                if (edge_off(p, x, y, vertical)) continue;
                dbk_luma_seg(p, x, y, vertical);
            }
        if (p->chroma == 0) continue;
        /* chroma: edges on the 8x8 chroma grid; per 4-luma-line segment */
        int lines = vertical ? 4 / p->sh : 4 / p->sw;
        for (int ci = 1; ci < 3; ci++)
            for (int yc = 0; yc < p->chh; yc += (vertical ? lines : 8))
                for (int xc = 0; xc < p->cw; xc += (vertical ? 8 : lines)) {
                    int e = vertical ? xc : yc;
                    if (e == 0 || (e & 7)) continue;
                    int xl = xc * p->sw, yl = yc * p->sh;
                    int f = p->flg[(yl >> 2) * p->w4 + (xl >> 2)];
                    if (!(f & (vertical ? F_EDGE_V : F_EDGE_H))) continue;
                    if (edge_off(p, xl, yl, vertical)) continue;
                    dbk_chroma_seg(p, ci, xc, yc, vertical, lines);
                }
    }
}

/* ===================================================================== */
/* SAO — H.265 8.7.3                                                      */
/* ===================================================================== */
/* 8.7.3.2: SaoOffsetVal 0 when the neighbour (xn,yn) of (x,y) is in another
 * slice whose boundary with it is not filtered across */
static int sao_slice_off(const pic_t *p, int x, int y, int xn, int yn) {
    const int sc = slice_at(p, x, y), sn = slice_at(p, xn, yn);
    if (sc == sn) return 0;
    const int later = zscan_addr(p, xn, yn) < zscan_addr(p, x, y) ? sc : sn;
    return !p->slices[later].lf_across;
}

static void sao_picture(pic_t *p, uint16_t *out[3], const int ops[3]) {
    int ncomp = p->chroma ? 3 : 1;
    static const int hpos[4][2] = {{-1, 1}, {0, 0}, {-1, 1}, {1, -1}};
    static const int vpos[4][2] = {{0, 0}, {-1, 1}, {-1, 1}, {-1, 1}};
    for (int ci = 0; ci < ncomp; ci++) {
        int PW = ci ? p->cw : p->W, PH = ci ? p->chh : p->H;
        int sw = ci ? p->sw : 1, sh = ci ? p->sh : 1;
        int bd = ci ? p->bdC : p->bdY, maxv = (1 << bd) - 1;
        const uint16_t *in = p->pl[ci];
        int ps = p->ps[ci];
        for (int y = 0; y < PH; y++) memcpy(out[ci] + (size_t)y * ops[ci], in + (size_t)y * ps, sizeof(uint16_t) * PW);
        int cwid = p->ctb / sw, chei = p->ctb / sh;
        for (int ry = 0; ry < p->hctb; ry++)
            for (int rx = 0; rx < p->wctb; rx++) {
                const sao_ctb *s = &p->sao[ry * p->wctb + rx];
                int t = s->type[ci];
                if (!t) continue;
                int bandTable[32] = {0};
                if (t == 1)
                    for (int k = 0; k < 4; k++) bandTable[(k + s->band[ci]) & 31] = k + 1;
                int x0 = rx * cwid, y0 = ry * chei;
                for (int y = y0; y < y0 + chei && y < PH; y++)
                    for (int x = x0; x < x0 + cwid && x < PW; x++) {
                        int xl = x * sw, yl = y * sh;
                        if (p->flg[(yl >> 2) * p->w4 + (xl >> 2)] & F_NOFILT) continue;
                        int v = in[y * ps + x];
                        int o;
                        if (t == 2) {
                            int cl = s->eo[ci];
                            int ax = x + hpos[cl][0], ay = y + vpos[cl][0];
                            int bx = x + hpos[cl][1], by = y + vpos[cl][1];
                            if (ax < 0 || ay < 0 || ax >= PW || ay >= PH || bx < 0 || by < 0 || bx >= PW || by >= PH)
                                continue;
                            /* 8.7.3.2: a neighbour in another tile with
                             * loop_filter_across_tiles_enabled_flag 0 ⇒ SaoOffsetVal 0 */
                            if (!p->pps->lf_across_tiles) {
                                int tc = tile_at(p, xl, yl);
                                if (tile_at(p, ax * sw, ay * sh) != tc || tile_at(p, bx * sw, by * sh) != tc) continue;
                            }
                            /* a neighbour in another slice: the flag of the later of the two slices (in
                             * MinTbAddrZs order) decides */
                            if (sao_slice_off(p, xl, yl, ax * sw, ay * sh) || sao_slice_off(p, xl, yl, bx * sw, by * sh))
                                continue;
                            int a = in[ay * ps + ax], b = in[by * ps + bx];
                            int e = 2 + (v > a) - (v < a) + (v > b) - (v < b);
                            if (e == 0 || e == 1 || e == 2) e = (e == 2) ? 0 : e + 1;
                            o = s->off[ci][e];
                        } else {
                            o = s->off[ci][bandTable[v >> (bd - 5)]];
                        }
                        out[ci][(size_t)y * ops[ci] + x] = (uint16_t)CLIP3(0, maxv, v + o);
                    }
            }
    }
}

/* ===================================================================== */
/* Slice header + slice data                                              */
/* ===================================================================== */
typedef struct {
    int first, dependent, address; /* first_slice_segment_in_pic_flag, dependent_slice_segment_flag,
                                      slice_segment_address (raster) */
    int idr, slice_type, qp_delta, sao_l, sao_c, cb_off, cr_off;
    int dbk_disabled, beta, tc, lf_across;
    int num_entry, entry[1024];
    size_t data_bit; /* RBSP bit offset of slice_segment_data() */
} slice_hdr;

/* 7.3.6.1 slice_segment_header() — slice.rs:44-204 (which takes only the
 * first segment: slice.rs:61-64); a dependent segment carries only the
 * address and entry points, its other fields are the slice's (the caller
 * copies them) */
static int parse_slice_header(br_t *b, int nal_type, const hevc_sps *s, const hevc_pps *pp, int nctb, slice_hdr *h) {
    memset(h, 0, sizeof(*h));
    h->first = (int)br_u(b, 1);
    if (nal_type >= 16 && nal_type <= 23) br_u(b, 1);
    br_ue(b);
    if (!h->first) {
        if (pp->dependent_slices) h->dependent = (int)br_u(b, 1);
        int bits = 0;
        while ((1 << bits) < nctb) bits++;
        h->address = (int)br_u(b, bits);
        if (h->address >= nctb) return oracle_fail("slice_segment_address out of range");
    }
    if (h->dependent) goto entry_points;
    br_u(b, pp->num_extra_bits);
    h->slice_type = (int)br_ue(b);
    if (h->slice_type != 2) return oracle_fail("only I slices are supported");
    if (pp->output_flag_present) br_u(b, 1);
    if (s->separate_colour_plane) br_u(b, 2);
    h->idr = (nal_type == 19 || nal_type == 20);
    if (!h->idr) {
        br_u(b, s->log2_max_poc_lsb);
        int sps_flag = (int)br_u(b, 1);
        if (!sps_flag) {
            int nd[65];
            memcpy(nd, s->st_rps_num_delta, sizeof(nd));
            if (parse_st_rps(b, s->num_st_rps, s->num_st_rps, nd)) return -1;
        } else if (s->num_st_rps > 1) {
            int bits = 0;
            while ((1 << bits) < s->num_st_rps) bits++;
            br_u(b, bits);
        }
        if (s->long_term_refs_present) {
            int nsps = 0;
            if (s->num_lt_sps > 0) nsps = (int)br_ue(b);
            int npics = (int)br_ue(b);
            for (int i = 0; i < nsps + npics; i++) {
                if (i < nsps) {
                    if (s->num_lt_sps > 1) {
                        int bits = 0;
                        while ((1 << bits) < s->num_lt_sps) bits++;
                        br_u(b, bits);
                    }
                } else {
                    br_u(b, s->log2_max_poc_lsb);
                    br_u(b, 1);
                }
                if (br_u(b, 1)) br_ue(b);
            }
        }
        if (s->temporal_mvp) br_u(b, 1);
    }
    if (s->sao) {
        h->sao_l = (int)br_u(b, 1);
        if (s->chroma_format_idc != 0) h->sao_c = (int)br_u(b, 1);
    }
    h->qp_delta = br_se(b);
    if (pp->slice_chroma_qp_offsets_present) { h->cb_off = br_se(b); h->cr_off = br_se(b); }
    int override = 0;
    if (pp->deblock_override_enabled) override = (int)br_u(b, 1);
    h->dbk_disabled = pp->deblock_disabled;
    h->beta = pp->beta_offset_div2;
    h->tc = pp->tc_offset_div2;
    if (override) {
        h->dbk_disabled = (int)br_u(b, 1);
        if (!h->dbk_disabled) { h->beta = br_se(b); h->tc = br_se(b); }
    }
    h->lf_across = pp->loop_filter_across_slices;
    if (pp->loop_filter_across_slices && (h->sao_l || h->sao_c || !h->dbk_disabled)) h->lf_across = (int)br_u(b, 1);
entry_points:
    if (pp->tiles || pp->wpp) {
        h->num_entry = (int)br_ue(b);
        if (h->num_entry > 1024) return oracle_fail("too many entry points");
        if (h->num_entry > 0) {
            int len = (int)br_ue(b) + 1;
            if (len > 32) return oracle_fail("bad offset_len");
            for (int i = 0; i < h->num_entry; i++) h->entry[i] = (int)br_u(b, len) + 1;
        }
    }
    if (pp->slice_header_ext) {
        int l = (int)br_ue(b);
        for (int i = 0; i < l; i++) br_u(b, 8);
    }
    /* byte_alignment(): one bit equal to 1 then zeros */
    if (br_u(b, 1) != 1) return oracle_fail("slice header alignment bit");
    while (b->bit & 7) br_u(b, 1);
    h->data_bit = b->bit;
    if (b->err) return oracle_fail("slice header overrun");
    return 0;
}

/* rbsp byte offset → raw payload offset (ep[] holds the raw indices of the
 * removed 0x03 bytes) */
static size_t rbsp_to_raw(size_t rb, const uint32_t *ep, int nep) {
    size_t r = 0, raw = 0;
    int e = 0;
    while (r < rb) {
        if (e < nep && ep[e] == raw) { raw++; e++; continue; }
        raw++;
        r++;
    }
    while (e < nep && ep[e] == raw) { raw++; e++; }
    return raw;
}

#define MAX_SEGMENTS 1024

/* Decode one coded picture: the VCL NAL units (slice segments) of an item's
 * length-prefixed NAL units, in order (heic/decoder.rs:146-164 takes the
 * one NAL of a single-slice picture).  Each slice segment starts at its
 * slice_segment_address and runs in tile scan until end_of_slice_segment_flag;
 * contexts at a segment / substream start follow 9.3.1 (tile start: init;
 * WPP row start: the stored row-above state if the above-right CTB is
 * available, else init; dependent segment: the previous segment's end state;
 * otherwise init). */
static int decode_picture(const hevc_ps *ps, const uint8_t *item, size_t item_len, uint16_t *outp[3],
                          const int ops[3], int tile_index, oracle_substream_check *checks, int max_checks,
                          int *n_checks) {
    init_tables();
    init_transform();
    const hevc_sps *s = &ps->sps;
    const hevc_pps *pp = &ps->pps;
    if (s->range_ext_any || pp->range_ext_any) return oracle_fail("range extension tools not supported");
    if (s->separate_colour_plane) return oracle_fail("separate_colour_plane_flag not supported");
    /* the VCL NAL units, 4-byte length prefixes */
    const uint8_t *nals[MAX_SEGMENTS];
    size_t nlen[MAX_SEGMENTS];
    int nn = 0;
    for (size_t pos = 0; pos < item_len;) {
        if (item_len - pos < 4) return oracle_fail("truncated NAL length prefix");
        size_t l = ((size_t)item[pos] << 24) | ((size_t)item[pos + 1] << 16) | ((size_t)item[pos + 2] << 8) | item[pos + 3];
        pos += 4;
        if (l < 3 || l > item_len - pos) return oracle_fail("NAL unit length out of range");
        if (((item[pos] >> 1) & 63) < 32) {
            if (nn == MAX_SEGMENTS) return oracle_fail("too many slice segments");
            nals[nn] = item + pos;
            nlen[nn++] = l;
        }
        pos += l;
    }
    if (!nn) return oracle_fail("no VCL NAL unit in the picture");
    pic_t *p = (pic_t *)calloc(1, sizeof(pic_t));
    int ret = -1;
    slice_hdr *h = (slice_hdr *)malloc(sizeof(slice_hdr));
    uint8_t *rbsp = NULL;
    uint32_t *ep = NULL;
    p->sps = s;
    p->pps = pp;
    p->W = s->width;
    p->H = s->height;
    p->log2ctb = s->log2_ctb;
    p->ctb = 1 << s->log2_ctb;
    p->wctb = (p->W + p->ctb - 1) >> p->log2ctb;
    p->hctb = (p->H + p->ctb - 1) >> p->log2ctb;
    p->minTb = s->log2_min_tb;
    p->minCb = s->log2_min_cb;
    p->chroma = s->chroma_format_idc;
    p->sw = (p->chroma == 1 || p->chroma == 2) ? 2 : 1; /* SubWidthC, SubHeightC (Table 6-1) */
    p->sh = p->chroma == 1 ? 2 : 1;
    p->cw = p->chroma ? p->W / p->sw : 0;
    p->chh = p->chroma ? p->H / p->sh : 0;
    p->bdY = s->bit_depth_y;
    p->bdC = s->bit_depth_c;
    p->qpbdY = 6 * (p->bdY - 8);
    p->qpbdC = 6 * (p->bdC - 8);
    p->w4 = (p->W + 3) >> 2;
    p->h4 = (p->H + 3) >> 2;
    for (int ci = 0; ci < (p->chroma ? 3 : 1); ci++) {
        int w = ci ? p->cw : p->W, hh = ci ? p->chh : p->H;
        p->ps[ci] = w;
        p->pl[ci] = (uint16_t *)calloc((size_t)w * hh, sizeof(uint16_t));
    }
    const int nctb = p->wctb * p->hctb;
    p->ipm = (uint8_t *)calloc((size_t)p->w4 * p->h4, 1);
    p->depth = (uint8_t *)calloc((size_t)p->w4 * p->h4, 1);
    p->flg = (uint8_t *)calloc((size_t)p->w4 * p->h4, 1);
    p->qpy = (int8_t *)calloc((size_t)p->w4 * p->h4, 1);
    p->sao = (sao_ctb *)calloc((size_t)nctb, sizeof(sao_ctb));
    p->slice_rs = (int *)malloc(sizeof(int) * (size_t)nctb);
    for (int i = 0; i < nctb; i++) p->slice_rs[i] = -1;
    p->slices = (slice_par *)calloc((size_t)nn, sizeof(slice_par));
    build_scaling(p);
    if (tile_scan_init(p)) goto out;
    int next_ts = 0, cur_slice = -1, any_sao = 0, substream = 0;
    for (int k = 0; k < nn; k++) {
        const uint8_t *nal = nals[k];
        const size_t nal_len = nlen[k];
        free(rbsp);
        free(ep);
        rbsp = (uint8_t *)malloc(nal_len);
        ep = (uint32_t *)malloc(sizeof(uint32_t) * (nal_len / 3 + 4));
        int nep = 0;
        size_t rn = ep_remove(nal + 2, nal_len - 2, rbsp, ep, &nep, (int)(nal_len / 3 + 4));
        br_t hb = {rbsp, rn, 0, 0};
        if (parse_slice_header(&hb, (nal[0] >> 1) & 63, s, pp, nctb, h)) goto out;
        if (h->first != (k == 0)) { oracle_fail("first_slice_segment_in_pic_flag out of order"); goto out; }
        if (p->rs2ts[h->address] != next_ts) { oracle_fail("slice segments out of order or overlapping"); goto out; }
        if (!h->dependent) {
            slice_par *sl = &p->slices[++cur_slice];
            sl->qp = pp->init_qp + h->qp_delta;
            sl->sao_l = h->sao_l;
            sl->sao_c = h->sao_c;
            sl->dbk_disabled = h->dbk_disabled;
            sl->beta = h->beta;
            sl->tc = h->tc;
            sl->cb_off = h->cb_off;
            sl->cr_off = h->cr_off;
            sl->lf_across = h->lf_across;
            sl->addr_rs = h->address;
            any_sao |= sl->sao_l || sl->sao_c;
        } else if (cur_slice < 0) {
            oracle_fail("dependent slice segment without a slice");
            goto out;
        }
        const slice_par *sl = &p->slices[cur_slice];
        p->slice_qp = sl->qp;
        p->sao_luma = sl->sao_l;
        p->sao_chroma = sl->sao_c;
        p->dbk_disabled = sl->dbk_disabled;
        p->beta_off = sl->beta;
        p->tc_off = sl->tc;
        p->cb_qp_off = sl->cb_off;
        p->cr_qp_off = sl->cr_off;
        /* substream raw starts of this segment */
        size_t sub_raw[1025];
        sub_raw[0] = rbsp_to_raw(h->data_bit >> 3, ep, nep);
        for (int i = 0; i < h->num_entry; i++) sub_raw[i + 1] = sub_raw[i] + (size_t)h->entry[i];
        p->c.b.d = rbsp;
        p->c.b.n = rn;
        p->c.b.bit = h->data_bit;
        int ctbAddr = next_ts, seg_sub = 0;
        size_t sub_start_rbsp = h->data_bit >> 3;
        uint32_t sub_bins0 = p->c.bins;
        int sub_first = 1; /* the next CTU starts a substream */
        for (;;) { /* ctbAddr is CtbAddrInTs: tile scan (7.3.8.1) */
            int rs = p->ts2rs[ctbAddr], rx = rs % p->wctb, ry = rs / p->wctb;
            p->ctb_x = rx << p->log2ctb;
            p->ctb_y = ry << p->log2ctb;
            p->slice_rs[rs] = cur_slice;
            if (sub_first) {
                /* 9.3.1 context variables at a substream start */
                const int tile_start = ctbAddr == 0 || p->tile_rs[rs] != p->tile_rs[p->ts2rs[ctbAddr - 1]];
                if (tile_start) {
                    cabac_init_ctx(&p->c, p->slice_qp);
                } else if (pp->wpp && first_ctb_in_tile_row(p, rx, ry)) {
                    if (p->wpp_saved && avail_zs(p, p->ctb_x, p->ctb_y, p->ctb_x + p->ctb, p->ctb_y - p->ctb)) {
                        memcpy(p->c.st, p->wpp_st, CTX_NUM);
                        memcpy(p->c.mps, p->wpp_mps, CTX_NUM);
                    } else {
                        cabac_init_ctx(&p->c, p->slice_qp);
                    }
                } else if (h->dependent && ctbAddr == next_ts) {
                    memcpy(p->c.st, p->ds_st, CTX_NUM);
                    memcpy(p->c.mps, p->ds_mps, CTX_NUM);
                } else {
                    cabac_init_ctx(&p->c, p->slice_qp);
                }
                if (cabac_init_engine(&p->c)) goto out;
                /* 8.6.1: qPY_PREV = SliceQpY at the first QG of a slice or a tile */
                if (tile_start || (ctbAddr == next_ts && !h->dependent)) p->first_qg_in_slice = 1;
                sub_first = 0;
            }
            if (p->sao_luma || p->sao_chroma) parse_sao(p, rx, ry);
            if (coding_quadtree(p, p->ctb_x, p->ctb_y, p->log2ctb, 0)) goto out;
            if (pp->wpp && wpp_storage_point(p, rs)) {
                memcpy(p->wpp_st, p->c.st, CTX_NUM);
                memcpy(p->wpp_mps, p->c.mps, CTX_NUM);
                p->wpp_saved = 1;
            }
            int end = dec_term(&p->c);
            ctbAddr++;
            int cut_end = !end && ctbAddr == nctb && (g_debug_flags & 4);
            /* WPP: every CTB row of a tile is a substream (the next CTB in tile scan is on another row) */
            int row_end = pp->wpp && (ctbAddr == nctb || p->ts2rs[ctbAddr] / p->wctb != ry);
            int tile_end = pp->tiles && ctbAddr < nctb && p->tile_rs[p->ts2rs[ctbAddr]] != p->tile_rs[rs];
            if (end || row_end || tile_end || cut_end) {
                int ok = 1;
                if (!end) ok = dec_term(&p->c); /* end_of_subset_one_bit */
                /* the last consumed bit must be 1 and the rest of the byte 0 */
                size_t pos = p->c.b.bit;
                if (pos == 0 || ((pos - 1) >> 3) >= rn || !((rbsp[(pos - 1) >> 3] >> (7 - ((pos - 1) & 7))) & 1))
                    ok = 0; /* (a reader past the end: a truncated substream) */
                while (pos & 7) {
                    if ((pos >> 3) < rn && ((rbsp[pos >> 3] >> (7 - (pos & 7))) & 1)) ok = 0;
                    pos++;
                }
                if (checks && *n_checks < max_checks) {
                    oracle_substream_check *ck = &checks[(*n_checks)++];
                    ck->tile = (uint32_t)tile_index;
                    ck->substream = (uint32_t)substream; /* in the picture, over its segments */
                    ck->raw_start = (uint32_t)rbsp_to_raw(sub_start_rbsp, ep, nep);
                    ck->raw_entry = seg_sub <= h->num_entry ? (uint32_t)sub_raw[seg_sub] : 0xffffffffu;
                    ck->term_ok = (uint32_t)(ok && (end ? (k + 1 < nn || ctbAddr == nctb) : 1));
                    ck->bins = p->c.bins - sub_bins0;
                }
                substream++;
                if (end) {
                    if (k + 1 == nn && ctbAddr != nctb) { oracle_fail("end_of_slice_segment before last CTU"); goto out; }
                    if (k + 1 < nn && ctbAddr == nctb) { oracle_fail("slice segments after the last CTU"); goto out; }
                    if (seg_sub != h->num_entry) { oracle_fail("entry points do not match the substreams"); goto out; }
                    if (pp->dependent_slices) { /* 9.3.2.4 storage for a following dependent segment */
                        memcpy(p->ds_st, p->c.st, CTX_NUM);
                        memcpy(p->ds_mps, p->c.mps, CTX_NUM);
                    }
                    break;
                }
                if (!ok) { oracle_fail("end_of_subset_one_bit mismatch"); goto out; }
                if (cut_end) break;
                /* byte_alignment + engine re-init at the next substream */
                p->c.b.bit = pos;
                seg_sub++;
                sub_start_rbsp = pos >> 3;
                sub_bins0 = p->c.bins;
                sub_first = 1;
            }
            if (ctbAddr >= nctb) { oracle_fail("missing end_of_slice_segment_flag"); goto out; }
        }
        next_ts = ctbAddr;
    }
    if (next_ts != nctb && !(g_debug_flags & 4)) { oracle_fail("slice segments do not cover the picture"); goto out; }
    if (!(g_debug_flags & 1)) deblock_picture(p);
    {
        /* SAO into full-size temp, then crop into caller planes */
        uint16_t *full[3] = {0, 0, 0};
        int fps[3] = {p->W, p->cw, p->cw};
        int nc = p->chroma ? 3 : 1;
        for (int ci = 0; ci < nc; ci++)
            full[ci] = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)(ci ? p->cw * p->chh : p->W * p->H));
        if (any_sao && !(g_debug_flags & 2)) sao_picture(p, full, fps);
        else
            for (int ci = 0; ci < nc; ci++)
                memcpy(full[ci], p->pl[ci], sizeof(uint16_t) * (size_t)(ci ? p->cw * p->chh : p->W * p->H));
        for (int ci = 0; ci < nc; ci++) {
            int sw = ci ? p->sw : 1, shh = ci ? p->sh : 1;
            int cl = s->conf_l / sw, ct = s->conf_t / shh;
            int ow = s->out_w / sw, oh = s->out_h / shh;
            if (!outp[ci]) continue;
            for (int y = 0; y < oh; y++)
                memcpy(outp[ci] + (size_t)y * ops[ci], full[ci] + (size_t)(y + ct) * fps[ci] + cl,
                       sizeof(uint16_t) * ow);
        }
        for (int ci = 0; ci < nc; ci++) free(full[ci]);
    }
    ret = 0;
out:
    for (int ci = 0; ci < 3; ci++) free(p->pl[ci]);
    free(p->ipm);
    free(p->depth);
    free(p->flg);
    free(p->qpy);
    free(p->sao);
    free(p->rs2ts);
    free(p->ts2rs);
    free(p->tile_rs);
    free(p->slice_rs);
    free(p->slices);
    for (int a = 0; a < 4; a++)
        for (int m = 0; m < 6; m++) free(p->sf[a][m]);
    free(p);
    free(h);
    free(rbsp);
    free(ep);
    return ret;
}

/* ===================================================================== */
/* Tile / HEIC entry points                                               */
/* ===================================================================== */
int oracle_decode_tile(const uint8_t *hvcc, size_t hvcc_len, const uint8_t *item, size_t item_len, uint16_t *y,
                       int ypitch, uint16_t *cb, int cbpitch, uint16_t *cr, int crpitch) {
    hevc_ps ps;
    if (hevc_parse_hvcc(hvcc, hvcc_len, &ps)) return -1;
    uint16_t *o[3] = {y, cb, cr};
    int op[3] = {ypitch, cbpitch, crpitch};
    int nchk = 0;
    return decode_picture(&ps, item, item_len, o, op, 0, NULL, 0, &nchk);
}

void oracle_image_free(oracle_image *img) {
    for (int i = 0; i < 3; i++) { free(img->plane[i]); img->plane[i] = NULL; }
}

#define FOURCC(a, b, c, d) (((uint32_t)(a) << 24) | ((uint32_t)(b) << 16) | ((uint32_t)(c) << 8) | (uint32_t)(d))

int oracle_decode_heic(const uint8_t *data, size_t len, oracle_image *out, oracle_substream_check *checks,
                       int max_checks, int *n_checks) {
    memset(out, 0, sizeof(*out));
    int dummy = 0;
    if (!n_checks) n_checks = &dummy;
    *n_checks = 0;
    heif_file *f = (heif_file *)calloc(1, sizeof(heif_file));
    int ret = -1;
    uint32_t *ids = (uint32_t *)malloc(sizeof(uint32_t) * HEIF_MAX_TO);
    if (heif_parse(data, len, f)) goto done;
    heif_item *pi = heif_item_by_id(f, f->primary);
    if (!pi) { oracle_fail("primary item not found"); goto done; }
    int rows = 1, cols = 1, ow = 0, oh = 0, nt;
    if (pi->type == FOURCC('g', 'r', 'i', 'd')) {
        size_t gl;
        uint8_t *g = heif_item_data(f, pi, &gl);
        if (!g || gl < 8) { free(g); oracle_fail("bad grid descriptor"); goto done; }
        int fl = (g[1] & 1) ? 4 : 2;
        rows = g[2] + 1;
        cols = g[3] + 1;
        ow = 0;
        oh = 0;
        for (int i = 0; i < fl; i++) { ow = (ow << 8) | g[4 + i]; oh = (oh << 8) | g[4 + fl + i]; }
        free(g);
        nt = heif_grid_tiles(f, pi->id, ids, HEIF_MAX_TO);
        if (nt != rows * cols) { oracle_fail("grid tile count mismatch"); goto done; }
    } else if (pi->type == FOURCC('h', 'v', 'c', '1')) {
        ids[0] = pi->id;
        nt = 1;
    } else {
        oracle_fail("unsupported primary item type");
        goto done;
    }
    hevc_ps ps;
    {
        heif_item *t0 = heif_item_by_id(f, ids[0]);
        const heif_prop *hv = t0 ? heif_item_prop(f, t0, FOURCC('h', 'v', 'c', 'C')) : NULL;
        if (!hv) { oracle_fail("tile has no hvcC"); goto done; }
        if (hevc_parse_hvcc(data + hv->off, hv->len, &ps)) goto done;
    }
    int tw = ps.sps.out_w, th = ps.sps.out_h;
    if (pi->type != FOURCC('g', 'r', 'i', 'd')) { ow = tw; oh = th; }
    int chroma = ps.sps.chroma_format_idc;
    out->width = (uint32_t)ow;
    out->height = (uint32_t)oh;
    out->chroma_format_idc = (uint32_t)chroma;
    out->bit_depth = (uint32_t)ps.sps.bit_depth_y;
    int sw = (chroma == 1 || chroma == 2) ? 2 : 1, sh = chroma == 1 ? 2 : 1; /* SubWidthC, SubHeightC */
    int np = chroma ? 3 : 1;
    for (int ci = 0; ci < np; ci++) {
        out->pw[ci] = (uint32_t)(ci ? (ow + sw - 1) / sw : ow);
        out->ph[ci] = (uint32_t)(ci ? (oh + sh - 1) / sh : oh);
        out->plane[ci] = (uint16_t *)calloc((size_t)out->pw[ci] * out->ph[ci], sizeof(uint16_t));
    }
    /* full-grid scratch (uncropped), then crop */
    int gw = cols * tw, gh = rows * th;
    uint16_t *grid[3] = {0, 0, 0};
    int gp[3] = {gw, gw / sw, gw / sw};
    for (int ci = 0; ci < np; ci++)
        grid[ci] = (uint16_t *)calloc((size_t)(ci ? (gw / sw) * (gh / sh) : gw * gh), sizeof(uint16_t));
    for (int t = 0; t < nt; t++) {
        heif_item *it = heif_item_by_id(f, ids[t]);
        if (!it) { oracle_fail("tile item missing"); goto free_grid; }
        size_t il;
        uint8_t *item = heif_item_data(f, it, &il);
        if (!item) goto free_grid;
        int r = t / cols, c = t % cols;
        uint16_t *o[3] = {0, 0, 0};
        for (int ci = 0; ci < np; ci++) {
            int x = c * tw / (ci ? sw : 1), y = r * th / (ci ? sh : 1);
            o[ci] = grid[ci] + (size_t)y * gp[ci] + x;
        }
        int rc = decode_picture(&ps, item, il, o, gp, t, checks, max_checks, n_checks);
        free(item);
        if (rc) goto free_grid;
    }
    for (int ci = 0; ci < np; ci++)
        for (uint32_t y = 0; y < out->ph[ci]; y++)
            memcpy(out->plane[ci] + (size_t)y * out->pw[ci], grid[ci] + (size_t)y * gp[ci],
                   sizeof(uint16_t) * out->pw[ci]);
    ret = 0;
free_grid:
    for (int ci = 0; ci < np; ci++) free(grid[ci]);
done:
    if (ret) oracle_image_free(out);
    free(ids);
    free(f);
    return ret;
}
