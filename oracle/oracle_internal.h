/* oracle_internal.h — shared types of the CPU oracle (TEST INFRASTRUCTURE ONLY). */
#ifndef HEIF_ORACLE_INTERNAL_H
#define HEIF_ORACLE_INTERNAL_H

#include "oracle.h"

#define HEIF_MAX_ITEMS 256
#define HEIF_MAX_EXTENTS 8
#define HEIF_MAX_PROPS 16
#define HEIF_MAX_PROPS_TOTAL 1024
#define HEIF_MAX_REFS 64
#define HEIF_MAX_TO 1024

typedef struct {
    uint32_t id, type;
    int hidden;
    int construction_method;
    int n_extents;
    uint64_t ext_off[HEIF_MAX_EXTENTS], ext_len[HEIF_MAX_EXTENTS];
    int n_props;
    uint32_t props[HEIF_MAX_PROPS]; /* 1-based ipco indices */
} heif_item;

typedef struct {
    uint32_t type;
    size_t off, len; /* payload within the file */
} heif_prop;

typedef struct {
    uint32_t type, from;
    int n_to;
    uint32_t to[HEIF_MAX_TO];
} heif_ref;

typedef struct {
    const uint8_t *data;
    size_t len;
    uint32_t primary;
    int n_items;
    heif_item items[HEIF_MAX_ITEMS];
    int n_props;
    heif_prop props[HEIF_MAX_PROPS_TOTAL];
    int n_refs;
    heif_ref refs[HEIF_MAX_REFS];
    size_t iloc_s, iloc_e, ipma_s, ipma_e;
    size_t idat_off, idat_len;
} heif_file;

int heif_parse(const uint8_t *d, size_t n, heif_file *f);
heif_item *heif_item_by_id(heif_file *f, uint32_t id);
const heif_prop *heif_item_prop(heif_file *f, heif_item *it, uint32_t type);
uint8_t *heif_item_data(heif_file *f, heif_item *it, size_t *len);
int heif_grid_tiles(heif_file *f, uint32_t grid_id, uint32_t *tiles, int max);

/* ---- HEVC parameter sets (H.265 7.3.2.2 / 7.3.2.3) ---- */
#define HEVC_MAX_TILE_DIM 64
typedef struct {
    int chroma_format_idc, separate_colour_plane;
    int width, height;                 /* pic_width/height_in_luma_samples */
    int conf_l, conf_r, conf_t, conf_b; /* in luma samples */
    int out_w, out_h;
    int bit_depth_y, bit_depth_c;
    int log2_max_poc_lsb;
    int log2_min_cb, log2_ctb, log2_min_tb, log2_max_tb;
    int max_th_depth_inter, max_th_depth_intra;
    int scaling_list_enabled;
    int amp, sao, pcm;
    int pcm_bd_y, pcm_bd_c, log2_min_pcm, log2_max_pcm, pcm_loop_filter_disabled;
    int num_st_rps;
    int st_rps_num_delta[65];
    int long_term_refs_present, num_lt_sps;
    int temporal_mvp, strong_intra_smoothing;
    int range_ext_any;
    uint8_t sl[4][6][64];  /* ScalingList (coded order) */
    int sl_dc[4][6];
} hevc_sps;

typedef struct {
    int dependent_slices, output_flag_present, num_extra_bits;
    int sign_hiding, cabac_init_present, init_qp;
    int constrained_intra, transform_skip;
    int cu_qp_delta, diff_cu_qp_delta_depth;
    int cb_qp_offset, cr_qp_offset, slice_chroma_qp_offsets_present;
    int transquant_bypass, tiles, wpp;
    /* 7.4.3.3 tile layout: columns / rows (1 when tiles is 0), explicit sizes in
     * CTBs when not uniform_spacing (the last one is implied) */
    int tile_cols, tile_rows, tile_uniform, lf_across_tiles;
    int tile_col_w[HEVC_MAX_TILE_DIM], tile_row_h[HEVC_MAX_TILE_DIM];
    int loop_filter_across_slices;
    int deblock_override_enabled, deblock_disabled, beta_offset_div2, tc_offset_div2;
    int scaling_list_present;
    uint8_t sl[4][6][64];
    int sl_dc[4][6];
    int lists_mod, log2_parallel_merge, slice_header_ext;
    int range_ext_any;
} hevc_pps;

typedef struct {
    hevc_sps sps;
    hevc_pps pps;
} hevc_ps;

int hevc_parse_hvcc(const uint8_t *p, size_t n, hevc_ps *ps);
int oracle_fail(const char *msg);

#endif
