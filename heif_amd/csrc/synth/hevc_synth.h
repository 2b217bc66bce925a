/* hevc_synth.h — synthetic HEVC intra bitstream generator (see hevc_synth.c).
 * Data generator for tests and benchmarks; not part of the decode path. */
#ifndef HEVC_SYNTH_H
#define HEVC_SYNTH_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define SYNTH_MAX_TILES 8

typedef struct {
    int32_t width, height;            /* pic_width/height_in_luma_samples (multiples of MinCbSize) */
    int32_t conf_right, conf_bottom;  /* conformance-window crop in luma samples (even for 4:2:0) */
    int32_t chroma_format;            /* chroma_format_idc: 0 = 4:0:0, 1 = 4:2:0, 2 = 4:2:2, 3 = 4:4:4 */
    int32_t bit_depth;                /* 8..10, luma = chroma */
    int32_t log2_ctb, log2_min_cb, log2_min_tb, log2_max_tb, max_th_depth_intra;
    int32_t sign_hiding, cu_qp_delta, diff_cu_qp_delta_depth;
    int32_t transform_skip, tq_bypass, scaling_list, strong_intra;
    int32_t init_qp, slice_qp_delta, cb_qp_offset, cr_qp_offset;
    int32_t sao, deblock_disabled, beta_offset_div2, tc_offset_div2;
    int32_t density;                  /* sig_coeff_flag probability, percent */
    int32_t wpp;                      /* entropy_coding_sync_enabled_flag: 1 = one substream per CTB row
                                         with entry points, 0 = the whole slice in one substream */
    /* HEVC tiles (tiles_enabled_flag when tile_cols * tile_rows > 1; needs wpp 0):
     * uniform_spacing_flag, else column widths / row heights in CTBs for all
     * but the last column / row; loop_filter_across_tiles_enabled_flag */
    int32_t tile_cols, tile_rows, tile_uniform, tile_lf_across;
    int32_t tile_col_w[SYNTH_MAX_TILES], tile_row_h[SYNTH_MAX_TILES];
    /* slice segments of slice_ctus CTUs (tile scan; 0 = one segment).  A new
     * slice k > 0 takes SliceQpY + (7k mod 5) - 2 and its own SAO flags;
     * slice_dependent 1: every segment after the first is a dependent one,
     * 2: odd-numbered segments are; slice_lf_across 0: no loop filtering across
     * slices (pps flag 0), 1: across every slice boundary, 2: the even-numbered
     * slices' flag is 1; slice_dbk_vary: slices k > 0 override the deblocking
     * (disabled when k mod 3 = 2, beta k mod 3 - 1, tc 1 - k mod 3) */
    int32_t slice_ctus, slice_dependent, slice_lf_across, slice_dbk_vary;
    /* PCM coding units: pcm_enabled_flag, PCM sample bit depths (1..bit_depth),
     * CU sizes log2 [pcm_log2_min, pcm_log2_max] (3..5), pcm_loop_filter_disabled_flag,
     * pcm_flag probability in percent for a CU that may take it */
    int32_t pcm, pcm_bd_y, pcm_bd_c, pcm_log2_min, pcm_log2_max, pcm_lf_disabled, pcm_pct;
} synth_params;

/* Each returns the NAL unit length (2-byte header included, emulation
 * prevention applied) or a negative value (-1 allocation / -2 parameters /
 * -3 capacity). */
long synth_vps(const synth_params *p, uint8_t *out, size_t cap);
long synth_sps(const synth_params *p, uint8_t *out, size_t cap);
long synth_pps(const synth_params *p, uint8_t *out, size_t cap);
/* One IDR picture (a single I slice; WPP or tile substreams + entry points). */
long synth_picture(const synth_params *p, uint64_t seed, uint8_t *out, size_t cap);
/* The picture's slice segments as 4-byte-length-prefixed NAL units (a HEIF
 * item's layout); synth_picture takes single-segment pictures only. */
long synth_picture_item(const synth_params *p, uint64_t seed, uint8_t *out, size_t cap);
int synth_check_params(const synth_params *p);

#ifdef __cplusplus
}
#endif
#endif
