/*
 * oracle.h — CPU restatement of the friendlymatthew/heif HEIC decode path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in heif_amd/ links, loads or calls this
 * code; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * use it, and only as the checker / CPU baseline.
 *
 * Parity status: PARTIALLY PINNED.
 *   - The pieces the reference implements are pinned against the reference's
 *     own known-answer tests (ue/se Tables 9-2/9-3 and EP removal:
 *     src/hevc/rbsp_reader.rs:139-303; TR Table 9-39 and chroma-mode Table
 *     9-41: src/cabac/decoder.rs:286-373) and against its metadata golden
 *     values (tests/libheif_comparison.rs:102-111).
 *   - Pixel reconstruction is NOT computed by the reference (sao() and
 *     coding_quadtree() are todo!() at src/hevc/slice.rs:249-255) and its
 *     pixel oracle (libheif 1.18.2 via libheif-rs 1.1.0, Cargo.lock:43-56)
 *     is absent from this image.  Pixels are therefore a restatement of
 *     ITU-T H.265 (clauses cited per function) whose parse is self-checked
 *     on every WPP substream (terminate bit + entry-point position), and
 *     whose planes are committed as golden hashes: "parity unpinned" for
 *     reconstruction in the sense of the task statement.
 */
#ifndef HEIF_ORACLE_H
#define HEIF_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- reference known-answer hooks ---------------------------------- */

/* rbsp_reader.rs:11-39 (same rule: 00 00 03 xx, xx<=3 or at end). Returns
 * output length; out must hold n bytes. */
size_t oracle_remove_emulation_prevention(const uint8_t *in, size_t n, uint8_t *out);
/* rbsp_reader.rs:87-113: decode one ue(v)/se(v) from the start of buf.
 * Returns 0 on success. */
int oracle_read_ue(const uint8_t *buf, size_t n, uint32_t *val);
int oracle_read_se(const uint8_t *buf, size_t n, int32_t *val);
/* cabac/decoder.rs:166-190 TR binarization over an explicit bin string.
 * Returns decoded value, *used = bins consumed, or -1 on underrun. */
int oracle_decode_tr_bins(const uint8_t *bins, int nbins, int c_max, int c_rice, int *used);
/* cabac/decoder.rs:192-204 intra_chroma_pred_mode bins (Table 9-41). */
int oracle_decode_chroma_mode_bins(const uint8_t *bins, int nbins, int *used);
/* cabac/decoder.rs:230-261 coeff_abs_level_remaining over explicit bins. */
int oracle_decode_coeff_abs_level_remaining_bins(const uint8_t *bins, int nbins,
                                                 int c_rice, int *used);

/* ---- container metadata (tests/libheif_comparison.rs:182-275) -------- */
typedef struct {
    uint32_t primary_item_id;
    uint32_t ispe_width, ispe_height;    /* primary item ispe */
    uint32_t width, height;              /* after irot swap */
    uint32_t rotation;                   /* irot angle (x90 deg ccw) */
    uint32_t luma_bits, chroma_bits;     /* from tile SPS */
    uint32_t num_thumbnails;
    uint32_t is_grid, grid_rows, grid_cols, out_width, out_height;
    uint32_t num_tiles;
    uint32_t tile_width, tile_height;    /* coded (cropped) tile size */
    uint32_t chroma_format_idc;
} oracle_meta;

int oracle_read_meta(const uint8_t *data, size_t len, oracle_meta *out);

/* ---- decode ---------------------------------------------------------- */
typedef struct {
    uint32_t width, height;        /* cropped output (grid output size) */
    uint32_t chroma_format_idc;    /* 0 = 4:0:0, 1 = 4:2:0 */
    uint32_t bit_depth;
    /* planes as uint16 samples, row-major, tight: Y width*height,
     * Cb/Cr ((width+1)/2)*((height+1)/2) for 4:2:0 */
    uint16_t *plane[3];
    uint32_t pw[3], ph[3];
} oracle_image;

/* Per-substream parse self-check record. */
typedef struct {
    uint32_t tile;             /* tile index */
    uint32_t substream;        /* WPP row (or 0) */
    uint32_t raw_start;        /* raw NAL byte offset where decoding started */
    uint32_t raw_entry;        /* raw NAL byte offset given by the entry point */
    uint32_t term_ok;          /* terminate bin == 1 exactly at last CTU, and
                                  trailing alignment bits are 1,0.. */
    uint32_t bins;             /* bins decoded in this substream */
} oracle_substream_check;

/* Decode a whole HEIC file (grid or single hvc1 primary item).  Planes are
 * malloc'd; free with oracle_image_free.  checks may be NULL; otherwise it
 * receives up to max_checks records and *n_checks the count. */
int oracle_decode_heic(const uint8_t *data, size_t len, oracle_image *out,
                       oracle_substream_check *checks, int max_checks, int *n_checks);
void oracle_image_free(oracle_image *img);

/* Tile-level entry used by the CPU baseline (one tile per task):
 * decode one length-prefixed tile item given the hvcC record bytes.
 * Writes planes of the coded picture (cropped to the SPS conformance window)
 * into caller buffers with the given pitches (in samples, uint16). */
int oracle_decode_tile(const uint8_t *hvcc, size_t hvcc_len,
                       const uint8_t *item, size_t item_len,
                       uint16_t *y, int ypitch, uint16_t *cb, int cbpitch,
                       uint16_t *cr, int crpitch);

/* Enumerate tiles of the primary grid item: fills item offsets/lengths
 * (into data) and the hvcC property bytes offset/length.  Returns count. */
int oracle_list_tiles(const uint8_t *data, size_t len, uint32_t *off, uint32_t *ln,
                      int max, uint32_t *hvcc_off, uint32_t *hvcc_len);
/* The same for any coded image item (item_id 0 = primary), and the first
 * auxiliary image ('auxl' → primary) of a file, 0 if none. */
int oracle_list_item_tiles(const uint8_t *data, size_t len, uint32_t item_id, uint32_t *off, uint32_t *ln,
                           int max, uint32_t *hvcc_off, uint32_t *hvcc_len);
uint32_t oracle_aux_item(const uint8_t *data, size_t len);

const char *oracle_last_error(void);
/* bring-up: bit0 skips deblocking, bit1 skips SAO, bit2 lets a picture end
 * like a non-last tile, bit3 counts 4:2:0 chroma TBs (thread-local) */
void oracle_set_debug_flags(int flags);
/* the bit3 counts: out[2][35][2] = [log2 - 2][IntraPredModeC][cbf] */
void oracle_chroma_tb_hist(uint32_t *out, int reset);

#ifdef __cplusplus
}
#endif
#endif
