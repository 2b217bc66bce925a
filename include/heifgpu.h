/*
 * heifgpu.h — C ABI of the MI355X-native HEIC (HEVC intra still) decode path.
 *
 * Drop-in boundary for friendlymatthew/heif:
 *   - heifgpu_image_parse / heifgpu_image_info replace the host half of
 *     HeicDecoder::decode (src/heic/decoder.rs:12-112: HeifReader::read,
 *     hvcC → VPS/SPS/PPS, primary item → grid tiles → slice headers);
 *   - heifgpu_decode_batch replaces the serial per-tile loop
 *     (src/heic/decoder.rs:114-119: SliceSegmentReader::try_new +
 *     read_data, src/hevc/slice.rs:19-42, :206-256) and, unlike the
 *     reference (which returns Result<()> and panics at slice.rs:250), writes
 *     the reconstructed Y/Cb/Cr planes.
 * The test hooks at the end expose the host pieces the reference unit-tests
 * (src/hevc/rbsp_reader.rs:139-303, src/cabac/decoder.rs:286-373,
 * tests/libheif_comparison.rs:9-112).
 *
 * Conventions: functions return 0 on success and a negative HEIFGPU_E_*
 * code on failure (the reference's anyhow::Result / ensure! / bail!);
 * heifgpu_last_error() returns the message of the last failure on the
 * calling thread.  All pointers are plain host or device pointers; no
 * framework types cross the boundary.  A context is bound to one device and
 * must not be used from two threads at once; distinct contexts may run
 * concurrently (one per GPU).
 */
#ifndef HEIFGPU_H
#define HEIFGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HEIFGPU_ABI_VERSION 6

enum {
    HEIFGPU_OK = 0,
    HEIFGPU_E_INVALID = -1,     /* bad argument */
    HEIFGPU_E_PARSE = -2,       /* container / parameter-set / slice-header error */
    HEIFGPU_E_UNSUPPORTED = -3, /* valid stream using a tool outside this path */
    HEIFGPU_E_DEVICE = -4,      /* HIP runtime error */
    HEIFGPU_E_DECODE = -5       /* a picture's bitstream failed the kernel checks */
};

/* per-image status bits reported by heifgpu_batch_status */
enum {
    HEIFGPU_ST_CABAC_INIT = 1 << 0,
    HEIFGPU_ST_SUBSTREAM_END = 1 << 1,
    HEIFGPU_ST_OVERRUN = 1 << 2,
    HEIFGPU_ST_SYNTAX = 1 << 3,
    HEIFGPU_ST_UNSUPPORTED = 1 << 4,
    HEIFGPU_ST_CAPACITY = 1 << 5
};

typedef struct heifgpu_image heifgpu_image; /* host-parsed HEIC image */
typedef struct heifgpu_ctx heifgpu_ctx;     /* per-device decoder context */
typedef struct heifgpu_batch heifgpu_batch; /* device-resident batch */

typedef struct {
    uint32_t width, height;       /* output (grid-cropped) size, coded orientation */
    uint32_t chroma_format_idc;   /* 0 = 4:0:0, 1 = 4:2:0, 2 = 4:2:2, 3 = 4:4:4 (Cb/Cr planes
                                     ceil(w / SubWidthC) x ceil(h / SubHeightC)) */
    uint32_t bit_depth;           /* luma bit depth (chroma equal) */
    uint32_t bytes_per_sample;    /* 1 for 8-bit, 2 otherwise */
    uint32_t grid_rows, grid_cols;/* 1x1 for a single coded item */
    uint32_t tile_width, tile_height;
    uint32_t num_tiles;
    uint32_t rotation;            /* irot angle, anticlockwise in 90-degree units */
    uint32_t ispe_width, ispe_height;
    uint32_t coded_bytes;         /* sum of tile item bytes */
    uint32_t primary_item_id;
    uint32_t num_thumbnails;
    uint32_t matrix_coeffs, full_range;
    uint32_t item_id;             /* the decoded item (primary_item_id unless parsed by item) */
    uint32_t aux_item_id;         /* first auxiliary image of the primary ('auxl'), 0 if none */
} heifgpu_image_info;

typedef struct {
    void *plane[3];               /* device pointers, caller-owned (Y, Cb, Cr) */
    int32_t pitch[3];             /* bytes per row */
} heifgpu_planes;

/* decode options of heifgpu_batch_prepare_ex */
typedef struct {
    /* Single-image tile split across GPUs: only grid tiles k
     * (row-major) with k % tile_stride == tile_offset are decoded, each into
     * its window of the full-size output planes; the other windows are not
     * written.  0 or 1 = every tile.  Tiles are independent IDR pictures
     * (src/heic/decoder.rs:98-119 decodes them one by one). */
    uint32_t tile_stride, tile_offset;
    /* CABAC parse mode: HEIFGPU_PARSE_AUTO picks by batch
     * size (spread up to 1536 pictures, lanes above; lanes whatever is asked
     * for a batch with dependent slice segments starting inside a CTB row);
     * HEIFGPU_PARSE_LANES packs one substream per lane (throughput);
     * HEIFGPU_PARSE_SOLO runs one substream per wavefront, a picture's rows in
     * one workgroup; HEIFGPU_PARSE_SPREAD one substream per wavefront, every
     * row its own workgroup (latency of small batches).  HEIFGPU_PARSE_ROWS
     * (ABI 5 only: one picture per lane, one CTB row of up to 64 pictures per
     * wavefront) was removed in ABI 6, as it won only on batches that repeat
     * bitstreams; prepare answers HEIFGPU_E_UNSUPPORTED. */
    uint32_t parse_mode;
    /* lanes mode: pictures per wavefront (0 = adaptive; larger values are
     * capped at 64 / CTB rows) */
    uint32_t pics_per_wave;
    /* sets of parse outputs (ABI 4): 0 = the default (3, or HEIFGPU_PIPELINE);
     * 1 = no overlap; 2 = parse n+1 beside the reconstruction of n; 3 = parse
     * n+2, transform n+1 and reconstruction n overlap.  Every set holds its own
     * TU / coefficient / residual / map arenas (~3.2 MB per 512x512 picture),
     * so a memory-tight caller can ask for fewer.  Taken when the batch is
     * created (the first prepare); reloads keep it. */
    uint32_t pipeline_sets;
} heifgpu_batch_opts;

enum {
    HEIFGPU_PARSE_AUTO = 0,
    HEIFGPU_PARSE_LANES = 1,
    HEIFGPU_PARSE_SOLO = 2,
    HEIFGPU_PARSE_SPREAD = 3,
    HEIFGPU_PARSE_ROWS = 4 /* removed in ABI 6: HEIFGPU_E_UNSUPPORTED */
};

/* ---- host: demux + parameter sets + slice headers ------------------- */
/* data is copied; the returned image owns its bytes. */
int heifgpu_image_parse(const uint8_t *data, size_t len, heifgpu_image **out);
/* n independent files parsed on `threads` host threads (<= 0: all hardware
 * threads).  out[i] is NULL when file i failed; rc[i] (optional) receives its
 * code.  Returns 0 when every file parsed, else the first failure's code. */
int heifgpu_image_parse_many(const uint8_t *const *data, const size_t *len, size_t n, int threads,
                             heifgpu_image **out, int *rc);
/* Any coded image item by ID (0 = primary), e.g. the HDR gain map the primary
 * references through 'auxl' (info.aux_item_id; src/heif/grammar.rs:202-207
 * parses the reference but nothing decodes it).  Grid or single hvc1 item. */
int heifgpu_image_parse_item(const uint8_t *data, size_t len, uint32_t item_id, heifgpu_image **out);
int heifgpu_image_get_info(const heifgpu_image *img, heifgpu_image_info *info);
void heifgpu_image_free(heifgpu_image *img);

/* ---- device context --------------------------------------------------- */
int heifgpu_create(int device, heifgpu_ctx **out);
void heifgpu_destroy(heifgpu_ctx *ctx);
const char *heifgpu_last_error(void);

/* ---- batched decode ----------------------------------------------------
 * heifgpu_batch_prepare flattens n images (all must share bit depth and
 * chroma format) into device descriptors, uploads their bitstreams
 * (complete on return) and allocates the work arenas.
 * heifgpu_batch_prepare_ex does the same with options (NULL = defaults) and
 * without waiting for the upload: the host work (flattening into a pinned
 * staging buffer) is done on return, the host-to-device copies run on an
 * internal upload stream that the next heifgpu_batch_decode of the batch
 * waits for.  With *inout == NULL it creates a batch; otherwise it reloads
 * *inout with the new images, reusing its device arenas when they are large
 * enough (the copies wait for every decode still reading the old contents).
 * Two batches reloaded alternately overlap host parsing and upload of batch
 * n + 1 with the decode of batch n.  heifgpu_batch_decode
 * then enqueues the five decode stages on `stream` (a hipStream_t; NULL =
 * the device's null stream, as everywhere in HIP) and returns immediately; out[i] receives
 * image i.  It may be called repeatedly on the same batch (the bench times
 * exactly this call).  heifgpu_batch_status synchronises the stream and
 * returns the per-image status words (0 = ok): the OR over every decode of
 * the batch since the previous heifgpu_batch_status call or the last
 * (re)load, so damage seen by any of several pipelined decodes is reported;
 * the call clears them. */
int heifgpu_batch_prepare(heifgpu_ctx *ctx, const heifgpu_image *const *imgs, size_t n, heifgpu_batch **out);
int heifgpu_batch_prepare_ex(heifgpu_ctx *ctx, const heifgpu_image *const *imgs, size_t n,
                             const heifgpu_batch_opts *opts, heifgpu_batch **inout);
int heifgpu_batch_decode(heifgpu_ctx *ctx, heifgpu_batch *batch, const heifgpu_planes *out, void *stream);
int heifgpu_batch_status(heifgpu_ctx *ctx, heifgpu_batch *batch, uint32_t *status, void *stream);
/* ABI 5.  A reload does not wait for the previous load's decodes in flight;
 * their status words stay with that load (heifgpu_batch_status reports the
 * current load only).  This reads and clears them: per image of the load
 * before the current one (*n_prev images, 0 if there is none; status must
 * hold cap >= *n_prev words; status = NULL only sets *n_prev and reads
 * nothing), after its last decode.  The words survive until the batch is
 * reloaded again.  Returns HEIFGPU_E_DECODE if any is nonzero. */
int heifgpu_batch_status_previous(heifgpu_ctx *ctx, heifgpu_batch *batch, uint32_t *status, size_t cap,
                                  size_t *n_prev, void *stream);
/* HEIFGPU_ABI_VERSION of the library.  Call this first: a caller built
 * against another version (e.g. ABI 3's 16-byte heifgpu_batch_opts) must not
 * call the other entry points.  ABI 6: HEIFGPU_PARSE_ROWS removed; a reload
 * that fails no longer costs heifgpu_batch_status_previous the last good
 * load's status. */
int heifgpu_abi_version(void);
void heifgpu_batch_free(heifgpu_batch *batch);
/* stage timing (ms per decode call, from HIP events on the streams the
 * kernels run on, enabled with heifgpu_set_timing(ctx, 1)): the mean over the
 * decode calls since the previous query (or since timing was enabled) of
 * parse, transform, intra, deblock, sao/output, and (last) the
 * emulation-prevention pass k_rbsp; the query resets the mean.  k_rbsp and
 * k_parse run on an internal parse stream, k_transform on an internal
 * transform stream and the rest on an internal recon stream, over three sets
 * of parse outputs, so decode n+2's parse, decode n+1's transform and decode
 * n's reconstruction overlap (HEIFGPU_PIPELINE=2: two sets, the transform on
 * the recon stream). */
int heifgpu_set_timing(heifgpu_ctx *ctx, int enable);
int heifgpu_stage_times(heifgpu_ctx *ctx, float ms[6]);
/* convenience: prepare + decode + status + free */
int heifgpu_decode_batch(heifgpu_ctx *ctx, const heifgpu_image *const *imgs, size_t n, const heifgpu_planes *out,
                         void *stream, uint32_t *status);

/* Gather of a tile split: copies the visible windows of the grid tiles k with
 * k % tile_stride == tile_offset from `src` (planes decoded by a batch with
 * those options) into `dst` (full-size planes) with one kernel launch on
 * `stream`, a stream of dst's device.  src may live on another device: a
 * pointer of this process (peer access is enabled here) or a peer process's
 * planes mapped with heifgpu_ipc_open; the kernel reads them over xGMI.
 * Ordering: the copy reads src when it runs on `stream`, so the caller must
 * order `stream` after the decode that wrote src (synchronise that decode, or
 * make `stream` wait for an event recorded after it; across processes, the
 * owner synchronises before it signals the gathering process).  `info`
 * describes the image (heifgpu_image_get_info). */
int heifgpu_gather_tiles(const heifgpu_image_info *info, const heifgpu_planes *dst, const heifgpu_planes *src,
                         uint32_t tile_stride, uint32_t tile_offset, void *stream);

/* Cross-process device memory (the tile split with one process per GPU):
 * heifgpu_ipc_export describes the device allocation holding `dev_ptr` (a HIP
 * IPC handle plus the pointer's offset in it); another process passes the
 * 72 bytes (e.g. over torch.distributed) to heifgpu_ipc_open, which maps the
 * allocation on `device` and returns the same byte's address there.
 * heifgpu_ipc_close unmaps a pointer heifgpu_ipc_open returned.  The owner
 * must keep the allocation alive until every importer has closed it. */
typedef struct {
    uint8_t handle[64];  /* hipIpcMemHandle_t */
    uint64_t offset;     /* dev_ptr - allocation base */
} heifgpu_ipc_handle;
int heifgpu_ipc_export(const void *dev_ptr, heifgpu_ipc_handle *out);
int heifgpu_ipc_open(int device, const heifgpu_ipc_handle *h, void **dev_ptr);
int heifgpu_ipc_close(void *dev_ptr);

/* ---- YCbCr -> RGB with the irot rotation (libheif's default output) -------
 * Converts one decoded image (planes as written by heifgpu_batch_decode,
 * `info` from heifgpu_image_get_info) into interleaved 8-bit R,G,B at `rgb`
 * (device, caller-owned, rgb_pitch bytes per row), rotated anticlockwise by
 * info->rotation * 90 degrees: the output is height x width for rotation 1
 * and 3.  Matrix from info->matrix_coeffs (H.273: 1 BT.709, 9 BT.2020 NCL,
 * anything else BT.601), range from info->full_range, 4:2:0 / 4:2:2 chroma by
 * sample replication, samples above 8 bits rounded down to 8.  Fixed point: 16
 * fractional bits, round half up, clip to 0..255.  Asynchronous on `stream`. */
int heifgpu_ycbcr_to_rgb(heifgpu_ctx *ctx, const heifgpu_image_info *info, const heifgpu_planes *in, void *rgb,
                         int32_t rgb_pitch, void *stream);

/* ---- host test hooks (reference unit-test surface) -------------------- */
size_t heifgpu_remove_emulation_prevention(const uint8_t *in, size_t n, uint8_t *out); /* rbsp_reader.rs:11-39 */
int heifgpu_read_ue(const uint8_t *buf, size_t n, uint32_t *val);                      /* rbsp_reader.rs:87-99 */
int heifgpu_read_se(const uint8_t *buf, size_t n, int32_t *val);                       /* rbsp_reader.rs:101-113 */
/* the kernels' binarizations (cabac/decoder.rs:152-261) over explicit bins;
 * return the value (or -1 on underrun), *used = bins consumed */
int heifgpu_bins_truncated_rice(const uint8_t *bins, int n, int c_max, int c_rice, int *used);
int heifgpu_bins_chroma_pred_mode(const uint8_t *bins, int n, int *used);
int heifgpu_bins_coeff_abs_level_remaining(const uint8_t *bins, int n, int c_rice, int *used);
int heifgpu_bins_exp_golomb(const uint8_t *bins, int n, int k, int *used);

/* parsed parameter sets + slice header of one tile (grammar.rs:224-572;
 * the values SURVEY Appendix A lists for halfmoonbay) */
typedef struct {
    int32_t nal_unit_type, slice_type, first_slice_segment_in_pic;
    int32_t general_profile_idc, general_level_idc;
    int32_t pic_width, pic_height, chroma_format_idc, bit_depth_luma, bit_depth_chroma;
    int32_t log2_max_poc_lsb, log2_min_cb, log2_ctb, log2_min_tb, log2_max_tb;
    int32_t max_th_depth_inter, max_th_depth_intra;
    int32_t scaling_list_enabled, amp, sao, pcm, num_short_term_ref_pic_sets, long_term_refs;
    int32_t temporal_mvp, strong_intra_smoothing;
    int32_t video_full_range, colour_primaries, transfer_characteristics, matrix_coeffs;
    int32_t init_qp, sign_data_hiding, cabac_init_present, constrained_intra_pred, transform_skip;
    int32_t cu_qp_delta_enabled, diff_cu_qp_delta_depth, cb_qp_offset, cr_qp_offset;
    int32_t slice_chroma_qp_offsets_present, transquant_bypass, tiles_enabled, entropy_coding_sync;
    int32_t loop_filter_across_slices, deblocking_control_present, deblocking_override_enabled;
    int32_t deblocking_disabled, beta_offset_div2, tc_offset_div2, log2_parallel_merge_level;
    int32_t slice_sao_luma, slice_sao_chroma, slice_qp_y, num_entry_point_offsets;
    int32_t slice_data_raw_offset, payload_bytes;
    uint32_t entry_point_offset[64]; /* offset_minus1 + 1 (raw bytes), first 64 */
} heifgpu_tile_params;
int heifgpu_image_tile_params(const heifgpu_image *img, uint32_t tile, heifgpu_tile_params *out);

/* ---- tuning hook ------------------------------------------------------ */
/* k_parse_lanes counters (s_memtime cycles: whole wave, passes, per unit
 * kind CTU / tree / TB / sub-block / CTU end; lanes that ran a unit),
 * summed over waves since the last call, then reset.  Returns the number of
 * counters written, or 0 for the product build (counters compiled out; the
 * `make prof` library has them). */
int heifgpu_debug_counters(uint64_t *out, int n);
/* The CABAC parse geometry a prepared batch launches: mode
 * (HEIFGPU_PARSE_LANES / _SOLO / _SPREAD), workgroups (waves in lanes mode,
 * pictures in solo mode, substreams in spread mode), pictures per wave (lanes)
 * and waves per workgroup (solo). */
int heifgpu_batch_parse_geometry(const heifgpu_batch *batch, uint32_t *mode, uint32_t *workgroups,
                                 uint32_t *pics_per_wave, uint32_t *waves_per_workgroup);

#ifdef __cplusplus
}
#endif
#endif
