// desc.hpp — descriptors shared by the C++ host and the gfx950 kernels.
//
// The host (heif_amd/csrc/host) parses the container, VPS/SPS/PPS and slice
// headers (reference: src/heif/reader.rs, src/hevc/parameter_set_reader.rs,
// src/hevc/slice.rs:44-204) and flattens a batch of pictures into these
// plain structs; the kernels (heif_amd/csrc/kernels) own everything from
// slice_segment_data() on (reference: src/hevc/slice.rs:206-256 and the
// todo!()s it leaves).
#pragma once
#include <stdint.h>

namespace hg {

// SeqParams.flags
enum : uint32_t {
    SP_SCALING_LIST = 1u << 0,
    SP_SIGN_HIDING = 1u << 1,
    SP_TRANSFORM_SKIP = 1u << 2,
    SP_TQ_BYPASS = 1u << 3,
    SP_CU_QP_DELTA = 1u << 4,
    SP_WPP = 1u << 5,
    SP_STRONG_INTRA = 1u << 6,
    SP_PCM = 1u << 7,
    SP_PCM_LOOP_FILTER_DISABLED = 1u << 8,
    SP_SAO = 1u << 9,
    // one HEVC tile of a tiled picture decoded as its own picture (batch.cpp),
    // not the last tile: its substream ends in end_of_slice_segment_flag 0 and
    // end_of_subset_one_bit 1 (7.3.8.1)
    SP_SUBSET_END = 1u << 10,
    // several slice segments in the picture, each starting at a CTB row: the
    // substream table has one entry per CTB row (SUB_* flags below)
    SP_ROW_SEGMENTS = 1u << 11,
};

// substream table entries (PicDesc::sub_first..): raw offset | flags.  With
// SP_ROW_SEGMENTS, SUB_SEG_END marks a row whose last CTU ends a slice segment
// (end_of_slice_segment_flag = 1), and SUB_CONTINUE a row of a picture without
// WPP that starts no substream of its own (the segment's engine runs on).
enum : uint32_t {
    SUB_OFFSET = 0x3fffffffu,
    SUB_CONTINUE = 1u << 30,
    SUB_SEG_END = 1u << 31,
};

// Per distinct SPS/PPS pair (derived values only; H.265 7.4.3.2 / 7.4.3.3).
struct SeqParams {
    int32_t width, height;        // pic_width/height_in_luma_samples
    int32_t log2_ctb, log2_min_cb, log2_min_tb, log2_max_tb;
    int32_t max_th_depth_intra;
    int32_t chroma_format;        // chroma_format_idc: 0 (4:0:0), 1 (4:2:0), 2 (4:2:2), 3 (4:4:4)
    int32_t bit_depth_y, bit_depth_c;
    uint32_t flags;
    int32_t diff_cu_qp_delta_depth;
    int32_t cb_qp_offset, cr_qp_offset;
    int32_t log2_min_pcm, log2_max_pcm, pcm_bd_y, pcm_bd_c;
    int32_t conf_l, conf_t;       // luma samples
    int32_t out_w, out_h;         // conformance-cropped size
    uint32_t sf_off;              // byte offset of this set's ScalingFactor block
    int32_t pad[3];
};

// log2 SubWidthC / SubHeightC of a chroma_format_idc (Table 6-1): a W x H
// picture's chroma planes are (W >> chroma_sx) x (H >> chroma_sy)
constexpr int chroma_sx(int fmt) { return fmt == 1 || fmt == 2 ? 1 : 0; }
constexpr int chroma_sy(int fmt) { return fmt == 1 ? 1 : 0; }

// Scaling factor block layout (bytes, from sf_off): for sizeId 0..3 and
// matrixId 0..5, n*n factors m[y*n+x] (n = 4<<sizeId), in this order.
constexpr uint32_t sf_size_offset(int size_id) {
    return size_id == 0 ? 0u : size_id == 1 ? 6u * 16u : size_id == 2 ? 6u * (16u + 64u) : 6u * (16u + 64u + 256u);
}
constexpr uint32_t kSfBlockBytes = 6u * (16u + 64u + 256u + 1024u);

// One coded picture (= one HEIF grid tile, or a single-item image).
struct PicDesc {
    uint64_t bits_off;    // byte offset of the NAL payload (after the 2-byte NAL header)
    uint32_t bits_len;    // payload bytes (raw, EP bytes included)
    uint32_t sub_first;   // first entry in the substream table
    uint32_t n_sub;       // number of substreams (num_entry_point_offsets + 1)
    uint32_t seq;         // SeqParams index
    int32_t slice_qp, cb_qp_off, cr_qp_off;
    int32_t sao_luma, sao_chroma, dbk_disabled, beta_off, tc_off;
    uint32_t image;       // output image index
    int32_t out_x, out_y; // luma position of the cropped picture in the output image
    // work-arena offsets
    uint64_t recon_off;   // bytes: Y (width*height samples), then Cb, Cr
    uint64_t resid_off;   // int16 elements: same layout as recon
    uint64_t map_off;     // bytes: qpy[w4*h4], flags[w4*h4], then bottom CtDepth per CTB row [hctb][w8]
    uint64_t sao_off;     // SaoParams index of CTB 0
    uint64_t tu_off;      // TuRec index of row 0 (row r at tu_off + r*tu_cap_row)
    uint64_t coef_off;    // Coef index of row 0
    uint32_t row_off;     // index of row 0 in the per-row counters
    uint32_t tu_cap_row, coef_cap_row;
    uint32_t flags;       // PD_*
    // A picture whose HEVC tiles / slices are filtered across their boundaries
    // is decoded as sub-pictures (PD_CHILD: parse, transform and intra
    // prediction only) put together into an assembly picture (PD_ASSEMBLY: no
    // coded data; k_assemble copies its children's samples, QP / edge maps and
    // SAO parameters in, then deblocking and SAO + output run on it whole).
    int32_t org_x, org_y;     // PD_CHILD: luma position in its assembly
    uint32_t child0, nchild;  // PD_ASSEMBLY: its children are pictures [child0, child0 + nchild)
};

enum : uint32_t {
    PD_CHILD = 1u << 0,
    PD_ASSEMBLY = 1u << 1,
    // bits 16-30: SP_ROW_SEGMENTS, the dependent slice segments starting inside a
    // CTB row (their data offsets follow the end entry of the substream table, then
    // with WPP one count per row of those starting in earlier rows; in flags, so
    // PicDesc and the parse's LanePic keep their layout)
    PD_NMID_SHIFT = 16,
    PD_NMID_MAX = 0x7fffu,
};

struct OutImage {
    uint64_t plane[3];    // device pointers (caller-owned)
    int32_t pitch[3];     // bytes
    int32_t width, height;// output (cropped grid) size in luma samples
};

// TuRec.flags
enum : uint8_t {
    TU_CIDX_MASK = 3,
    TU_CBF = 1u << 2,
    TU_TSKIP = 1u << 3,
    TU_BYPASS = 1u << 4,
    TU_DST = 1u << 5,
    TU_PCM = 1u << 6,     // pcm_sample(): the "coefficients" are the samples (BYPASS is set too)
};

// One transform block in decoding order (luma or chroma), written by the
// parse kernel, consumed by the transform and intra kernels.
struct TuRec {
    uint16_t x, y;        // top-left in component samples
    uint8_t log2;         // TB size (component)
    uint8_t flags;        // cIdx | TU_*
    uint8_t mode;         // IntraPredModeY / IntraPredModeC
    uint8_t qp;           // qP (Qp'Y / Qp'Cb / Qp'Cr) for scaling
    uint32_t coef;        // first Coef index
    uint16_t ncoef;       // nonzero coefficients
    uint16_t ctu;         // CTU column this TB belongs to
};
static_assert(sizeof(TuRec) == 16, "TuRec layout");

// Coefficient words of a TB.  A coded TB is a run of 16-byte sub-block
// records (SbRec: TuRec.coef = its first word, TuRec.ncoef = 4 x records),
// in decoding order:
//   w0: significance by scan position n (bit n) | the sign bins in decoding
//       order (descending n) from bit 31 down;
//   w1, w2: abs - 1 per scan position n as nibble n (15: escape, the level is
//       in the row's escape list);
//   w3: xS (3 bits) | yS << 3 (3) | scanIdx << 6 (2) | sign hidden << 8 |
//       row-relative word index of the record's first escape << 9 (its later
//       escapes, in descending n, at the indices below it: the escape list
//       grows down from the end of the row's coefficient space).
// The sign of a position of rank r (significant positions above it) is bit
// 31 - r of w0, except the lowest significant position when the sign is
// hidden: the parity of the sub-block's sum of levels (7.4.9.11).
// A PCM TB (TU_PCM) instead holds one word per sample: value << 16 | raster
// position.
typedef uint32_t Coef;

// SAO parameters of one CTB (7.3.8.3 semantics, SaoOffsetVal already signed).
struct alignas(4) SaoParams {
    int8_t type[3];       // SaoTypeIdx
    uint8_t band_eo[3];   // sao_band_position or SaoEoClass
    int16_t off[3][4];    // SaoOffsetVal[1..4]
    int16_t pad;          // 32 bytes: word-aligned for k_parse_lanes' L1-bypassing reads
};
static_assert(sizeof(SaoParams) == 32, "SaoParams layout");

// Per-picture status word bits (kernels OR these in).
enum : uint32_t {
    ST_OK = 0,
    ST_CABAC_INIT = 1u << 0,      // ivlOffset 510/511
    ST_SUBSTREAM_END = 1u << 1,   // end_of_subset_one_bit / end_of_slice_segment_flag mismatch
    ST_OVERRUN = 1u << 2,         // read past substream
    ST_SYNTAX = 1u << 3,          // out-of-range syntax element
    ST_UNSUPPORTED = 1u << 4,     // pcm_flag = 1 etc.
    ST_CAPACITY = 1u << 5,        // TU/coef row capacity exceeded
};

// map flags (per 4x4 luma block)
enum : uint8_t {
    MF_EDGE_V = 1,   // left edge of the block is a transform/prediction block edge
    MF_EDGE_H = 2,   // top edge is
    MF_NOFILT = 4,   // cu_transquant_bypass (or PCM with loop filter disabled)
};

}  // namespace hg
