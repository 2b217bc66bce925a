// hevc_ps.hpp — HEVC high-level syntax on the host.
// Mirrors src/hevc/parameter_set_reader.rs (video/sequence/picture_parameter_set_rbsp
// :7,36,351), src/hevc/grammar.rs (NalUnitHeader :349-369, SequenceParameterSet
// :387-508, PictureParameterSet :510-548, SliceSegmentHeader :550-572) and the
// I-slice header of src/hevc/slice.rs:44-204.  Unlike the reference it keeps
// the scaling lists (+ Table 7-5/7-6 defaults), the tile sizes, parses
// st_ref_pic_set / HRD / range-extension flags, and locates WPP entry points
// in raw NAL bytes.
#pragma once
#include <array>
#include <cstdint>
#include <vector>

#include "rbsp.hpp"

namespace hg {

struct NalUnitHeader {  // grammar.rs:349-369
    uint16_t raw = 0;
    int nal_unit_type() const { return (raw >> 9) & 63; }
    int nuh_layer_id() const { return (raw >> 3) & 63; }
    int temporal_id_plus1() const { return raw & 7; }
};

struct ScalingLists {
    // ScalingList[sizeId][matrixId][i] in coded (up-right diagonal) order, + DC
    std::array<std::array<std::array<uint8_t, 64>, 6>, 4> list{};
    std::array<std::array<int, 6>, 4> dc{};
    void set_default();
    // ScalingFactor m[y*n+x] for sizeId/matrixId (7.4.5)
    void factors(int size_id, int matrix_id, uint8_t *out) const;
};

struct VideoParameterSet {
    int vps_id = 0, max_layers_minus1 = 0, max_sub_layers_minus1 = 0;
    int general_profile_idc = 0, general_level_idc = 0;
};

struct SequenceParameterSet {
    int sps_id = 0, vps_id = 0, max_sub_layers_minus1 = 0;
    int general_profile_idc = 0, general_level_idc = 0;
    int chroma_format_idc = 1;
    bool separate_colour_plane_flag = false;
    int pic_width_in_luma_samples = 0, pic_height_in_luma_samples = 0;
    int conf_win_left = 0, conf_win_right = 0, conf_win_top = 0, conf_win_bottom = 0;  // luma samples
    int bit_depth_luma_minus8 = 0, bit_depth_chroma_minus8 = 0;
    int log2_max_pic_order_cnt_lsb = 4;
    int log2_min_luma_coding_block_size = 3, log2_ctb_size = 4;
    int log2_min_tb_size = 2, log2_max_tb_size = 5;
    int max_transform_hierarchy_depth_inter = 0, max_transform_hierarchy_depth_intra = 0;
    bool scaling_list_enabled_flag = false;
    ScalingLists scaling;
    bool amp_enabled_flag = false, sample_adaptive_offset_enabled_flag = false;
    bool pcm_enabled_flag = false, pcm_loop_filter_disabled_flag = false;
    int pcm_bit_depth_luma = 0, pcm_bit_depth_chroma = 0, log2_min_pcm = 0, log2_max_pcm = 0;
    int num_short_term_ref_pic_sets = 0;
    std::vector<int> st_rps_num_delta_pocs;
    bool long_term_ref_pics_present_flag = false;
    int num_long_term_ref_pics_sps = 0;
    bool sps_temporal_mvp_enabled_flag = false, strong_intra_smoothing_enabled_flag = false;
    // VUI colour (grammar.rs VUI enums)
    bool video_full_range_flag = false;
    int colour_primaries = 2, transfer_characteristics = 2, matrix_coeffs = 2;
    bool range_extension_tools = false;

    int chroma_array_type() const { return separate_colour_plane_flag ? 0 : chroma_format_idc; }
    int pic_width_in_ctbs_y() const { return (pic_width_in_luma_samples + (1 << log2_ctb_size) - 1) >> log2_ctb_size; }
    int pic_height_in_ctbs_y() const { return (pic_height_in_luma_samples + (1 << log2_ctb_size) - 1) >> log2_ctb_size; }
    int out_width() const { return pic_width_in_luma_samples - conf_win_left - conf_win_right; }
    int out_height() const { return pic_height_in_luma_samples - conf_win_top - conf_win_bottom; }
};

struct PictureParameterSet {
    int pps_id = 0, sps_id = 0;
    bool dependent_slice_segments_enabled_flag = false, output_flag_present_flag = false;
    int num_extra_slice_header_bits = 0;
    bool sign_data_hiding_enabled_flag = false, cabac_init_present_flag = false;
    int init_qp_minus26 = 0;
    bool constrained_intra_pred_flag = false, transform_skip_enabled_flag = false;
    bool cu_qp_delta_enabled_flag = false;
    int diff_cu_qp_delta_depth = 0;
    int pps_cb_qp_offset = 0, pps_cr_qp_offset = 0;
    bool pps_slice_chroma_qp_offsets_present_flag = false;
    bool transquant_bypass_enabled_flag = false, tiles_enabled_flag = false, entropy_coding_sync_enabled_flag = false;
    int num_tile_columns = 1, num_tile_rows = 1;
    std::vector<int> column_widths, row_heights;  // kept (reference drops them, :393-400)
    bool uniform_spacing_flag = true, loop_filter_across_tiles_enabled_flag = false;
    bool pps_loop_filter_across_slices_enabled_flag = false;
    bool deblocking_filter_control_present_flag = false;
    bool deblocking_filter_override_enabled_flag = false, pps_deblocking_filter_disabled_flag = false;
    int pps_beta_offset_div2 = 0, pps_tc_offset_div2 = 0;
    bool pps_scaling_list_data_present_flag = false;
    ScalingLists scaling;  // effective lists (PPS, else SPS)
    bool lists_modification_present_flag = false;
    int log2_parallel_merge_level = 2;
    bool slice_segment_header_extension_present_flag = false;
    bool range_extension_tools = false;
};

struct SliceSegmentHeader {  // grammar.rs:550-572 + entry points in raw bytes
    bool first_slice_segment_in_pic_flag = true;
    bool dependent_slice_segment_flag = false;
    uint32_t slice_segment_address = 0;  // first CTB, raster scan
    bool slice_loop_filter_across_slices_enabled_flag = false;
    int slice_pic_parameter_set_id = 0;
    int slice_type = 2;
    bool slice_sao_luma_flag = false, slice_sao_chroma_flag = false;
    int slice_qp_delta = 0, slice_cb_qp_offset = 0, slice_cr_qp_offset = 0;
    bool slice_deblocking_filter_disabled_flag = false;
    int slice_beta_offset_div2 = 0, slice_tc_offset_div2 = 0;
    int num_entry_point_offsets = 0;
    std::vector<uint32_t> entry_point_offset;  // offset_minus1 + 1, raw bytes
    uint32_t slice_data_raw_offset = 0;        // raw payload byte where slice_segment_data() starts
};

// 6.5.1 (6-3..6-6): tile column / row boundaries in CTBs, num + 1 entries
// each ({0, PicWidthInCtbsY} without tiles).  Throws HeifError when explicit
// sizes leave no CTB for the last column / row.
void tile_boundaries(const SequenceParameterSet &sps, const PictureParameterSet &pps, std::vector<int> &col_bd,
                     std::vector<int> &row_bd);

VideoParameterSet video_parameter_set_rbsp(const std::vector<uint8_t> &rbsp);
SequenceParameterSet sequence_parameter_set_rbsp(const std::vector<uint8_t> &rbsp);
PictureParameterSet picture_parameter_set_rbsp(const std::vector<uint8_t> &rbsp, const SequenceParameterSet &sps);

// Parses the I-slice header of a VCL NAL payload (raw bytes after the 2-byte
// NAL header, EP bytes included) — slice.rs:44-204, which takes the first
// segment of a picture only (slice.rs:61-64); a later segment's address and
// dependent flag are read here too (a dependent segment's other fields are
// its slice's, left at their defaults).
SliceSegmentHeader slice_segment_header(const uint8_t *payload, size_t len, NalUnitHeader nal,
                                        const SequenceParameterSet &sps, const PictureParameterSet &pps);

struct HevcConfig {  // HEVCDecoderConfigurationRecord (grammar.rs:156-221)
    int length_size_minus_one = 3;
    std::vector<std::vector<uint8_t>> vps, sps, pps;  // raw NAL units incl. header
};
HevcConfig parse_hvcc(const uint8_t *p, size_t n);

}  // namespace hg
