// hevc_ps.cpp — see hevc_ps.hpp.
#include "hevc_ps.hpp"

#include <algorithm>
#include <cstring>

namespace hg {

std::vector<uint8_t> RbspReader::remove_emulation_prevention(const uint8_t *in, size_t n, std::vector<uint32_t> *ep_raw) {
    std::vector<uint8_t> out;
    out.reserve(n);
    size_t i = 0;
    while (i < n) {
        const uint8_t *z = static_cast<const uint8_t *>(memchr(in + i, 0, n - i));
        if (!z) {
            out.insert(out.end(), in + i, in + n);
            break;
        }
        size_t zp = size_t(z - in);
        out.insert(out.end(), in + i, in + zp);
        out.push_back(0);
        if (zp + 2 < n && in[zp + 1] == 0 && in[zp + 2] == 3 && (zp + 3 >= n || in[zp + 3] <= 3)) {
            out.push_back(0);
            if (ep_raw) ep_raw->push_back(uint32_t(zp + 2));
            i = zp + 3;
        } else {
            i = zp + 1;
        }
    }
    return out;
}

namespace {

// 6.5.3 up-right diagonal scan of an 8x8 / 4x4 block: (x, y) for position i
void diag_scan(int blk, int *xs, int *ys) {
    int i = 0, x = 0, y = 0;
    while (i < blk * blk) {
        while (y >= 0) {
            if (x < blk && y < blk) {
                xs[i] = x;
                ys[i] = y;
                ++i;
            }
            --y;
            ++x;
        }
        y = x;
        x = 0;
    }
}

// Table 7-6, raster order (the matrices are symmetric)
const uint8_t kIntra8[64] = {16, 16, 16, 16, 17, 18, 21, 24, 16, 16, 16, 16, 17, 19, 22, 25, 16, 16, 17, 18, 20, 22,
                             25, 29, 16, 16, 18, 21, 24, 27, 31, 36, 17, 17, 20, 24, 30, 35, 41, 47, 18, 19, 22, 27,
                             35, 44, 54, 65, 21, 22, 25, 31, 41, 54, 70, 88, 24, 25, 29, 36, 47, 65, 88, 115};
const uint8_t kInter8[64] = {16, 16, 16, 16, 17, 18, 20, 24, 16, 16, 16, 17, 18, 20, 24, 25, 16, 16, 17, 18, 20, 24,
                             25, 28, 16, 17, 18, 20, 24, 25, 28, 33, 17, 18, 20, 24, 25, 28, 33, 41, 18, 20, 24, 25,
                             28, 33, 41, 54, 20, 24, 25, 28, 33, 41, 54, 71, 24, 25, 28, 33, 41, 54, 71, 91};

void default_list(int size_id, int matrix_id, std::array<uint8_t, 64> &l, int &dc) {
    if (size_id == 0) {
        l.fill(16);
    } else {
        int xs[64], ys[64];
        diag_scan(8, xs, ys);
        const uint8_t *m = matrix_id < 3 ? kIntra8 : kInter8;
        for (int i = 0; i < 64; ++i) l[i] = m[ys[i] * 8 + xs[i]];
    }
    dc = 16;
}

// 7.3.4 scaling_list_data()
void scaling_list_data(RbspReader &r, ScalingLists &s) {
    for (int size_id = 0; size_id < 4; ++size_id) {
        int step = size_id == 3 ? 3 : 1;
        for (int mid = 0; mid < 6; mid += step) {
            bool pred_mode = r.read_flag();
            int coef_num = std::min(64, 1 << (4 + (size_id << 1)));
            if (!pred_mode) {
                int delta = r.read_ue_max(5, "scaling_list_pred_matrix_id_delta");
                if (delta == 0) {
                    default_list(size_id, mid, s.list[size_id][mid], s.dc[size_id][mid]);
                } else {
                    int ref = mid - delta * step;
                    if (ref < 0) throw HeifError("scaling_list_pred_matrix_id_delta out of range");
                    s.list[size_id][mid] = s.list[size_id][ref];
                    s.dc[size_id][mid] = s.dc[size_id][ref];
                }
            } else {
                int next = 8;
                if (size_id > 1) {
                    next = r.read_se_range(-7, 247, "scaling_list_dc_coef_minus8") + 8;
                    s.dc[size_id][mid] = next;
                }
                for (int i = 0; i < coef_num; ++i) {
                    next = (next + r.read_se_range(-128, 127, "scaling_list_delta_coef") + 256) % 256;
                    s.list[size_id][mid][i] = uint8_t(next);
                }
                if (size_id <= 1) s.dc[size_id][mid] = 16;
            }
        }
    }
    for (int mid : {1, 2, 4, 5}) {  // 32x32 chroma (4:4:4 only) follows 16x16
        s.list[3][mid] = s.list[2][mid];
        s.dc[3][mid] = s.dc[2][mid];
    }
}

// 7.3.3 profile_tier_level(1, maxNumSubLayersMinus1)
void profile_tier_level(RbspReader &r, int max_sub_minus1, int *profile_idc, int *level_idc) {
    r.read_bits(3);
    *profile_idc = int(r.read_bits(5));
    r.read_bits(32);
    r.read_bits(16);
    r.read_bits(32);  // 4 source flags + 43 constraint bits + 1 = 48 bits total
    *level_idc = int(r.read_bits(8));
    bool spp[8] = {}, slp[8] = {};
    for (int i = 0; i < max_sub_minus1; ++i) {
        spp[i] = r.read_flag();
        slp[i] = r.read_flag();
    }
    if (max_sub_minus1 > 0)
        for (int i = max_sub_minus1; i < 8; ++i) r.read_bits(2);
    for (int i = 0; i < max_sub_minus1; ++i) {
        if (spp[i]) r.skip_bits(88);
        if (slp[i]) r.skip_bits(8);
    }
}

void sub_layer_hrd(RbspReader &r, int cpb_cnt, bool sub_pic) {
    for (int j = 0; j <= cpb_cnt; ++j) {
        r.read_ue();
        r.read_ue();
        if (sub_pic) {
            r.read_ue();
            r.read_ue();
        }
        r.read_flag();
    }
}

// E.2.2 hrd_parameters (the reference's stub at :338-349 is incomplete)
void hrd_parameters(RbspReader &r, bool common, int max_sub_minus1) {
    bool nal = false, vcl = false, sub_pic = false;
    if (common) {
        nal = r.read_flag();
        vcl = r.read_flag();
        if (nal || vcl) {
            sub_pic = r.read_flag();
            if (sub_pic) r.read_bits(8 + 5 + 1 + 5);
            r.read_bits(8);
            if (sub_pic) r.read_bits(4);
            r.read_bits(15);
        }
    }
    for (int i = 0; i <= max_sub_minus1; ++i) {
        bool fixed_general = r.read_flag();
        bool fixed_cvs = fixed_general ? true : r.read_flag();
        bool low_delay = false;
        if (fixed_cvs) r.read_ue();
        else low_delay = r.read_flag();
        int cpb_cnt = low_delay ? 0 : int(r.read_ue());
        if (nal) sub_layer_hrd(r, cpb_cnt, sub_pic);
        if (vcl) sub_layer_hrd(r, cpb_cnt, sub_pic);
    }
}

// E.2.1 vui_parameters (parameter_set_reader.rs:252-336)
void vui_parameters(RbspReader &r, SequenceParameterSet &s) {
    if (r.read_flag() && r.read_bits(8) == 255) r.read_bits(32);
    if (r.read_flag()) r.read_flag();
    if (r.read_flag()) {
        r.read_bits(3);
        s.video_full_range_flag = r.read_flag();
        if (r.read_flag()) {
            s.colour_primaries = int(r.read_bits(8));
            s.transfer_characteristics = int(r.read_bits(8));
            s.matrix_coeffs = int(r.read_bits(8));
        }
    }
    if (r.read_flag()) {
        r.read_ue();
        r.read_ue();
    }
    r.read_bits(3);
    if (r.read_flag())
        for (int i = 0; i < 4; ++i) r.read_ue();
    if (r.read_flag()) {
        r.read_bits(32);
        r.read_bits(32);
        if (r.read_flag()) r.read_ue();
        if (r.read_flag()) hrd_parameters(r, true, s.max_sub_layers_minus1);
    }
    if (r.read_flag()) {
        r.read_bits(3);
        for (int i = 0; i < 5; ++i) r.read_ue();
    }
}

// 7.3.7 st_ref_pic_set — keeps NumDeltaPocs only (reference skips it, :225-250)
void st_ref_pic_set(RbspReader &r, int idx, int num_sets, std::vector<int> &num_delta) {
    bool inter = idx != 0 && r.read_flag();
    if (inter) {
        int delta_idx = idx == num_sets ? r.read_ue_max(uint32_t(idx - 1), "delta_idx_minus1") + 1 : 1;
        int ref = idx - delta_idx;
        if (ref < 0) throw HeifError("st_ref_pic_set: bad delta_idx");
        r.read_flag();
        r.read_ue();
        int cnt = 0;
        for (int j = 0; j <= num_delta[size_t(ref)]; ++j) {
            bool used = r.read_flag();
            bool use_delta = used ? true : r.read_flag();
            if (used || use_delta) ++cnt;
        }
        num_delta[size_t(idx)] = cnt;
    } else {
        int neg = r.read_ue_max(16, "num_negative_pics"), pos = r.read_ue_max(16, "num_positive_pics");
        if (neg > 16 || pos > 16) throw HeifError("st_ref_pic_set: too many pictures");
        for (int i = 0; i < neg + pos; ++i) {
            r.read_ue();
            r.read_flag();
        }
        num_delta[size_t(idx)] = neg + pos;
    }
}

int ceil_log2(int v) {
    int b = 0;
    while ((1 << b) < v) ++b;
    return b;
}

}  // namespace

void ScalingLists::set_default() {
    for (int s = 0; s < 4; ++s)
        for (int m = 0; m < 6; ++m) default_list(s, m, list[s][m], dc[s][m]);
}

void ScalingLists::factors(int size_id, int matrix_id, uint8_t *out) const {
    int n = 4 << size_id;
    if (size_id == 0) {
        int xs[16], ys[16];
        diag_scan(4, xs, ys);
        for (int i = 0; i < 16; ++i) out[ys[i] * 4 + xs[i]] = list[0][matrix_id][i];
        return;
    }
    int xs[64], ys[64];
    diag_scan(8, xs, ys);
    int rep = n / 8;
    for (int i = 0; i < 64; ++i)
        for (int j = 0; j < rep; ++j)
            for (int k = 0; k < rep; ++k) out[(ys[i] * rep + j) * n + xs[i] * rep + k] = list[size_id][matrix_id][i];
    if (size_id >= 2) out[0] = uint8_t(dc[size_id][matrix_id]);
}

VideoParameterSet video_parameter_set_rbsp(const std::vector<uint8_t> &rbsp) {
    RbspReader r(rbsp.data(), rbsp.size());
    VideoParameterSet v;
    v.vps_id = int(r.read_bits(4));
    r.read_bits(2);
    v.max_layers_minus1 = int(r.read_bits(6));
    v.max_sub_layers_minus1 = int(r.read_bits(3));
    r.read_flag();
    if (r.read_bits(16) != 0xffff) throw HeifError("vps_reserved_0xffff_16bits");
    profile_tier_level(r, v.max_sub_layers_minus1, &v.general_profile_idc, &v.general_level_idc);
    return v;
}

// 7.4.3.2 semantic constraints the kernels rely on (block-size ladders, PCM
// sizes, picture size in whole minimum CBs), then this path's profile limits
void validate_sps(const SequenceParameterSet &s) {
    const int min_cb = s.log2_min_luma_coding_block_size, ctb = s.log2_ctb_size;
    const int min_tb = s.log2_min_tb_size, max_tb = s.log2_max_tb_size;
    if (ctb < 4 || ctb > 6 || min_cb < 3 || min_cb > ctb) throw HeifError("SPS coding block sizes out of range");
    if (min_tb < 2 || min_tb >= min_cb || max_tb > 5 || max_tb > ctb)
        throw HeifError("SPS transform block sizes out of range");
    if (s.max_transform_hierarchy_depth_intra > ctb - min_tb || s.max_transform_hierarchy_depth_inter > ctb - min_tb)
        throw HeifError("max_transform_hierarchy_depth out of range");
    if (s.pic_width_in_luma_samples <= 0 || s.pic_height_in_luma_samples <= 0 ||
        (s.pic_width_in_luma_samples & ((1 << min_cb) - 1)) || (s.pic_height_in_luma_samples & ((1 << min_cb) - 1)))
        throw HeifError("picture size is not a multiple of MinCbSizeY");
    if (s.pcm_enabled_flag &&
        (s.log2_max_pcm > (ctb < 5 ? ctb : 5) || s.log2_min_pcm < (min_cb < 5 ? min_cb : 5) ||
         s.pcm_bit_depth_luma > 8 + s.bit_depth_luma_minus8 ||
         s.pcm_bit_depth_chroma > 8 + s.bit_depth_chroma_minus8))
        throw HeifError("PCM parameters out of range");
    // up to 12 bits (Main 12 / RExt 12-bit profiles): without extended_precision_processing
    // (a range-extension tool, rejected) the coefficients keep 16 bits and a residual
    // clipped to int16 still reconstructs exactly for sample depths below 16; parity-tested
    // at 8..12 bits (tests/test_synth.py)
    if (s.bit_depth_luma_minus8 > 4 || s.bit_depth_chroma_minus8 > 4)
        throw UnsupportedError("bit depth above 12 (only 8..12-bit streams are parity-tested on this path)");
}

SequenceParameterSet sequence_parameter_set_rbsp(const std::vector<uint8_t> &rbsp) {
    RbspReader r(rbsp.data(), rbsp.size());
    SequenceParameterSet s;
    s.vps_id = int(r.read_bits(4));
    s.max_sub_layers_minus1 = int(r.read_bits(3));
    r.read_flag();
    profile_tier_level(r, s.max_sub_layers_minus1, &s.general_profile_idc, &s.general_level_idc);
    s.sps_id = r.read_ue_max(15, "sps_seq_parameter_set_id");
    s.chroma_format_idc = r.read_ue_max(3, "chroma_format_idc");
    if (s.chroma_format_idc == 3) s.separate_colour_plane_flag = r.read_flag();
    // 16888 = sqrt(8 * MaxLumaPs) of level 6.2 (A.4.1), the largest legal dimension
    s.pic_width_in_luma_samples = r.read_ue_max(16888, "pic_width_in_luma_samples");
    s.pic_height_in_luma_samples = r.read_ue_max(16888, "pic_height_in_luma_samples");
    int sw = (s.chroma_format_idc == 1 || s.chroma_format_idc == 2) ? 2 : 1;
    int sh = s.chroma_format_idc == 1 ? 2 : 1;
    if (r.read_flag()) {
        // 7.4.3.2: SubWidthC * (left + right) < pic_width, likewise vertically
        const uint32_t l = r.read_ue(), rt = r.read_ue(), t = r.read_ue(), b = r.read_ue();
        if (uint64_t(sw) * (uint64_t(l) + rt) >= uint64_t(s.pic_width_in_luma_samples) ||
            uint64_t(sh) * (uint64_t(t) + b) >= uint64_t(s.pic_height_in_luma_samples))
            throw HeifError("conformance window out of range");
        s.conf_win_left = int(l) * sw;
        s.conf_win_right = int(rt) * sw;
        s.conf_win_top = int(t) * sh;
        s.conf_win_bottom = int(b) * sh;
    }
    s.bit_depth_luma_minus8 = r.read_ue_max(8, "bit_depth_luma_minus8");
    s.bit_depth_chroma_minus8 = r.read_ue_max(8, "bit_depth_chroma_minus8");
    s.log2_max_pic_order_cnt_lsb = r.read_ue_max(12, "log2_max_pic_order_cnt_lsb_minus4") + 4;
    bool ordering = r.read_flag();
    for (int i = ordering ? 0 : s.max_sub_layers_minus1; i <= s.max_sub_layers_minus1; ++i) {
        r.read_ue();
        r.read_ue();
        r.read_ue();
    }
    s.log2_min_luma_coding_block_size = r.read_ue_max(3, "log2_min_luma_coding_block_size_minus3") + 3;
    s.log2_ctb_size = s.log2_min_luma_coding_block_size + r.read_ue_max(3, "log2_diff_max_min_luma_coding_block_size");
    s.log2_min_tb_size = r.read_ue_max(3, "log2_min_luma_transform_block_size_minus2") + 2;
    s.log2_max_tb_size = s.log2_min_tb_size + r.read_ue_max(3, "log2_diff_max_min_luma_transform_block_size");
    s.max_transform_hierarchy_depth_inter = r.read_ue_max(4, "max_transform_hierarchy_depth_inter");
    s.max_transform_hierarchy_depth_intra = r.read_ue_max(4, "max_transform_hierarchy_depth_intra");
    s.scaling.set_default();
    s.scaling_list_enabled_flag = r.read_flag();
    if (s.scaling_list_enabled_flag && r.read_flag()) scaling_list_data(r, s.scaling);
    s.amp_enabled_flag = r.read_flag();
    s.sample_adaptive_offset_enabled_flag = r.read_flag();
    s.pcm_enabled_flag = r.read_flag();
    if (s.pcm_enabled_flag) {
        s.pcm_bit_depth_luma = int(r.read_bits(4)) + 1;
        s.pcm_bit_depth_chroma = int(r.read_bits(4)) + 1;
        s.log2_min_pcm = r.read_ue_max(2, "log2_min_pcm_luma_coding_block_size_minus3") + 3;
        s.log2_max_pcm = s.log2_min_pcm + r.read_ue_max(2, "log2_diff_max_min_pcm_luma_coding_block_size");
        s.pcm_loop_filter_disabled_flag = r.read_flag();
    }
    s.num_short_term_ref_pic_sets = r.read_ue_max(64, "num_short_term_ref_pic_sets");
    s.st_rps_num_delta_pocs.assign(65, 0);
    for (int i = 0; i < s.num_short_term_ref_pic_sets; ++i)
        st_ref_pic_set(r, i, s.num_short_term_ref_pic_sets, s.st_rps_num_delta_pocs);
    s.long_term_ref_pics_present_flag = r.read_flag();
    if (s.long_term_ref_pics_present_flag) {
        s.num_long_term_ref_pics_sps = r.read_ue_max(32, "num_long_term_ref_pics_sps");
        for (int i = 0; i < s.num_long_term_ref_pics_sps; ++i) {
            r.read_bits(s.log2_max_pic_order_cnt_lsb);
            r.read_flag();
        }
    }
    s.sps_temporal_mvp_enabled_flag = r.read_flag();
    s.strong_intra_smoothing_enabled_flag = r.read_flag();
    if (r.read_flag()) vui_parameters(r, s);
    if (r.read_flag()) {  // sps_extension_present_flag (reference errors here, :153-158)
        bool range = r.read_flag();
        r.read_bits(3 + 4);
        if (range) s.range_extension_tools = r.read_bits(9) != 0;
    }
    validate_sps(s);
    return s;
}

PictureParameterSet picture_parameter_set_rbsp(const std::vector<uint8_t> &rbsp, const SequenceParameterSet &sps) {
    RbspReader r(rbsp.data(), rbsp.size());
    PictureParameterSet p;
    p.pps_id = r.read_ue_max(63, "pps_pic_parameter_set_id");
    p.sps_id = r.read_ue_max(15, "pps_seq_parameter_set_id");
    p.dependent_slice_segments_enabled_flag = r.read_flag();
    p.output_flag_present_flag = r.read_flag();
    p.num_extra_slice_header_bits = int(r.read_bits(3));
    p.sign_data_hiding_enabled_flag = r.read_flag();
    p.cabac_init_present_flag = r.read_flag();
    r.read_ue();
    r.read_ue();
    p.init_qp_minus26 = r.read_se();
    p.constrained_intra_pred_flag = r.read_flag();
    p.transform_skip_enabled_flag = r.read_flag();
    p.cu_qp_delta_enabled_flag = r.read_flag();
    if (p.cu_qp_delta_enabled_flag)
        p.diff_cu_qp_delta_depth = r.read_ue_max(uint32_t(sps.log2_ctb_size - sps.log2_min_luma_coding_block_size),
                                                 "diff_cu_qp_delta_depth");
    p.pps_cb_qp_offset = r.read_se_range(-12, 12, "pps_cb_qp_offset");
    p.pps_cr_qp_offset = r.read_se_range(-12, 12, "pps_cr_qp_offset");
    p.pps_slice_chroma_qp_offsets_present_flag = r.read_flag();
    r.read_flag();  // weighted_pred_flag
    r.read_flag();  // weighted_bipred_flag
    p.transquant_bypass_enabled_flag = r.read_flag();
    p.tiles_enabled_flag = r.read_flag();
    p.entropy_coding_sync_enabled_flag = r.read_flag();
    if (p.tiles_enabled_flag) {
        int nc = r.read_ue_max(19, "num_tile_columns_minus1") + 1, nr = r.read_ue_max(21, "num_tile_rows_minus1") + 1;
        if (nc > sps.pic_width_in_ctbs_y() || nr > sps.pic_height_in_ctbs_y())
            throw HeifError("more tile columns / rows than CTBs");
        p.num_tile_columns = nc;
        p.num_tile_rows = nr;
        p.uniform_spacing_flag = r.read_flag();
        if (!p.uniform_spacing_flag) {
            // bounded by the picture (7.4.3.3.1), so the boundary sums in tile_boundaries cannot overflow
            for (int i = 0; i < nc - 1; ++i)
                p.column_widths.push_back(
                    r.read_ue_max(uint32_t(sps.pic_width_in_ctbs_y() - 1), "column_width_minus1") + 1);
            for (int i = 0; i < nr - 1; ++i)
                p.row_heights.push_back(r.read_ue_max(uint32_t(sps.pic_height_in_ctbs_y() - 1), "row_height_minus1") + 1);
        }
        p.loop_filter_across_tiles_enabled_flag = r.read_flag();
    }
    p.pps_loop_filter_across_slices_enabled_flag = r.read_flag();
    p.deblocking_filter_control_present_flag = r.read_flag();
    if (p.deblocking_filter_control_present_flag) {
        p.deblocking_filter_override_enabled_flag = r.read_flag();
        p.pps_deblocking_filter_disabled_flag = r.read_flag();
        if (!p.pps_deblocking_filter_disabled_flag) {
            p.pps_beta_offset_div2 = r.read_se_range(-6, 6, "pps_beta_offset_div2");
            p.pps_tc_offset_div2 = r.read_se_range(-6, 6, "pps_tc_offset_div2");
        }
    }
    p.scaling = sps.scaling;
    p.pps_scaling_list_data_present_flag = r.read_flag();
    if (p.pps_scaling_list_data_present_flag) {
        p.scaling.set_default();
        scaling_list_data(r, p.scaling);
    }
    p.lists_modification_present_flag = r.read_flag();
    p.log2_parallel_merge_level = r.read_ue_max(uint32_t(sps.log2_ctb_size - 2), "log2_parallel_merge_level_minus2") + 2;
    p.slice_segment_header_extension_present_flag = r.read_flag();
    if (r.read_flag()) {
        bool range = r.read_flag();
        r.read_bits(3 + 4);
        if (range) {
            if (p.transform_skip_enabled_flag && r.read_ue() != 0) p.range_extension_tools = true;
            if (r.read_flag()) p.range_extension_tools = true;  // cross_component_prediction
            if (r.read_flag()) p.range_extension_tools = true;  // chroma_qp_offset_list
            else {
                if (r.read_ue() != 0) p.range_extension_tools = true;
                if (r.read_ue() != 0) p.range_extension_tools = true;
            }
        }
    }
    if (p.init_qp_minus26 < -(26 + 6 * sps.bit_depth_luma_minus8) || p.init_qp_minus26 > 25)
        throw HeifError("init_qp_minus26 out of range");
    return p;
}

namespace {
SliceSegmentHeader slice_segment_header_prefix(const uint8_t *payload, size_t len, size_t full_len, NalUnitHeader nal,
                                               const SequenceParameterSet &sps, const PictureParameterSet &pps);
}  // namespace

SliceSegmentHeader slice_segment_header(const uint8_t *payload, size_t len, NalUnitHeader nal,
                                        const SequenceParameterSet &sps, const PictureParameterSet &pps) {
    // The header is short: parse it from an EP-stripped prefix of the payload
    // (stripping the whole 35 KB payload of a tile dominated host parse time),
    // and only when it does not fit there from the whole payload.
    constexpr size_t kPrefix = 4096;
    if (len > kPrefix) {
        try {
            return slice_segment_header_prefix(payload, kPrefix, len, nal, sps, pps);
        } catch (const HeifError &) {
            // fall through: a header longer than the prefix, or a genuine error reported from the full payload
        }
    }
    return slice_segment_header_prefix(payload, len, len, nal, sps, pps);
}

namespace {
// the header from the first `len` bytes of a payload of `full_len` bytes
SliceSegmentHeader slice_segment_header_prefix(const uint8_t *payload, size_t len, size_t full_len, NalUnitHeader nal,
                                               const SequenceParameterSet &sps, const PictureParameterSet &pps) {
    std::vector<uint32_t> ep;
    std::vector<uint8_t> rbsp = RbspReader::remove_emulation_prevention(payload, len, &ep);
    RbspReader r(rbsp.data(), rbsp.size());
    SliceSegmentHeader h;
    int t = nal.nal_unit_type();
    h.first_slice_segment_in_pic_flag = r.read_flag();
    if (t >= 16 && t <= 23) r.read_flag();  // no_output_of_prior_pics_flag
    h.slice_pic_parameter_set_id = r.read_ue_max(63, "slice_pic_parameter_set_id");
    if (!h.first_slice_segment_in_pic_flag) {
        if (pps.dependent_slice_segments_enabled_flag) h.dependent_slice_segment_flag = r.read_flag();
        const uint32_t nctb = uint32_t(sps.pic_width_in_ctbs_y()) * uint32_t(sps.pic_height_in_ctbs_y());
        h.slice_segment_address = r.read_bits(ceil_log2(int(nctb)));
        if (h.slice_segment_address >= nctb) throw HeifError("slice_segment_address out of range");
    }
    h.slice_loop_filter_across_slices_enabled_flag = pps.pps_loop_filter_across_slices_enabled_flag;
    if (!h.dependent_slice_segment_flag) {  // a dependent segment carries only the address and entry points
        r.read_bits(pps.num_extra_slice_header_bits);
        h.slice_type = r.read_ue_max(2, "slice_type");
        if (h.slice_type != 2) throw HeifError("P/B slices are not supported (still images are intra)");
        if (pps.output_flag_present_flag) r.read_flag();
        if (sps.separate_colour_plane_flag) r.read_bits(2);
        if (t != 19 && t != 20) {  // not IDR: POC + RPS (the reference skips these, slice.rs:85)
            r.read_bits(sps.log2_max_pic_order_cnt_lsb);
            if (!r.read_flag()) {
                std::vector<int> nd = sps.st_rps_num_delta_pocs;
                st_ref_pic_set(r, sps.num_short_term_ref_pic_sets, sps.num_short_term_ref_pic_sets, nd);
            } else if (sps.num_short_term_ref_pic_sets > 1) {
                r.read_bits(ceil_log2(sps.num_short_term_ref_pic_sets));
            }
            if (sps.long_term_ref_pics_present_flag) {
                int nsps = sps.num_long_term_ref_pics_sps > 0 ? r.read_ue_max(uint32_t(sps.num_long_term_ref_pics_sps), "num_long_term_sps") : 0;
                int npics = r.read_ue_max(32, "num_long_term_pics");
                for (int i = 0; i < nsps + npics; ++i) {
                    if (i < nsps) {
                        if (sps.num_long_term_ref_pics_sps > 1) r.read_bits(ceil_log2(sps.num_long_term_ref_pics_sps));
                    } else {
                        r.read_bits(sps.log2_max_pic_order_cnt_lsb);
                        r.read_flag();
                    }
                    if (r.read_flag()) r.read_ue();
                }
            }
            if (sps.sps_temporal_mvp_enabled_flag) r.read_flag();
        }
        if (sps.sample_adaptive_offset_enabled_flag) {
            h.slice_sao_luma_flag = r.read_flag();
            if (sps.chroma_array_type() != 0) h.slice_sao_chroma_flag = r.read_flag();
        }
        h.slice_qp_delta = r.read_se();
        {  // 7.4.7.1: SliceQpY in [-QpBdOffsetY, +51]
            const int qp = 26 + pps.init_qp_minus26 + h.slice_qp_delta;
            if (qp < -6 * sps.bit_depth_luma_minus8 || qp > 51) throw HeifError("SliceQpY out of range");
        }
        if (pps.pps_slice_chroma_qp_offsets_present_flag) {
            h.slice_cb_qp_offset = r.read_se_range(-12, 12, "slice_cb_qp_offset");
            h.slice_cr_qp_offset = r.read_se_range(-12, 12, "slice_cr_qp_offset");
            if (pps.pps_cb_qp_offset + h.slice_cb_qp_offset < -12 || pps.pps_cb_qp_offset + h.slice_cb_qp_offset > 12 ||
                pps.pps_cr_qp_offset + h.slice_cr_qp_offset < -12 || pps.pps_cr_qp_offset + h.slice_cr_qp_offset > 12)
                throw HeifError("chroma QP offsets out of range");
        }
        bool override_flag = pps.deblocking_filter_override_enabled_flag ? r.read_flag() : false;
        h.slice_deblocking_filter_disabled_flag = pps.pps_deblocking_filter_disabled_flag;
        h.slice_beta_offset_div2 = pps.pps_beta_offset_div2;
        h.slice_tc_offset_div2 = pps.pps_tc_offset_div2;
        if (override_flag) {
            h.slice_deblocking_filter_disabled_flag = r.read_flag();
            if (!h.slice_deblocking_filter_disabled_flag) {
                h.slice_beta_offset_div2 = r.read_se_range(-6, 6, "slice_beta_offset_div2");
                h.slice_tc_offset_div2 = r.read_se_range(-6, 6, "slice_tc_offset_div2");
            }
        }
        if (pps.pps_loop_filter_across_slices_enabled_flag &&
            (h.slice_sao_luma_flag || h.slice_sao_chroma_flag || !h.slice_deblocking_filter_disabled_flag))
            h.slice_loop_filter_across_slices_enabled_flag = r.read_flag();
    }
    if (pps.tiles_enabled_flag || pps.entropy_coding_sync_enabled_flag) {
        const int max_entries = sps.pic_height_in_ctbs_y() * (pps.tiles_enabled_flag ? sps.pic_width_in_ctbs_y() : 1);
        h.num_entry_point_offsets = r.read_ue_max(uint32_t(max_entries), "num_entry_point_offsets");
        if (h.num_entry_point_offsets > 0) {
            const int bits = r.read_ue_max(31, "offset_len_minus1") + 1;
            for (int i = 0; i < h.num_entry_point_offsets; ++i) h.entry_point_offset.push_back(r.read_bits(bits) + 1);
        }
    }
    if (pps.slice_segment_header_extension_present_flag) {
        const int l = r.read_ue_max(256, "slice_segment_header_extension_length");
        r.skip_bits(size_t(l) * 8);
    }
    r.byte_alignment();
    // rbsp byte offset → raw payload offset
    size_t rb = r.byte_position(), raw = 0, k = 0, e = 0;
    while (k < rb) {
        if (e < ep.size() && ep[e] == raw) {
            ++raw;
            ++e;
            continue;
        }
        ++raw;
        ++k;
    }
    while (e < ep.size() && ep[e] == raw) {
        ++raw;
        ++e;
    }
    h.slice_data_raw_offset = uint32_t(raw);
    uint64_t total = raw;
    for (uint32_t o : h.entry_point_offset) total += o;
    if (total >= full_len) throw HeifError("entry points exceed the NAL unit");
    return h;
}
}  // namespace

void tile_boundaries(const SequenceParameterSet &sps, const PictureParameterSet &pps, std::vector<int> &col_bd,
                     std::vector<int> &row_bd) {
    for (int pass = 0; pass < 2; ++pass) {
        const int n = !pps.tiles_enabled_flag ? 1 : pass ? pps.num_tile_rows : pps.num_tile_columns;
        const int tot = pass ? sps.pic_height_in_ctbs_y() : sps.pic_width_in_ctbs_y();
        const std::vector<int> &ex = pass ? pps.row_heights : pps.column_widths;
        std::vector<int> &bd = pass ? row_bd : col_bd;
        bd.assign(size_t(n) + 1, 0);
        for (int i = 0; i < n; ++i) {
            const int sz = (!pps.tiles_enabled_flag || pps.uniform_spacing_flag)
                               ? ((i + 1) * tot) / n - (i * tot) / n
                               : (i + 1 < n ? ex[size_t(i)] : tot - bd[size_t(i)]);
            if (sz <= 0 || bd[size_t(i)] + sz > tot) throw HeifError("tile sizes exceed the picture");
            bd[size_t(i) + 1] = bd[size_t(i)] + sz;
        }
    }
}

HevcConfig parse_hvcc(const uint8_t *p, size_t n) {
    if (n < 23) throw HeifError("hvcC too short");
    HevcConfig c;
    c.length_size_minus_one = p[21] & 3;
    size_t pos = 22;
    int narr = p[pos++];
    for (int a = 0; a < narr; ++a) {
        if (pos + 3 > n) throw HeifError("hvcC overrun");
        int type = p[pos] & 0x3f;
        int cnt = (p[pos + 1] << 8) | p[pos + 2];
        pos += 3;
        for (int k = 0; k < cnt; ++k) {
            if (pos + 2 > n) throw HeifError("hvcC overrun");
            size_t l = (size_t(p[pos]) << 8) | p[pos + 1];
            pos += 2;
            if (pos + l > n) throw HeifError("hvcC overrun");
            std::vector<uint8_t> nal(p + pos, p + pos + l);
            if (type == 32) c.vps.push_back(std::move(nal));
            else if (type == 33) c.sps.push_back(std::move(nal));
            else if (type == 34) c.pps.push_back(std::move(nal));
            pos += l;
        }
    }
    return c;
}

}  // namespace hg
