// heic_image.cpp — see heic_image.hpp.
#include "heic_image.hpp"

#include <algorithm>
#include <map>

namespace hg {

namespace {

// read_hvcc_nal_unit (decoder.rs:135-143): 2-byte header + EP-stripped RBSP
std::vector<uint8_t> nal_rbsp(const std::vector<uint8_t> &nal) {
    if (nal.size() < 3) throw HeifError("nal unit is too short");
    return RbspReader::remove_emulation_prevention(nal.data() + 2, nal.size() - 2);
}

void check_supported(const SequenceParameterSet &s, const PictureParameterSet &p) {
    if (s.separate_colour_plane_flag) throw UnsupportedError("separate_colour_plane_flag");
    if (s.bit_depth_luma_minus8 != s.bit_depth_chroma_minus8) throw UnsupportedError("luma/chroma bit depth differ");
    if (s.range_extension_tools || p.range_extension_tools) throw UnsupportedError("range-extension coding tools");
    // HEVC tiles decode as sub-pictures (batch.cpp), with WPP each tile's CTB rows
    // its substreams (9.3.1: a row of a tile syncs with the tile's row above)
    if (s.pic_width_in_luma_samples > 8192 || s.pic_height_in_luma_samples > 8192)
        throw UnsupportedError("picture larger than 8192");
    if (s.pic_width_in_luma_samples % (1 << s.log2_min_luma_coding_block_size) ||
        s.pic_height_in_luma_samples % (1 << s.log2_min_luma_coding_block_size))
        throw HeifError("picture size not a multiple of MinCbSizeY");
}

// The slice segments of a picture: in order and covering it (7.4.7.1), and
// each with one entry point per tile / WPP row.  A dependent segment takes its
// slice's header values (7.4.7.1), copied in here.  The GPU path decodes
// several slices as one sub-picture per slice (batch.cpp), so every segment
// must start at a CTB row (a slice's dependent segments are concatenated);
// with HEVC tiles every segment must start at a tile (slices of whole tiles,
// each tile a sub-picture with its slice's values) and nothing is filtered
// across the tiles.  Loop filtering across the
// slices' boundaries is either off for all (independent sub-pictures) or on
// for all, with one set of deblocking values (sub-pictures of an assembly
// filtered whole).
void check_segments(TileJob &job, const ParamSet &ps) {
    for (size_t k = 1; k < job.segs.size(); ++k) {
        SliceSegmentHeader &sh = job.segs[k].sh;
        if (!sh.dependent_slice_segment_flag) continue;
        const SliceSegmentHeader &s = job.segs[k - 1].sh;  // (already inherited when dependent itself)
        sh.slice_type = s.slice_type;
        sh.slice_sao_luma_flag = s.slice_sao_luma_flag;
        sh.slice_sao_chroma_flag = s.slice_sao_chroma_flag;
        sh.slice_qp_delta = s.slice_qp_delta;
        sh.slice_cb_qp_offset = s.slice_cb_qp_offset;
        sh.slice_cr_qp_offset = s.slice_cr_qp_offset;
        sh.slice_deblocking_filter_disabled_flag = s.slice_deblocking_filter_disabled_flag;
        sh.slice_beta_offset_div2 = s.slice_beta_offset_div2;
        sh.slice_tc_offset_div2 = s.slice_tc_offset_div2;
        sh.slice_loop_filter_across_slices_enabled_flag = s.slice_loop_filter_across_slices_enabled_flag;
    }
    const SequenceParameterSet &sps = ps.sps;
    const PictureParameterSet &pps = ps.pps;
    const uint32_t pw = uint32_t(sps.pic_width_in_ctbs_y());
    for (size_t k = 0; k < job.segs.size(); ++k) {
        const SliceSegmentHeader &sh = job.segs[k].sh;
        if (sh.first_slice_segment_in_pic_flag != (k == 0)) throw HeifError("first_slice_segment_in_pic_flag out of order");
        if (k > 0 && sh.slice_segment_address <= job.segs[k - 1].sh.slice_segment_address)
            throw HeifError("slice segments out of order");
        if (k == 0) continue;
        if (pps.tiles_enabled_flag) {
            // slices of whole tiles (7.4.7.1 allows that or tiles of whole slices): each
            // tile decodes with its slice's header values; nothing may be filtered across
            const uint32_t x = sh.slice_segment_address % pw, y = sh.slice_segment_address / pw;
            const bool at_tile = std::find(ps.col_bd.begin(), ps.col_bd.end(), int(x)) != ps.col_bd.end() &&
                                 std::find(ps.row_bd.begin(), ps.row_bd.end(), int(y)) != ps.row_bd.end();
            if (!at_tile)
                throw UnsupportedError("several slice segments together with HEVC tiles (a segment starting inside a tile)");
            if (pps.loop_filter_across_tiles_enabled_flag)
                throw UnsupportedError("several slice segments together with HEVC tiles filtered across tiles");
            continue;
        }
        // a dependent segment inside a row continues its slice's substream there
        // (the row's, with WPP): the parse switches to its data (batch.cpp)
        if (sh.slice_segment_address % pw && !sh.dependent_slice_segment_flag)
            throw UnsupportedError("a slice segment starting inside a CTB row");
        if (sh.dependent_slice_segment_flag) continue;  // the loop-filter rules below are per slice
        size_t second = 1;  // the second slice
        while (job.segs[second].sh.dependent_slice_segment_flag) ++second;
        const SliceSegmentHeader &s1 = job.segs[second].sh;
        if (sh.slice_loop_filter_across_slices_enabled_flag != s1.slice_loop_filter_across_slices_enabled_flag)
            throw UnsupportedError("slices filtered across some slice boundaries only");
        const SliceSegmentHeader &s0 = job.segs[0].sh;
        if (s1.slice_loop_filter_across_slices_enabled_flag &&
            (sh.slice_deblocking_filter_disabled_flag != s0.slice_deblocking_filter_disabled_flag ||
             sh.slice_beta_offset_div2 != s0.slice_beta_offset_div2 ||
             sh.slice_tc_offset_div2 != s0.slice_tc_offset_div2))
            throw UnsupportedError("slices filtered across their boundaries with different deblocking values");
    }
    const size_t ntiles = (ps.col_bd.size() - 1) * (ps.row_bd.size() - 1);
    // tiles: one substream per tile, or with WPP one per CTB row of each tile
    const size_t nsub_tiles = pps.entropy_coding_sync_enabled_flag
                                  ? (ps.col_bd.size() - 1) * size_t(sps.pic_height_in_ctbs_y())
                                  : ntiles;
    size_t nsub_segs = 0;
    for (const SliceSeg &g : job.segs) nsub_segs += size_t(g.sh.num_entry_point_offsets) + 1;
    if (pps.tiles_enabled_flag && nsub_segs != nsub_tiles)
        throw HeifError("tiled picture without one entry point per tile (per tile row with WPP)");
    if (pps.entropy_coding_sync_enabled_flag && !pps.tiles_enabled_flag)
        for (size_t k = 0; k < job.segs.size(); ++k) {
            // the rows the segment's CTUs touch (it may start and end inside rows)
            const uint32_t r0 = job.segs[k].sh.slice_segment_address / pw;
            const uint32_t r1 = k + 1 < job.segs.size() ? (job.segs[k + 1].sh.slice_segment_address - 1) / pw + 1
                                                        : uint32_t(sps.pic_height_in_ctbs_y());
            if (uint32_t(job.segs[k].sh.num_entry_point_offsets) + 1 != r1 - r0)
                throw HeifError("WPP slice without one entry point per CTB row");
        }
}

}  // namespace

ParsedImage parse_heic(const uint8_t *data, size_t len, uint32_t item_id) {
    HeifReader reader(data, len);
    Heif heif = reader.read();
    ParsedImage img;
    img.primary_item_id = heif.primary_item_id;
    img.item_id = item_id ? item_id : heif.primary_item_id;
    for (const auto &r : heif.references)  // 'auxl' from an auxiliary image to the primary
        if (r.type == fourcc('a', 'u', 'x', 'l') && !img.aux_item_id)
            for (uint32_t t : r.to)
                if (t == heif.primary_item_id) img.aux_item_id = r.from;
    const ItemInfo *pi = heif.item_info_by_item_id(img.item_id);
    if (!pi) throw HeifError("item " + std::to_string(img.item_id) + " not found in item_info");
    if (const Property *ispe = heif.item_property(*pi, fourcc('i', 's', 'p', 'e'))) {
        if (ispe->length < 12) throw HeifError("ispe too short");
        const uint8_t *q = data + ispe->offset + 4;
        img.ispe_width = (uint32_t(q[0]) << 24) | (uint32_t(q[1]) << 16) | (uint32_t(q[2]) << 8) | q[3];
        img.ispe_height = (uint32_t(q[4]) << 24) | (uint32_t(q[5]) << 16) | (uint32_t(q[6]) << 8) | q[7];
    }
    if (const Property *irot = heif.item_property(*pi, fourcc('i', 'r', 'o', 't')))
        if (irot->length >= 1) img.rotation = data[irot->offset] & 3;
    // colr of type nclx (ISO/IEC 23008-12 6.5.5; reader.rs:525 leaves it todo!()):
    // its matrix / range override the SPS VUI for RGB conversion.  An item may
    // carry both an ICC ('prof') and an nclx colr, so scan all of them.
    for (uint32_t idx : pi->properties) {
        if (idx == 0 || idx > heif.properties.size()) continue;
        const Property &p = heif.properties[idx - 1];
        if (p.type != fourcc('c', 'o', 'l', 'r') || p.length < 11) continue;
        const uint8_t *q = data + p.offset;
        if (((uint32_t(q[0]) << 24) | (uint32_t(q[1]) << 16) | (uint32_t(q[2]) << 8) | q[3]) != fourcc('n', 'c', 'l', 'x'))
            continue;
        img.nclx = true;
        img.nclx_matrix = (uint32_t(q[8]) << 8) | q[9];
        img.nclx_full_range = q[10] >> 7;
    }
    img.num_thumbnails = heif.num_thumbnails();

    std::vector<uint32_t> tile_ids;
    if (pi->type == fourcc('g', 'r', 'i', 'd')) {
        ImageGrid g = heif.grid(*pi);
        img.rows = g.rows;
        img.cols = g.cols;
        img.out_width = g.output_width;
        img.out_height = g.output_height;
        tile_ids = heif.references_from(fourcc('d', 'i', 'm', 'g'), pi->id);
        if (tile_ids.empty()) throw HeifError("grid " + std::to_string(pi->id) + " has no tile references");
        if (tile_ids.size() != size_t(g.rows) * g.cols) throw HeifError("grid tile count mismatch");
    } else if (pi->type == fourcc('h', 'v', 'c', '1')) {
        tile_ids.push_back(pi->id);
    } else {
        throw UnsupportedError("unsupported primary item type");
    }

    // one owned copy of every tile item's bytes; the tiles' payloads are views into it
    std::vector<const ItemInfo *> items;
    size_t coded_total = 0;
    for (uint32_t id : tile_ids) {
        const ItemInfo *it = heif.item_info_by_item_id(id);
        if (!it) throw HeifError("tile item " + std::to_string(id) + " not found");
        if (it->type != fourcc('h', 'v', 'c', '1')) throw UnsupportedError("grid tile is not hvc1");
        items.push_back(it);
        coded_total += heif.item_data(*it, nullptr);
    }
    img.coded.reserve(coded_total);
    std::vector<size_t> item_off;
    for (const ItemInfo *it : items) {
        item_off.push_back(img.coded.size());
        heif.item_data(*it, &img.coded);
    }
    item_off.push_back(img.coded.size());

    std::map<size_t, int> param_of_prop;  // hvcC property offset → params index
    for (size_t ti = 0; ti < items.size(); ++ti) {
        const ItemInfo *it = items[ti];
        const Property *hv = heif.item_property(*it, fourcc('h', 'v', 'c', 'C'));
        if (!hv) throw HeifError("missing HEVC decoder configuration");
        int param;
        auto found = param_of_prop.find(hv->offset);
        HevcConfig cfg = parse_hvcc(data + hv->offset, hv->length);
        if (found == param_of_prop.end()) {
            if (cfg.vps.empty()) throw HeifError("no VPS in hvcC");
            if (cfg.sps.empty()) throw HeifError("no SPS in hvcC");
            if (cfg.pps.empty()) throw HeifError("no PPS in hvcC");
            ParamSet ps;
            ps.key = cfg.sps[0];
            ps.key.insert(ps.key.end(), cfg.pps[0].begin(), cfg.pps[0].end());
            ps.vps = video_parameter_set_rbsp(nal_rbsp(cfg.vps[0]));
            ps.sps = sequence_parameter_set_rbsp(nal_rbsp(cfg.sps[0]));
            ps.pps = picture_parameter_set_rbsp(nal_rbsp(cfg.pps[0]), ps.sps);
            check_supported(ps.sps, ps.pps);
            tile_boundaries(ps.sps, ps.pps, ps.col_bd, ps.row_bd);
            param = int(img.params.size());
            img.params.push_back(std::move(ps));
            param_of_prop[hv->offset] = param;
        } else {
            param = found->second;
        }
        const ParamSet &ps = img.params[size_t(param)];
        // read_item_nal_unit (decoder.rs:146-164), generalised: length-prefixed NAL units,
        // the VCL ones are the picture's slice segments in order, non-VCL units skipped
        const uint8_t *item = img.coded.data() + item_off[ti];
        const size_t item_len = item_off[ti + 1] - item_off[ti];
        img.coded_bytes += uint32_t(item_len);
        int lsz = cfg.length_size_minus_one + 1;
        size_t pos = 0;
        TileJob job;
        job.param = param;
        while (pos < item_len) {
            if (pos + size_t(lsz) > item_len) throw HeifError("truncated NAL length prefix");
            size_t nl = 0;
            for (int k = 0; k < lsz; ++k) nl = (nl << 8) | item[pos + size_t(k)];
            pos += size_t(lsz);
            if (nl < 3 || nl > item_len - pos) throw HeifError("NAL unit length out of range");
            NalUnitHeader h{uint16_t((item[pos] << 8) | item[pos + 1])};
            if (h.nal_unit_type() < 32) {
                SliceSeg sg;
                sg.nal = h;
                sg.payload = item + pos + 2;
                sg.payload_len = nl - 2;
                sg.sh = slice_segment_header(sg.payload, sg.payload_len, sg.nal, ps.sps, ps.pps);
                job.segs.push_back(sg);
            }
            pos += nl;
        }
        if (job.segs.empty()) throw HeifError("tile item holds no VCL NAL unit");
        check_segments(job, ps);
        img.tiles.push_back(std::move(job));
    }
    const SequenceParameterSet &s0 = img.params[0].sps;
    img.tile_width = uint32_t(s0.out_width());
    img.tile_height = uint32_t(s0.out_height());
    for (auto &ps : img.params) {
        if (ps.sps.out_width() != s0.out_width() || ps.sps.out_height() != s0.out_height())
            throw UnsupportedError("grid tiles of different sizes");
        if (ps.sps.bit_depth_luma_minus8 != s0.bit_depth_luma_minus8 || ps.sps.chroma_format_idc != s0.chroma_format_idc)
            throw UnsupportedError("grid tiles with different formats");
    }
    if (pi->type != fourcc('g', 'r', 'i', 'd')) {
        img.out_width = img.tile_width;
        img.out_height = img.tile_height;
    }
    if (img.out_width > img.cols * img.tile_width || img.out_height > img.rows * img.tile_height)
        throw HeifError("grid output larger than its tiles");
    return img;
}

}  // namespace hg
