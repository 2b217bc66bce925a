// batch.cpp — see batch.hpp.
#include "batch.hpp"
#include "../kernels/kernels.hpp"

#include <algorithm>
#include <cstdlib>

namespace hg {

namespace {

SeqParams make_seq(const ParamSet &ps, uint32_t sf_off) {
    const SequenceParameterSet &s = ps.sps;
    const PictureParameterSet &p = ps.pps;
    SeqParams q{};
    q.width = s.pic_width_in_luma_samples;
    q.height = s.pic_height_in_luma_samples;
    q.log2_ctb = s.log2_ctb_size;
    q.log2_min_cb = s.log2_min_luma_coding_block_size;
    q.log2_min_tb = s.log2_min_tb_size;
    q.log2_max_tb = s.log2_max_tb_size;
    q.max_th_depth_intra = s.max_transform_hierarchy_depth_intra;
    q.chroma_format = s.chroma_array_type();
    q.bit_depth_y = 8 + s.bit_depth_luma_minus8;
    q.bit_depth_c = 8 + s.bit_depth_chroma_minus8;
    uint32_t f = 0;
    if (s.scaling_list_enabled_flag) f |= SP_SCALING_LIST;
    if (p.sign_data_hiding_enabled_flag) f |= SP_SIGN_HIDING;
    if (p.transform_skip_enabled_flag) f |= SP_TRANSFORM_SKIP;
    if (p.transquant_bypass_enabled_flag) f |= SP_TQ_BYPASS;
    if (p.cu_qp_delta_enabled_flag) f |= SP_CU_QP_DELTA;
    if (p.entropy_coding_sync_enabled_flag) f |= SP_WPP;
    if (s.strong_intra_smoothing_enabled_flag) f |= SP_STRONG_INTRA;
    if (s.pcm_enabled_flag) f |= SP_PCM;
    if (s.pcm_loop_filter_disabled_flag) f |= SP_PCM_LOOP_FILTER_DISABLED;
    if (s.sample_adaptive_offset_enabled_flag) f |= SP_SAO;
    q.flags = f;
    q.diff_cu_qp_delta_depth = p.diff_cu_qp_delta_depth;
    q.cb_qp_offset = p.pps_cb_qp_offset;
    q.cr_qp_offset = p.pps_cr_qp_offset;
    q.log2_min_pcm = s.log2_min_pcm;
    q.log2_max_pcm = s.log2_max_pcm;
    q.pcm_bd_y = s.pcm_bit_depth_luma;
    q.pcm_bd_c = s.pcm_bit_depth_chroma;
    q.conf_l = s.conf_win_left;
    q.conf_t = s.conf_win_top;
    q.out_w = s.out_width();
    q.out_h = s.out_height();
    q.sf_off = sf_off;
    return q;
}

// k_parse_lanes lanes per WPP picture: a picture with more CTB rows wraps
// them round its lanes (lane r parses rows r, r + R, ...).  (r04 measured
// fewer lanes than rows per picture, 8 or 12, at 87-132 against 83.5 ms per
// step: the knob is gone, the wrap stays for pictures over 64 CTB rows.)
int max_lane_rows() { return 64; }

// a slice's header values of a picture
void slice_values(PicDesc &pd, const ParamSet &ps, const SliceSegmentHeader &sh) {
    pd.slice_qp = 26 + ps.pps.init_qp_minus26 + sh.slice_qp_delta;
    pd.cb_qp_off = sh.slice_cb_qp_offset;
    pd.cr_qp_off = sh.slice_cr_qp_offset;
    pd.sao_luma = sh.slice_sao_luma_flag;
    pd.sao_chroma = sh.slice_sao_chroma_flag;
    pd.dbk_disabled = sh.slice_deblocking_filter_disabled_flag;
    pd.beta_off = sh.slice_beta_offset_div2;
    pd.tc_off = sh.slice_tc_offset_div2;
}

void fill_scaling(const ParamSet &ps, uint8_t *blk) {
    for (int sid = 0; sid < 4; ++sid) {
        int n = 4 << sid;
        for (int m = 0; m < 6; ++m) ps.pps.scaling.factors(sid, m, blk + sf_size_offset(sid) + uint32_t(m * n * n));
    }
}

}  // namespace

HostBatch build_batch(const ParsedImage *const *imgs, size_t n, uint32_t tile_stride, uint32_t tile_offset,
                      bool defer_bits) {
    if (tile_stride == 0) tile_stride = 1;
    if (tile_offset >= tile_stride) throw HeifError("tile_offset must be below tile_stride");
    HostBatch hb;
    std::vector<std::vector<uint8_t>> seq_keys, sf_keys;  // SeqParams: PPS + picture geometry; ScalingFactor: PPS
    std::vector<uint32_t> sf_offs;
    // SeqParams index of (PPS, picture geometry); one ScalingFactor block per PPS
    auto seq_of = [&](const ParamSet &ps, SeqParams base) -> uint32_t {
        std::vector<uint8_t> key = ps.key;
        const int32_t g[7] = {base.width, base.height, base.conf_l, base.conf_t, base.out_w, base.out_h,
                              int32_t(base.flags)};
        const uint8_t *gb = reinterpret_cast<const uint8_t *>(g);
        key.insert(key.end(), gb, gb + sizeof(g));
        auto it = std::find(seq_keys.begin(), seq_keys.end(), key);
        if (it != seq_keys.end()) return uint32_t(it - seq_keys.begin());
        seq_keys.push_back(key);
        auto sf = std::find(sf_keys.begin(), sf_keys.end(), ps.key);
        if (sf == sf_keys.end()) {
            sf_keys.push_back(ps.key);
            sf_offs.push_back(uint32_t(hb.sf.size()));
            hb.sf.resize(hb.sf.size() + kSfBlockBytes);
            fill_scaling(ps, hb.sf.data() + sf_offs.back());
            sf = sf_keys.end() - 1;
        }
        base.sf_off = sf_offs[size_t(sf - sf_keys.begin())];
        hb.seqs.push_back(base);
        return uint32_t(hb.seqs.size() - 1);
    };
    // the work arenas of a picture (coded: it is parsed and reconstructed; an
    // assembly only holds samples, maps and SAO parameters), then the batch maxima
    auto add_picture = [&](PicDesc &pd, bool coded) {
        const SeqParams &sq = hb.seqs[pd.seq];
        const int ctb = 1 << sq.log2_ctb;
        const int wctb = (sq.width + ctb - 1) / ctb, hctb = (sq.height + ctb - 1) / ctb;
        const int w4 = (sq.width + 3) >> 2, h4 = (sq.height + 3) >> 2, w8 = (sq.width + 7) >> 3;
        const int cf = sq.chroma_format;
        const uint64_t samples = uint64_t(sq.width) * sq.height +
                                 (cf ? 2 * uint64_t(sq.width >> chroma_sx(cf)) * uint64_t(sq.height >> chroma_sy(cf)) : 0);
        pd.recon_off = hb.recon_bytes;
        hb.recon_bytes += (samples * uint64_t(hb.bps) + 255) & ~uint64_t(255);
        pd.map_off = hb.map_bytes;
        hb.map_bytes += (uint64_t(2) * w4 * h4 + uint64_t(hctb) * w8 + 255) & ~uint64_t(255);
        pd.sao_off = hb.sao_n;
        hb.sao_n += uint64_t(wctb) * hctb;
        pd.resid_off = hb.resid_elems;
        pd.row_off = hb.rows;
        pd.tu_off = hb.tu_n;
        pd.coef_off = hb.coef_n;
        hb.pics.push_back(pd);
        hb.pic_image.push_back(pd.image);
        hb.max_w = std::max(hb.max_w, sq.width);
        hb.max_wctb = std::max(hb.max_wctb, wctb);
        hb.max_log2ctb = std::max(hb.max_log2ctb, int(sq.log2_ctb));
        if (!coded) return;
        PicDesc &p = hb.pics.back();
        hb.resid_elems += (samples + 127) & ~uint64_t(127);
        hb.rows += uint32_t(hctb);
        // worst case per CTB row: every 8x8 CU split into four 4x4 luma TBs and
        // their chroma TBs (2 with 4:2:0, 4 with 4:2:2, 8 with 4:4:4); a
        // coefficient (or PCM sample) per sample
        const int tbs8 = cf == 3 ? 12 : (cf == 2 ? 8 : 6);
        p.tu_cap_row = uint32_t(wctb * (ctb / 8) * (ctb / 8) * tbs8 + 64);  // + staging trash slot / slack
        const int ctb_samples = ctb * ctb + (cf ? 2 * (ctb >> chroma_sx(cf)) * (ctb >> chroma_sy(cf)) : 0);
        p.coef_cap_row = uint32_t(wctb * ctb_samples + 64);  // + staging trash slot / slack
        hb.tu_n += uint64_t(p.tu_cap_row) * hctb;
        hb.coef_n += uint64_t(p.coef_cap_row) * hctb;
        hb.max_rows = std::max(hb.max_rows, hctb);
        const bool wpp = (sq.flags & SP_WPP) != 0;
        hb.lane_rows = std::max(hb.lane_rows, wpp ? std::min(hctb, max_lane_rows()) : 1);
        if (wpp && hctb > max_lane_rows()) hb.wpp_ring = 1;
        if (wpp) hb.max_wpp_rows = std::max(hb.max_wpp_rows, hctb);
    };
    for (size_t i = 0; i < n; ++i) {
        const ParsedImage &im = *imgs[i];
        const SequenceParameterSet &s0 = im.params[0].sps;
        int bps = s0.bit_depth_luma_minus8 > 0 ? 2 : 1;
        if (hb.bps == 0) {
            hb.bps = bps;
            hb.chroma = s0.chroma_array_type();
        } else if (hb.bps != bps || hb.chroma != s0.chroma_array_type()) {
            throw UnsupportedError("a batch must share bit depth and chroma format");
        }
        for (size_t t = tile_offset; t < im.tiles.size(); t += tile_stride) {
            const TileJob &tj = im.tiles[t];
            const ParamSet &ps = im.params[size_t(tj.param)];
            // A coded picture decodes as one or more independent sub-pictures
            // (heic_image.cpp accepts only layouts where nothing crosses their
            // boundaries): an HEVC tile (6.5.1) with no loop filter across tiles
            // becomes a picture of the tile's size whose one substream is the
            // tile's entry-point range; a slice starting at a CTB row with no
            // loop filter across slices becomes the band of rows it covers, with
            // its own slice header values and substreams.  Each is placed at its
            // offset in the cropped output.  Otherwise: one sub-picture, the
            // whole picture with all its substreams.
            struct Sub {
                int x0, y0, x1, y1;  // CTBs
                size_t seg, nseg;    // slice segments [seg, seg + nseg): a slice and its dependent segments
                int s0, s1;          // substreams [s0, s1) of a single segment
                bool subset_end;     // ends in end_of_subset_one_bit (a tile other than the last)
            };
            std::vector<Sub> subs_of;
            const int pctb = 1 << ps.sps.log2_ctb_size;
            const int pw = ps.sps.pic_width_in_ctbs_y(), ph = ps.sps.pic_height_in_ctbs_y();
            if (ps.pps.tiles_enabled_flag) {
                // substreams in tile scan: one per tile, or with WPP one per CTB row of each tile
                // in the slice segment holding the tile (segments of whole tiles, heic_image.cpp)
                const int ntc = int(ps.col_bd.size()) - 1, ntr = int(ps.row_bd.size()) - 1;
                const bool wpp = ps.pps.entropy_coding_sync_enabled_flag;
                size_t seg = 0;
                int s = 0;
                for (int ht = 0; ht < ntc * ntr; ++ht) {
                    const int tc = ht % ntc, tr = ht / ntc;
                    const int y0 = ps.row_bd[size_t(tr)], y1 = ps.row_bd[size_t(tr) + 1];
                    const uint32_t addr = uint32_t(y0 * pw + ps.col_bd[size_t(tc)]);
                    if (seg + 1 < tj.segs.size() && tj.segs[seg + 1].sh.slice_segment_address == addr) {
                        ++seg;
                        s = 0;
                    }
                    const int n = wpp ? y1 - y0 : 1;
                    if (s + n > tj.segs[seg].sh.num_entry_point_offsets + 1)
                        throw HeifError("slice segment without one entry point per tile (per tile row with WPP)");
                    // a tile other than its segment's last ends in end_of_subset_one_bit
                    const bool seg_last = s + n == tj.segs[seg].sh.num_entry_point_offsets + 1;
                    subs_of.push_back({ps.col_bd[size_t(tc)], y0, ps.col_bd[size_t(tc) + 1], y1, seg, 1, s, s + n,
                                       !seg_last});
                    s += n;
                }
            } else {
                for (size_t k = 0; k < tj.segs.size();) {  // one sub-picture per slice
                    size_t e = k + 1;
                    while (e < tj.segs.size() && tj.segs[e].sh.dependent_slice_segment_flag) ++e;
                    const int r0 = int(tj.segs[k].sh.slice_segment_address) / pw;
                    const int r1 = e < tj.segs.size() ? int(tj.segs[e].sh.slice_segment_address) / pw : ph;
                    subs_of.push_back({0, r0, pw, r1, k, e - k, 0, tj.segs[k].sh.num_entry_point_offsets + 1, false});
                    k = e;
                }
            }
            // Loop filters across the sub-pictures' boundaries (tiles with
            // loop_filter_across_tiles_enabled_flag, slices with
            // slice_loop_filter_across_slices_enabled_flag; heic_image.cpp takes
            // all-or-none): the sub-pictures are children of an assembly picture
            // of the whole picture, which k_assemble puts together before the
            // loop filters run on it (desc.hpp).
            const bool assemble =
                subs_of.size() > 1 && (ps.pps.tiles_enabled_flag ? ps.pps.loop_filter_across_tiles_enabled_flag
                                                                 : tj.segs[subs_of[1].seg].sh.slice_loop_filter_across_slices_enabled_flag);
            const uint32_t child0 = uint32_t(hb.pics.size());
            const int32_t grid_x = int32_t((t % im.cols) * im.tile_width), grid_y = int32_t((t / im.cols) * im.tile_height);
            for (const Sub &su : subs_of) {
                const SliceSeg &sg = tj.segs[su.seg];
                std::vector<uint32_t> starts{sg.sh.slice_data_raw_offset};  // the segment's substreams
                for (uint32_t e : sg.sh.entry_point_offset) starts.push_back(starts.back() + e);
                starts.push_back(uint32_t(sg.payload_len));
                SeqParams base = make_seq(ps, 0);
                int vis_dx = 0, vis_dy = 0;  // output offset of the sub-picture's visible part
                if (su.nseg > 1) base.flags |= SP_ROW_SEGMENTS;
                if (subs_of.size() > 1) {
                    const int x0 = su.x0 * pctb, y0 = su.y0 * pctb;
                    const int x1 = std::min(su.x1 * pctb, base.width), y1 = std::min(su.y1 * pctb, base.height);
                    // the picture's conformance window [conf_l, conf_l + out_w) clipped to the sub-picture
                    const int vx0 = std::max(x0, base.conf_l), vx1 = std::min(x1, base.conf_l + base.out_w);
                    const int vy0 = std::max(y0, base.conf_t), vy1 = std::min(y1, base.conf_t + base.out_h);
                    base.width = x1 - x0;
                    base.height = y1 - y0;
                    base.conf_l = vx0 - x0;
                    base.conf_t = vy0 - y0;
                    base.out_w = std::max(vx1 - vx0, 0);
                    base.out_h = std::max(vy1 - vy0, 0);
                    vis_dx = vx0 - ps.sps.conf_win_left;
                    vis_dy = vy0 - ps.sps.conf_win_top;
                    if (su.subset_end) base.flags |= SP_SUBSET_END;
                }
                const uint32_t seq = seq_of(ps, base);
                const SeqParams &sq = hb.seqs[seq];
                PicDesc pd{};
                pd.bits_off = hb.bits_size;
                pd.sub_first = uint32_t(hb.subs.size());
                std::vector<uint32_t> mids;  // data offsets of dependent segments starting inside a row
                std::vector<uint32_t> mid_prefix;  // WPP: per row, the mids starting in earlier rows
                if (su.nseg > 1 && !ps.pps.entropy_coding_sync_enabled_flag) {
                    // a slice of several segments without WPP: their slice data back
                    // to back, one substream-table entry per CTB row for the CTU at its
                    // start (a segment starting there: its data; otherwise the engine
                    // runs on, SUB_CONTINUE), SUB_SEG_END on a row whose last CTU ends a
                    // segment, and the data of each dependent segment starting inside a
                    // row after the end entry (their count in PicDesc.flags, PD_NMID_SHIFT; the parse switches to the
                    // next one where end_of_slice_segment_flag ends a segment inside a row)
                    std::vector<uint32_t> seg_off, seg_addr;
                    uint32_t off = 0;
                    for (size_t j = su.seg; j < su.seg + su.nseg; ++j) {
                        const SliceSeg &g = tj.segs[j];
                        const uint32_t d0 = g.sh.slice_data_raw_offset;
                        uint32_t d1 = uint32_t(g.payload_len);
                        while (d1 >= d0 + 3 && g.payload[d1 - 1] == 3 && g.payload[d1 - 2] == 0 && g.payload[d1 - 3] == 0)
                            d1 -= 3;  // (cabac_zero_words: see the WPP path below)
                        hb.pieces.push_back({g.payload + d0, d1 - d0, hb.bits_size + off});
                        seg_off.push_back(off);
                        seg_addr.push_back(g.sh.slice_segment_address);
                        if (j > su.seg && g.sh.slice_segment_address % uint32_t(pw)) mids.push_back(off);
                        off += d1 - d0;
                    }
                    size_t cov = 0;  // the segment holding the row's first CTU
                    for (int r = su.y0; r < su.y1; ++r) {
                        const uint32_t a0 = uint32_t(r * pw), a1 = uint32_t((r + 1) * pw);
                        while (cov + 1 < seg_addr.size() && seg_addr[cov + 1] <= a0) ++cov;
                        uint32_t v = seg_addr[cov] == a0 ? seg_off[cov] : (seg_off[cov] | SUB_CONTINUE);
                        if (std::find(seg_addr.begin() + 1, seg_addr.end(), a1) != seg_addr.end()) v |= SUB_SEG_END;
                        hb.subs.push_back(v);
                    }
                    pd.bits_len = off;
                    pd.n_sub = uint32_t(su.y1 - su.y0);
                } else if (su.nseg > 1) {
                    // a slice of several segments with WPP: their slice data back to back,
                    // one substream-table entry per CTB row (SUB_* flags, desc.hpp): the
                    // data, or the entry point, of the segment holding the row's first
                    // CTU.  Dependent segments starting inside a row: their data after
                    // the end entry as without WPP, then per row the count of those
                    // starting in earlier rows (where the row's lane starts counting)
                    uint32_t off = 0;
                    std::vector<int> mid_rows;
                    const size_t jend = su.seg + su.nseg;
                    for (size_t j = su.seg; j < jend; ++j) {
                        const SliceSeg &g = tj.segs[j];
                        const uint32_t d0 = g.sh.slice_data_raw_offset;
                        uint32_t d1 = uint32_t(g.payload_len);
                        // cabac_zero_words (00 00 03 each) would leave zero bytes before the
                        // next segment's data, where they could start an emulation-prevention pattern
                        while (d1 >= d0 + 3 && g.payload[d1 - 1] == 3 && g.payload[d1 - 2] == 0 && g.payload[d1 - 3] == 0)
                            d1 -= 3;
                        hb.pieces.push_back({g.payload + d0, d1 - d0, hb.bits_size + off});
                        const int a0 = int(g.sh.slice_segment_address);
                        const int a1 = j + 1 < jend ? int(tj.segs[j + 1].sh.slice_segment_address) : su.y1 * pw;
                        const int r0 = a0 / pw;
                        if (j > su.seg && a0 % pw) {
                            mids.push_back(off);
                            mid_rows.push_back(r0);
                        }
                        uint32_t e = off;  // the row's substream start within the concatenation
                        // the rows whose first CTU the segment holds: r * pw in [a0, a1)
                        for (int r = r0; r * pw < a1; ++r) {
                            if (r > r0) {
                                if (size_t(r - r0 - 1) >= g.sh.entry_point_offset.size())
                                    throw HeifError("WPP slice segment without one entry point per CTB row");
                                e += g.sh.entry_point_offset[size_t(r - r0 - 1)];
                            }
                            if (r * pw < a0) continue;  // starts inside row r0
                            uint32_t v = e;
                            if ((r + 1) * pw == a1 && j + 1 < jend) v |= SUB_SEG_END;
                            hb.subs.push_back(v);
                        }
                        off += d1 - d0;
                    }
                    pd.bits_len = off;
                    pd.n_sub = uint32_t(su.y1 - su.y0);
                    if (hb.subs.size() != pd.sub_first + pd.n_sub) throw HeifError("slice segments out of order");
                    if (!mids.empty()) {  // after the end entry and the mids (pushed below)
                        size_t k = 0;
                        for (int r = su.y0; r < su.y1; ++r) {
                            while (k < mid_rows.size() && mid_rows[k] < r) ++k;
                            mid_prefix.push_back(uint32_t(k));
                        }
                    }
                } else if (su.s0 > 0 || su.s1 + 1 < int(starts.size())) {
                    // a substream range alone (it starts after a nonzero byte: no EP state carries in)
                    const uint32_t r0 = starts[size_t(su.s0)], r1 = starts[size_t(su.s1)];
                    pd.bits_len = r1 - r0;
                    pd.n_sub = uint32_t(su.s1 - su.s0);
                    hb.pieces.push_back({sg.payload + r0, pd.bits_len, hb.bits_size});
                    for (int k = su.s0; k < su.s1; ++k) hb.subs.push_back(starts[size_t(k)] - r0);
                } else {  // the whole NAL payload (subs from the slice data start)
                    pd.bits_len = uint32_t(sg.payload_len);
                    pd.n_sub = uint32_t(sg.sh.num_entry_point_offsets + 1);
                    hb.pieces.push_back({sg.payload, sg.payload_len, hb.bits_size});
                    for (size_t k = 0; k + 1 < starts.size(); ++k) hb.subs.push_back(starts[k]);
                }
                hb.subs.push_back(pd.bits_len);
                for (uint32_t m : mids) hb.subs.push_back(m);
                for (uint32_t m : mid_prefix) hb.subs.push_back(m);  // raw only (k_rbsp remaps up to the mids)
                if (mids.size() > PD_NMID_MAX) throw UnsupportedError("over 32767 slice segments starting inside CTB rows");
                pd.flags |= uint32_t(mids.size()) << PD_NMID_SHIFT;
                hb.bits_size = (hb.bits_size + pd.bits_len + 63) & ~size_t(63);
                const int hctb = (sq.height + (1 << sq.log2_ctb) - 1) >> sq.log2_ctb;
                if ((sq.flags & SP_WPP) && int(pd.n_sub) != hctb)
                    throw HeifError("WPP picture without one entry point per CTB row");
                pd.seq = seq;
                slice_values(pd, ps, sg.sh);
                pd.image = uint32_t(i);
                pd.out_x = grid_x + vis_dx;
                pd.out_y = grid_y + vis_dy;
                if (assemble) {
                    pd.flags |= PD_CHILD;
                    pd.org_x = su.x0 * pctb;
                    pd.org_y = su.y0 * pctb;
                }
                add_picture(pd, true);
            }
            if (assemble) {  // the whole picture: no coded data, loop filters and output
                PicDesc pd{};
                pd.seq = seq_of(ps, make_seq(ps, 0));
                pd.bits_off = hb.bits_size;
                pd.sub_first = uint32_t(hb.subs.size());
                hb.subs.push_back(0);  // n_sub = 0: k_rbsp sees only the (empty) end entry
                slice_values(pd, ps, tj.segs[0].sh);  // the deblocking values (all alike: heic_image.cpp)
                for (const SliceSeg &sg : tj.segs) {
                    pd.sao_luma |= sg.sh.slice_sao_luma_flag;
                    pd.sao_chroma |= sg.sh.slice_sao_chroma_flag;
                }
                pd.image = uint32_t(i);
                pd.out_x = grid_x;
                pd.out_y = grid_y;
                pd.flags = PD_ASSEMBLY;
                pd.child0 = child0;
                pd.nchild = uint32_t(subs_of.size());
                add_picture(pd, false);
                hb.has_assembly = true;
            }
        }
    }
    hb.bits_size += 128;
    if (!defer_bits) {
        hb.bits.assign(hb.bits_size, 0);
        for (const HostBatch::Piece &pc : hb.pieces) std::copy(pc.src, pc.src + pc.len, hb.bits.data() + pc.dst);
        hb.pieces.clear();
    }
    return hb;
}

}  // namespace hg
