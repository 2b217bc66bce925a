// emu_check.cpp — TEST-ONLY driver: runs the decode kernels' own sources as
// host C++ (HG_HOST_EMU, see kernels/wave.hpp) and diffs every plane against
// the CPU oracle.  Never part of the product library.
//   emu_check file.heic [stages=5] [tile_stride tile_offset]
//   stages: 1 parse .. 5 full (3 = before deblocking); with a tile stride only
//   the grid tiles k % stride == offset are decoded (the tile split across GPUs):
//   their windows must match the oracle and every other sample must keep the
//   sentinel the planes start with
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../../oracle/oracle.h"
#include "../host/batch.hpp"
#include "../kernels/cabac.hpp"
#include "../kernels/kernels.hpp"

namespace hg {
thread_local EmuCtx g_emu;
}
using namespace hg;

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    setvbuf(stdout, nullptr, _IONBF, 0);  // every line out before a sanitizer abort
    int stages = argc > 2 ? atoi(argv[2]) : 5;
    const uint32_t tstride = argc > 4 ? uint32_t(atoi(argv[3])) : 1u, toff = argc > 4 ? uint32_t(atoi(argv[4])) : 0u;
    FILE *f = fopen(argv[1], "rb");
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::vector<uint8_t> data(static_cast<size_t>(n), 0);
    if (fread(data.data(), 1, size_t(n), f) != size_t(n)) return 2;
    fclose(f);
    ParsedImage im;
    HostBatch hb;
    try {  // the host's checks reject what the kernels never see (the API returns the error)
        im = parse_heic(data.data(), data.size());
        const ParsedImage *ims[1] = {&im};
        hb = build_batch(ims, 1, tstride, toff);
    } catch (const std::exception &e) {
        printf("host rejected: %s\n", e.what());
        return 3;
    }
    std::vector<TuRec> tus(hb.tu_n);
    std::vector<Coef> coefs(hb.coef_n);
    std::vector<uint32_t> rc(2 * hb.rows), status(hb.pics.size());
    std::vector<uint8_t> recon(hb.recon_bytes), maps(hb.map_bytes);
    std::vector<int16_t> resid(hb.resid_elems);
    std::vector<SaoParams> sao(hb.sao_n);
    const int W = int(im.out_width), H = int(im.out_height), bps = hb.bps;
    const int SX = chroma_sx(hb.chroma), SY = chroma_sy(hb.chroma);
    const int CW = (W + (1 << SX) - 1) >> SX, CH = (H + (1 << SY) - 1) >> SY;
    constexpr uint8_t kSentinel = 0xa5;
    std::vector<uint8_t> oy(size_t(W) * H * bps, kSentinel), ocb(size_t(CW) * CH * bps, kSentinel),
        ocr(size_t(CW) * CH * bps, kSentinel);
    OutImage out{};
    out.plane[0] = uint64_t(oy.data());
    out.plane[1] = uint64_t(ocb.data());
    out.plane[2] = uint64_t(ocr.data());
    out.pitch[0] = W * bps;
    out.pitch[1] = out.pitch[2] = CW * bps;
    out.width = W;
    out.height = H;
    BatchArgs a{};
    a.bits = hb.bits.data();
    a.pics = hb.pics.data();
    a.subs = hb.subs.data();
    std::vector<uint8_t> rbsp(hb.bits.size(), 0);
    std::vector<uint32_t> rsubs(hb.subs.size(), 0);
    a.rbsp = rbsp.data();
    a.rsubs = rsubs.data();
    std::vector<uint32_t> order;
    const int mode = parse_mode_for(PARSE_AUTO, int(hb.pics.size()), hb.pics.data());
    const int solo_waves = solo_waves_for(hb.lane_rows);
    int parse_group = 1;
    if (mode == PARSE_SPREAD) spread_parse_order(hb.pics.data(), int(hb.pics.size()), order);
    else
        parse_group = lanes_parse_order(hb.pics.data(), int(hb.pics.size()), hb.lane_rows, mode == PARSE_SOLO ? 1 : 0,
                                        order);
    std::vector<uint32_t> xprog(hb.rows + 1), xntu(hb.rows + hb.pics.size() + 1, 0);  // (+ the job counter)
    std::vector<uint8_t> xctx((hb.rows + 1) * size_t(CTX_PAD));
    a.parse_order = order.data();
    a.n_slots = int(order.size());
    a.parse_group = parse_group;
    a.seqs = hb.seqs.data();
    a.sf = hb.sf.data();
    a.outs = &out;
    a.tus = tus.data();
    a.coefs = coefs.data();
    a.row_counts = rc.data();
    a.recon = recon.data();
    a.resid = resid.data();
    a.maps = maps.data();
    a.sao = sao.data();
    a.status = status.data();
    a.n_pics = int(hb.pics.size());
    a.max_width = hb.max_w;
    a.max_wctb = hb.max_wctb;
    a.max_rows = hb.max_rows;
    a.max_log2ctb = hb.max_log2ctb;
    a.lane_rows = hb.lane_rows;
    a.parse_mode = mode;
    a.solo_waves = solo_waves;
    a.xprog = xprog.data();
    a.xctx = xctx.data();
    a.xjob = xprog.data() + hb.rows;
    const StreamKnobs knobs = stream_knobs_from_env();
    a.intra_stream = intra_stream_for(mode, int(hb.pics.size()), hb.has_assembly, knobs) ? 1 : 0;
    a.xntu = a.intra_stream ? xntu.data() : nullptr;
    a.stream_patience_us = knobs.patience_us;
    a.wpp_ring = mode == PARSE_SOLO ? (hb.max_wpp_rows > solo_waves ? 1 : 0) : hb.wpp_ring;
    a.has_assembly = hb.has_assembly ? 1 : 0;
    a.total_rows = int(hb.rows);
    a.bytes_per_sample = bps;
    a.chroma_format = hb.chroma;
    if (stages <= 0) {  // host only: container, parameter sets, slice headers, batch layout
        printf("host ok: %zu pictures\n", hb.pics.size());
        return 0;
    }
    // k_rbsp zeroes the decode's status words, row counts, progress words and TU
    // counts: start them as garbage, as a reused parse-output set holds them
    std::fill(rc.begin(), rc.end(), 0xa5a5a5a5u);
    std::fill(status.begin(), status.end(), 0x5au);
    std::fill(xprog.begin(), xprog.end(), 0x7777u);
    std::fill(xntu.begin(), xntu.end(), 0x3333u);
    emu_rbsp(a);
    emu_parse(a);
    uint32_t st = 0;
    for (uint32_t s : status) st |= s;
    uint64_t ntu = 0, ncoef = 0;
    for (uint32_t r = 0; r < hb.rows; ++r) {
        ntu += rc[2 * r];
        ncoef += rc[2 * r + 1];
    }
    if (getenv("HG_EMU_DEBUG_MODES")) {  // tuning aid: TB records with an out-of-range mode
        int shown = 0;
        for (const PicDesc &pd : hb.pics)
            for (uint32_t r = 0; r < (uint32_t)((hb.seqs[pd.seq].height + (1 << hb.seqs[pd.seq].log2_ctb) - 1) >> hb.seqs[pd.seq].log2_ctb); ++r) {
                const uint32_t nt = rc[2 * (pd.row_off + r)];
                for (uint32_t t = 0; t < nt && shown < 10; ++t) {
                    const TuRec &tu = tus[pd.tu_off + (uint64_t)r * pd.tu_cap_row + t];
                    if (tu.mode > 34) {
                        printf("bad mode %d pic %u row %u t %u x %d y %d log2 %d flags 0x%x ctu %d\n", tu.mode, (unsigned)(&pd - hb.pics.data()), r, t, tu.x, tu.y, tu.log2, tu.flags, tu.ctu);
                        ++shown;
                    }
                }
            }
    }
    printf("parse mode: %s\n", mode == PARSE_SOLO     ? "solo"
                               : mode == PARSE_SPREAD ? "spread"
                                                      : "lanes");
    printf("parse: status 0x%x, %llu TBs, %llu coefficients\n", st, (unsigned long long)ntu, (unsigned long long)ncoef);
    if (stages >= 2 && !a.intra_stream) emu_transform(a);  // (streaming: k_intra_stream transforms each TB)
    if (stages >= 3) {
        emu_intra(a);
        if (a.intra_stream) {  // the second launch: the pictures the first gave up on
            BatchArgs a2 = a;
            a2.stream_redo = 1;
            emu_intra(a2);
        }
    }
    if (stages >= 4) emu_deblock(a);
    if (stages >= 5) {
        emu_sao_out(a);
    } else {
        // copy the recon arena into the output planes (crop + grid placement, no SAO)
        int dbk = stages >= 4 ? 0 : 1;
        oracle_set_debug_flags(dbk | 2);
        for (const PicDesc &pd : hb.pics) {
            const SeqParams &sp = hb.seqs[pd.seq];
            for (int c = 0; c < 3; ++c) {
                if (c && !sp.chroma_format) break;
                const int sx = c ? SX : 0, sy = c ? SY : 0, PW = sp.width >> sx, PH = sp.height >> sy;
                size_t off = c == 0 ? 0 : size_t(sp.width) * sp.height + size_t(c - 1) * PW * PH;
                int vw = std::min(sp.out_w, W - pd.out_x) >> sx, vh = std::min(sp.out_h, H - pd.out_y) >> sy;
                for (int y = 0; y < vh; ++y)
                    for (int x = 0; x < vw; ++x) {
                        size_t src = (off + size_t(y + (sp.conf_t >> sy)) * PW + x + (sp.conf_l >> sx)) * bps;
                        uint8_t *dst = reinterpret_cast<uint8_t *>(out.plane[c]) +
                                       size_t((pd.out_y >> sy) + y) * out.pitch[c] + size_t((pd.out_x >> sx) + x) * bps;
                        memcpy(dst, recon.data() + pd.recon_off + src, size_t(bps));
                    }
            }
        }
    }
    if (stages < 3) return st ? 1 : 0;
    oracle_image ref;
    if (oracle_decode_heic(data.data(), data.size(), &ref, nullptr, 0, nullptr)) {
        printf("oracle failed: %s\n", oracle_last_error());
        return 1;
    }
    long bad_total = 0;
    const char *names[3] = {"Y", "Cb", "Cr"};
    for (int c = 0; c < 3; ++c) {
        const uint8_t *g = c == 0 ? oy.data() : (c == 1 ? ocb.data() : ocr.data());
        int pw = int(ref.pw[c]), ph = int(ref.ph[c]);
        long bad = 0;
        int fx = -1, fy = -1;
        const int sx = c ? SX : 0, sy = c ? SY : 0;
        for (int y = 0; y < ph; ++y)
            for (int x = 0; x < pw; ++x) {
                int gv = bps == 1 ? g[size_t(y) * pw + x] : reinterpret_cast<const uint16_t *>(g)[size_t(y) * pw + x];
                const uint32_t tile = uint32_t((y << sy) / int(im.tile_height)) * im.cols + uint32_t((x << sx) / int(im.tile_width));
                const int want = tile % tstride == toff ? int(ref.plane[c][size_t(y) * pw + x])
                                                        : (bps == 1 ? kSentinel : kSentinel * 0x101);
                if (gv != want) {
                    if (!bad) fx = x, fy = y;
                    ++bad;
                }
            }
        printf("%s: %ld mismatches", names[c], bad);
        if (bad) {
            printf(" first at (%d,%d) tile (%d,%d) emu %d ref %d", fx, fy, (fy << sy) / int(im.tile_height),
                   (fx << sx) / int(im.tile_width),
                   bps == 1 ? g[size_t(fy) * pw + fx] : 0, ref.plane[c][size_t(fy) * pw + fx]);
        }
        printf("\n");
        bad_total += bad;
    }
    oracle_image_free(&ref);
    printf("%s\n", bad_total || st ? "EMU PARITY FAIL" : "EMU PARITY OK");
    return bad_total || st ? 1 : 0;
}
