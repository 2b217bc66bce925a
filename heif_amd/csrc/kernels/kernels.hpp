// kernels.hpp — launch interface of the gfx950 decode pipeline.
//
// Pipeline per batch (6 launches):
//   0. k_rbsp       emulation-prevention removal + entry-point remap (7.3.1.1)
//   1. k_parse_lanes CABAC substreams (one per lane) → TU records +
//                   coefficients + QP/edge maps + SAO parameters
//                   (slice.rs:206-256 + todo!()s)
//   2. k_transform  dequant (8.6.2-3) + inverse DST/DCT (8.6.4) → residuals
//   3. k_intra      intra prediction (8.4.4.2) + reconstruction (8.6.7)
//   4. k_deblock    vertical then horizontal edges (8.7.2), in place (after
//                   k_assemble puts sub-picture assemblies together, if any)
//   5. k_sao_out    SAO (8.7.3) + crop + grid placement into the caller's planes
#pragma once
#include "../common/desc.hpp"
#include "wave.hpp"
#include <cstdlib>
#include <vector>

#if defined(HG_HOST_EMU)
#include <atomic>
#include <thread>
#endif

namespace hg {

struct BatchArgs {
    const uint8_t *bits;       // raw NAL payloads
    const PicDesc *pics;
    const uint32_t *subs;      // substream raw start offsets (n_sub + 1 per picture, last = len)
    uint8_t *rbsp;             // k_rbsp: NAL payloads with emulation prevention removed (same offsets as bits)
    uint32_t *rsubs;           // k_rbsp: substream start offsets into rbsp (last = RBSP length)
    const uint32_t *parse_order;  // k_parse_lanes: picture (minus pic0) of wave slot i (~0u: empty); null = identity
    int n_slots;               // entries of parse_order (wave slots; a multiple of the pictures per wave)
    const SeqParams *seqs;
    const uint8_t *sf;         // ScalingFactor blocks
    const OutImage *outs;
    TuRec *tus;
    Coef *coefs;
    uint32_t *row_counts;      // [row] = {ntu, ncoef}
    uint8_t *recon;            // sample arena (uint8 or uint16 samples)
    int16_t *resid;
    uint8_t *maps;
    SaoParams *sao;
    uint32_t *status;          // per picture
    int n_pics;                // pictures of this launch: [pic0, pic0 + n_pics)
    int pic0;
    int max_width;             // luma samples, batch max
    int max_wctb;
    int max_rows;              // CTB rows, batch max
    int total_rows;            // sum of CTB rows over pictures
    int bytes_per_sample;      // 1 or 2
    int chroma_format;         // chroma_format_idc, shared by the batch's pictures
    int parse_group;           // k_parse_lanes pictures per wave (lanes_parse_order's choice; launch_parse otherwise)
    int max_log2ctb;           // largest CTB size in the batch (sizes k_intra's LDS)
    int lane_rows;             // k_parse_lanes lanes per picture: max over pictures of (WPP ? min(rows, 64) : 1)
    int wpp_ring;              // some WPP picture has more CTB rows than lanes (its rows wrap round its lanes)
    int parse_mode;            // PARSE_LANES (k_parse_lanes) or PARSE_SOLO (k_parse_solo)
    int solo_waves;            // k_parse_solo waves per workgroup (solo_waves_for(lane_rows))
    uint32_t *xprog;           // spread mode: per-row WPP progress words (total_rows)
    uint8_t *xctx;             // spread mode: per-row context hand-off blocks (total_rows * CTX_PAD)
    uint32_t *xntu;            // streaming mode: per-row TU records written so far (null otherwise)
    uint32_t *xjob;            // spread parse: the job counter each workgroup dequeues its substream job from
    int intra_stream;          // k_intra transforms and reconstructs each row behind the spread parse (same launch window)
    int stream_redo;           // k_intra_stream's second launch (after the parse): the pictures the first gave up on
    uint32_t stream_patience_us;  // first launch: give a picture up after this long without parse progress (0: at once)
    int has_assembly;          // some picture is PD_ASSEMBLY (launch_deblock runs k_assemble first)
    int intra_split;           // k_intra: luma and chroma on separate waves (set by launch_intra)
};

// k_ycbcr_rgb (color.hip): one decoded image → interleaved RGB8, rotated
struct ColorArgs {
    uint64_t plane[3];  // Y, Cb, Cr (device)
    int32_t pitch[3];   // bytes
    uint64_t rgb;       // device
    int32_t rgb_pitch;
    int32_t w, h;            // decoded (coded-orientation) size
    int32_t out_w, out_h;    // rotated size
    int32_t rotation;        // irot, anticlockwise 90-degree units
    int32_t chroma, shift;   // chroma_format_idc (0: no chroma planes); bit depth - 8
    int32_t yoff, ys;        // luma offset (16 limited range / 0 full) and scale (16.16)
    int32_t cr_r, cb_g, cr_g, cb_b;  // H.273 chroma weights (16.16, limited range rescaled)
};
// k_gather_tiles (gather.hip): tile windows k % stride == offset of src → dst
struct GatherArgs {
    uint64_t dst[3], src[3];  // planes (device pointers; src may be a peer / IPC mapping)
    int32_t dpitch[3], spitch[3];
    int32_t planes, bps;      // 1 or 3 planes, bytes per sample
    int32_t sx, sy;           // log2 chroma subsampling (chroma_sx / chroma_sy)
    int32_t W, H;             // luma output size
    int32_t tw, th, cols, n_tiles, stride, offset;
};
// H.273 coefficients for matrix_coefficients / video_full_range_flag, rounded to 16.16
inline void color_coefs(uint32_t matrix, bool full, ColorArgs &c) {
    double kr = 0.299, kb = 0.114;  // BT.601 (5, 6, and the unspecified default)
    if (matrix == 1) kr = 0.2126, kb = 0.0722;
    else if (matrix == 9) kr = 0.2627, kb = 0.0593;
    const double kg = 1.0 - kr - kb;
    const double ys = full ? 1.0 : 255.0 / 219.0, cs = full ? 1.0 : 255.0 / 224.0;
    auto fx = [](double v) { return (int32_t)(v * 65536.0 + 0.5); };
    c.yoff = full ? 0 : 16;
    c.ys = fx(ys);
    c.cr_r = fx(2.0 * (1.0 - kr) * cs);
    c.cb_b = fx(2.0 * (1.0 - kb) * cs);
    c.cb_g = fx(2.0 * kb * (1.0 - kb) / kg * cs);
    c.cr_g = fx(2.0 * kr * (1.0 - kr) / kg * cs);
}

// parse modes (BatchArgs::parse_mode; heifgpu_batch_opts::parse_mode)
// (4 was r05's row waves, HEIFGPU_PARSE_ROWS: removed in ABI 6, prepare answers HEIFGPU_E_UNSUPPORTED)
enum : int { PARSE_AUTO = 0, PARSE_LANES = 1, PARSE_SOLO = 2, PARSE_SPREAD = 3 };
constexpr int kSoloMaxWaves = 16;
// host: BatchArgs::parse_order for a batch (size-balanced k_parse_lanes waves,
// or for solo mode with ppw_force = 1 one picture per workgroup, heaviest
// first); returns the pictures per wave it dealt for (BatchArgs::parse_group).
// ppw_force = 0: the adaptive choice.
int lanes_parse_order(const PicDesc *pics, int n, int lane_rows, int ppw_force, std::vector<uint32_t> &order);
// k_intra_stream (reconstruction behind the spread parse, k_transform folded in) for this batch
// (same box, spread, one-decode latency: 4 images 28.3 vs 33.7 ms streamed; 8
// images 44.4 vs 40.5, the reconstruction no longer keeps up with the parse)
constexpr int kStreamMaxPics = 192;
struct StreamKnobs {
    bool enabled = true;
    int max_pics = kStreamMaxPics;
    uint32_t patience_us = 200000;  // first launch: give a picture up after this long without parse progress
};
StreamKnobs stream_knobs_from_env();
bool intra_stream_for(int parse_mode, int n_pics, bool has_assembly, const StreamKnobs &k);
// the parse mode a batch of n_pics pictures runs in (requested: PARSE_*)
// (pics: the batch's pictures; one with dependent slice segments starting inside a
// CTB row (PicDesc.flags, PD_NMID_SHIFT) makes it a lanes parse: only that engine takes them)
int parse_mode_for(int requested, int n_pics, const PicDesc *pics = nullptr);
// spread mode's wave slots (row << 20 | picture); -1 if the batch exceeds the encoding
int spread_parse_order(const PicDesc *pics, int n, std::vector<uint32_t> &order);
int solo_waves_for(int lane_rows);

#if defined(HG_HOST_EMU)
// Runs kernel(a) over a gx * gy grid, one block at a time, with `waves` host
// threads per block (threadIdx.x = 64 * wave).  grid_stride kernels (which
// loop t = blockIdx.x*blockDim.x+threadIdx.x .. total) get a 1x1 geometry in x.
template <class K>
void emu_launch(K kernel, int gx, int gy, int waves, const BatchArgs &a, bool grid_stride = false,
                size_t dyn_lds = 0) {
    for (int by = 0; by < gy; ++by)
        for (int bx = 0; bx < (grid_stride ? 1 : gx); ++bx) {
            std::atomic<int> cnt{0}, gen{0};
            std::vector<std::thread> th;
            unsigned char *lds = dyn_lds ? static_cast<unsigned char *>(std::malloc(dyn_lds)) : nullptr;
            for (int w = 0; w < waves; ++w)
                th.emplace_back([&, w] {
                    g_emu.bidx = {unsigned(bx), unsigned(by), 0};
                    g_emu.tidx = {unsigned(grid_stride ? 0 : 64 * w), 0, 0};
                    g_emu.bdim = {unsigned(grid_stride ? 1 : 64 * waves), 1, 1};
                    g_emu.gdim = {unsigned(grid_stride ? 1 : gx), unsigned(gy), 1};
                    g_emu.bar_count = &cnt;
                    g_emu.bar_gen = &gen;
                    g_emu.bar_n = waves;
                    g_emu.smem = lds;
                    kernel(a);
                });
            for (auto &t : th) t.join();
            std::free(lds);
        }
}
void emu_rbsp(const BatchArgs &a);
void emu_parse(const BatchArgs &a);
void emu_transform(const BatchArgs &a);
void emu_intra(const BatchArgs &a);
void emu_deblock(const BatchArgs &a);
void emu_sao_out(const BatchArgs &a);
#else
hipError_t launch_rbsp(const BatchArgs &a, hipStream_t s);
hipError_t launch_ycbcr_rgb(const ColorArgs &c, int bytes_per_sample, hipStream_t s);
hipError_t launch_gather_tiles(const GatherArgs &g, hipStream_t s);
hipError_t launch_parse(const BatchArgs &a, hipStream_t s);
hipError_t launch_transform(const BatchArgs &a, hipStream_t s);
hipError_t launch_intra(const BatchArgs &a, hipStream_t s);
hipError_t launch_deblock(const BatchArgs &a, hipStream_t s);
hipError_t launch_sao_out(const BatchArgs &a, hipStream_t s);
hipError_t launch_status_fold(const uint32_t *status, uint32_t *sticky, int n, hipStream_t s);
#endif

}  // namespace hg
