// api.cpp — C ABI (include/heifgpu.h): host parsing, batch flattening, device
// arenas and the five-stage launch sequence.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/heifgpu.h"
#include "common/desc.hpp"
#include "host/batch.hpp"
#include "host/heic_image.hpp"
#include "kernels/cabac.hpp"
#include "kernels/kernels.hpp"

using namespace hg;

struct heifgpu_image {
    ParsedImage img;
};

// the C structs' layouts are part of the ABI (INTEGRATION.md's Rust binding mirrors them)
static_assert(sizeof(heifgpu_image_info) == 80, "heifgpu_image_info: 20 x uint32");
static_assert(sizeof(heifgpu_planes) == 40, "heifgpu_planes: 3 pointers + 3 int32 (+ padding)");
static_assert(sizeof(heifgpu_batch_opts) == 20, "heifgpu_batch_opts: 5 x uint32");
static_assert(sizeof(heifgpu_ipc_handle) == 72, "heifgpu_ipc_handle: 64-byte HIP handle + uint64 offset");
static_assert(HEIFGPU_PARSE_AUTO == PARSE_AUTO && HEIFGPU_PARSE_LANES == PARSE_LANES && HEIFGPU_PARSE_SOLO == PARSE_SOLO &&
                  HEIFGPU_PARSE_SPREAD == PARSE_SPREAD,
              "parse modes");
static_assert(sizeof(heifgpu_tile_params) == 55 * 4 + 64 * 4, "heifgpu_tile_params: 55 int32 + 64 uint32");

// Pipelined decode.  k_rbsp + k_parse run on an internal parse stream, the
// four reconstruction kernels on an internal recon stream.  A batch holds two
// sets of parse outputs (TU records, coefficients, maps, SAO, per-row counts,
// status, residual planes) used by alternate decode calls, so the parse of
// call n + 1 runs while call n reconstructs: neither depends on anything the
// caller can touch (the bitstreams are the batch's own) except k_sao_out,
// which writes the caller's planes and so waits for everything the caller
// enqueued on its stream before the call; the caller's stream waits for
// k_sao_out.  A set is reused only after the reconstruction that read it.
// HEIFGPU_PIPELINE=0 or 1 keeps one set (no overlap), 2 two sets on two
// streams (before r04 every value but 0 and 3 meant two); the default, 3 (or
// more), uses three sets and a third stream for k_transform, so
// parse n + 2, transform n + 1 and reconstruction n overlap.  While the parse
// was the critical path (r02) three sets lost (15.32 / 15.33 vs 15.67 / 15.64
// Gpix/s); since the r03 parse got faster the reconstruction stream sets the
// step and three sets win (same-box pairs at 20 steps: 18.56 / 18.49 vs
// 17.86 / 17.77 Gpix/s, profiles/r03d/ab_pipeline_sets.txt).
constexpr int kTimingSlots = 32;
struct heifgpu_ctx {
    int device = 0;
    bool timing = false;
    hipStream_t parse = nullptr, xform = nullptr, recon = nullptr, upload = nullptr;
    // k_rbsp of the next decode (its parse set's RBSP and zeroed words) beside the
    // running parse instead of in front of the next one on the parse stream
    hipStream_t prep = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    StreamKnobs stream;  // the streaming knobs, read once at heifgpu_create
    // timing ring, one slot per timed decode call: rbsp start, rbsp end, parse
    // end, transform start, transform end, recon start, 3 stage ends, parse
    // start.  heifgpu_stage_times folds every call since the previous query (a
    // slot about to be reused is folded first).
    hipEvent_t tev[kTimingSlots][10] = {};
    int timed_calls = 0, folded = 0;
    double acc[6] = {};
};

namespace {
// per-set words of the spread and rows parses: one progress word per CTB row, then the job counter
size_t xprog_words(const HostBatch &hb) { return size_t(hb.rows) + 1; }
// k_intra_stream: one TU count per CTB row, then one done word per picture (+ 1 spare)
size_t xntu_words(const HostBatch &hb) { return size_t(hb.rows) + hb.pics.size() + 1; }

// k_rbsp on its own stream (HEIFGPU_PREP_STREAM=0/1, read at context creation)
bool prep_stream_default() {
    const char *e = std::getenv("HEIFGPU_PREP_STREAM");
    return e && std::atoi(e) != 0;
}

// adds the stage times of the decode call recorded in `slot` to ctx->acc
hipError_t fold_timing(heifgpu_ctx *ctx, int slot) {
    hipEvent_t *e = ctx->tev[slot];
    hipError_t r = hipEventSynchronize(e[8]);
    if (r != hipSuccess) return r;
    float t = 0.f;
    if ((r = hipEventElapsedTime(&t, e[0], e[1])) != hipSuccess) return r;
    ctx->acc[5] += t;  // k_rbsp
    if ((r = hipEventElapsedTime(&t, e[9], e[2])) != hipSuccess) return r;
    ctx->acc[0] += t;  // k_parse
    if ((r = hipEventElapsedTime(&t, e[3], e[4])) != hipSuccess) return r;
    ctx->acc[1] += t;  // k_transform
    for (int i = 2; i < 5; ++i) {  // k_intra, k_deblock, k_sao_out
        if ((r = hipEventElapsedTime(&t, e[i + 3], e[i + 4])) != hipSuccess) return r;
        ctx->acc[i] += t;
    }
    return hipSuccess;
}
}  // namespace

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

// Test hook: HEIFGPU_FAULT_INJECT names a failure to inject ("prepare": a
// reload fails after it has begun to overwrite its descriptor generation).
// Read at every call, so one test process can switch it on and off.
bool fault_injected(const char *what) {
    const char *e = std::getenv("HEIFGPU_FAULT_INJECT");
    return e && std::strcmp(e, what) == 0;
}

#define HIP_TRY(expr)                                                                             \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return fail(HEIFGPU_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    size_t cap = 0;
    // count elements, reusing the allocation when it is large enough (a
    // reloaded batch, heifgpu_batch_prepare_ex); the caller has drained every
    // use of the old contents before a reallocation
    hipError_t alloc(size_t count) {
        n = count;
        if (p && count <= cap) return hipSuccess;
        if (p) {
            hipError_t e = hipFree(p);
            p = nullptr;
            cap = 0;
            if (e != hipSuccess) return e;
        }
        cap = std::max<size_t>(count, 1);
        return hipMalloc(reinterpret_cast<void **>(&p), cap * sizeof(T));
    }
};

// page-locked host staging of a batch's uploads (one hipMemcpyAsync source)
struct PinnedBuf {
    uint8_t *p = nullptr;
    size_t cap = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf &) = delete;
    PinnedBuf &operator=(const PinnedBuf &) = delete;
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
    hipError_t reserve(size_t bytes) {
        if (p && bytes <= cap) return hipSuccess;
        if (p) {
            hipError_t e = hipHostFree(p);
            p = nullptr;
            cap = 0;
            if (e != hipSuccess) return e;
        }
        cap = std::max<size_t>(bytes, 4096);
        return hipHostMalloc(reinterpret_cast<void **>(&p), cap, hipHostMallocDefault);
    }
};

}  // namespace

// outputs of one k_parse run (see heifgpu_ctx)
struct ParseSet {
    DevBuf<TuRec> tus;
    DevBuf<Coef> coefs;
    DevBuf<uint32_t> row_counts, status;
    DevBuf<uint8_t> maps;
    DevBuf<SaoParams> sao;
    DevBuf<int16_t> resid;  // k_transform -> k_intra
    // spread mode: per-row WPP progress words and (streaming) TU counts, per set
    // because k_intra_stream of this set's decode polls them while the next
    // decode's parse already runs
    DevBuf<uint32_t> xprog, xntu;
    // k_rbsp's output, per set so that the next decode's k_rbsp can run while
    // this set's parse still reads it
    DevBuf<uint8_t> rbsp;
    DevBuf<uint32_t> rsubs;
    hipEvent_t parsed = nullptr, transformed = nullptr, recon_done = nullptr, progreset = nullptr, prepped = nullptr;
    bool pending = false;  // recon_done recorded and not yet waited for by a parse
    ~ParseSet() {
        if (parsed) (void)hipEventDestroy(parsed);
        if (transformed) (void)hipEventDestroy(transformed);
        if (recon_done) (void)hipEventDestroy(recon_done);
        if (progreset) (void)hipEventDestroy(progreset);
        if (prepped) (void)hipEventDestroy(prepped);
    }
};

// The descriptors every stage reads (pictures, sequences, scaling factors,
// output planes) and the sticky status, in two generations: a reload writes
// the generation the previous load did not use, so it waits only for the
// decodes of the load before that (`done`), not for the ones in flight.
struct DescGen {
    DevBuf<PicDesc> pics;
    DevBuf<SeqParams> seqs;
    DevBuf<uint8_t> sf;
    DevBuf<OutImage> outs;
    DevBuf<uint32_t> sticky;  // per picture: OR of every decode's status since the last heifgpu_batch_status
    std::vector<OutImage> out_host;
    hipEvent_t done = nullptr;  // the last decode that read this generation (recon stream)
    bool pending = false;
    // the load this generation holds: picture -> image, image count (heifgpu_batch_status_previous
    // maps the sticky words of the load before the current one with these)
    std::vector<uint32_t> pic_image;
    size_t n_images = 0;
    bool loaded = false;
    ~DescGen() {
        if (done) (void)hipEventDestroy(done);
    }
};

struct heifgpu_batch {
    int device = 0;
    size_t n_images = 0;
    int n_pics = 0;
    uint32_t tile_stride = 1, tile_offset = 0;
    PinnedBuf stage;
    hipEvent_t uploaded = nullptr;  // the last load's H2D copies (upload stream)
    bool loaded = false;
    BatchArgs args{};
    // read by k_rbsp / the parse only: a reload waits for the parses in flight
    DevBuf<uint8_t> bits;
    DevBuf<uint32_t> subs, porder;
    DevBuf<uint8_t> xctx;
    // the sample arena: written by k_intra, which runs after every earlier
    // decode's k_sao_out on the one recon stream
    DevBuf<uint8_t> recon;
    DescGen gen[2];
    int cur = 0;
    ParseSet set[3];
    int n_sets = 1, next_set = 0, last_set = 0;
    std::vector<uint32_t> pic_image;  // picture → image
    std::vector<heifgpu_image_info> infos;
    ~heifgpu_batch() {
        if (uploaded) (void)hipEventDestroy(uploaded);
    }
};

extern "C" {

const char *heifgpu_last_error(void) { return g_err.c_str(); }

int heifgpu_image_parse(const uint8_t *data, size_t len, heifgpu_image **out) {
    return heifgpu_image_parse_item(data, len, 0, out);
}

int heifgpu_image_parse_item(const uint8_t *data, size_t len, uint32_t item_id, heifgpu_image **out) {
    if (!data || !out) return fail(HEIFGPU_E_INVALID, "null argument");
    *out = nullptr;
    try {
        auto im = std::make_unique<heifgpu_image>();
        im->img = parse_heic(data, len, item_id);
        *out = im.release();
        return HEIFGPU_OK;
    } catch (const UnsupportedError &e) {
        return fail(HEIFGPU_E_UNSUPPORTED, e.what());
    } catch (const std::exception &e) {
        return fail(HEIFGPU_E_PARSE, e.what());
    }
}

int heifgpu_image_parse_many(const uint8_t *const *data, const size_t *len, size_t n, int threads,
                             heifgpu_image **out, int *rc) {
    if (!data || !len || !out) return fail(HEIFGPU_E_INVALID, "null argument");
    for (size_t i = 0; i < n; ++i) out[i] = nullptr;
    std::vector<int> codes(n, HEIFGPU_OK);
    std::vector<std::string> msgs(n);
    std::atomic<size_t> next{0};
    auto worker = [&] {
        for (size_t i; (i = next.fetch_add(1)) < n;) {
            if (!data[i]) {
                codes[i] = HEIFGPU_E_INVALID;
                msgs[i] = "null data";
                continue;
            }
            try {
                auto im = std::make_unique<heifgpu_image>();
                im->img = parse_heic(data[i], len[i], 0);
                out[i] = im.release();
            } catch (const UnsupportedError &e) {
                codes[i] = HEIFGPU_E_UNSUPPORTED;
                msgs[i] = e.what();
            } catch (const std::exception &e) {
                codes[i] = HEIFGPU_E_PARSE;
                msgs[i] = e.what();
            }
        }
    };
    size_t nt = threads > 0 ? size_t(threads) : size_t(std::max(1u, std::thread::hardware_concurrency()));
    nt = std::min(nt, n);
    std::vector<std::thread> pool;
    for (size_t t = 1; t < nt; ++t) pool.emplace_back(worker);
    worker();
    for (auto &th : pool) th.join();
    int first = HEIFGPU_OK;
    for (size_t i = 0; i < n; ++i) {
        if (rc) rc[i] = codes[i];
        if (codes[i] != HEIFGPU_OK && first == HEIFGPU_OK) {
            first = codes[i];
            g_err = "image " + std::to_string(i) + ": " + msgs[i];
        }
    }
    return first;
}

int heifgpu_gather_tiles(const heifgpu_image_info *info, const heifgpu_planes *dst, const heifgpu_planes *src,
                         uint32_t tile_stride, uint32_t tile_offset, void *stream) {
    if (!info || !dst || !src) return fail(HEIFGPU_E_INVALID, "null argument");
    if (tile_stride == 0) tile_stride = 1;
    if (tile_offset >= tile_stride) return fail(HEIFGPU_E_INVALID, "tile_offset must be below tile_stride");
    if (info->chroma_format_idc > 3) return fail(HEIFGPU_E_INVALID, "chroma_format_idc");
    const int planes = info->chroma_format_idc ? 3 : 1;
    for (int c = 0; c < planes; ++c)
        if (!dst->plane[c] || !src->plane[c]) return fail(HEIFGPU_E_INVALID, "missing plane");
    hipPointerAttribute_t ad{}, as{};
    HIP_TRY(hipPointerGetAttributes(&ad, dst->plane[0]));
    HIP_TRY(hipPointerGetAttributes(&as, src->plane[0]));
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    HIP_TRY(hipSetDevice(ad.device));
    if (ad.device != as.device) {  // a pointer of another device in this process: read it over xGMI
        const hipError_t e = hipDeviceEnablePeerAccess(as.device, 0);
        (void)hipGetLastError();
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
            (void)hipSetDevice(cur);
            HIP_TRY(e);
        }
    }
    GatherArgs g{};
    for (int c = 0; c < 3; ++c) {
        g.dst[c] = reinterpret_cast<uint64_t>(dst->plane[c]);
        g.src[c] = reinterpret_cast<uint64_t>(src->plane[c]);
        g.dpitch[c] = dst->pitch[c];
        g.spitch[c] = src->pitch[c];
    }
    g.planes = planes;
    g.sx = chroma_sx(int(info->chroma_format_idc));
    g.sy = chroma_sy(int(info->chroma_format_idc));
    g.bps = int32_t(info->bytes_per_sample);
    g.W = int32_t(info->width);
    g.H = int32_t(info->height);
    g.cols = int32_t(std::max(1u, info->grid_cols));
    g.tw = int32_t(info->tile_width ? info->tile_width : info->width);
    g.th = int32_t(info->tile_height ? info->tile_height : info->height);
    g.n_tiles = int32_t(std::max(1u, info->num_tiles));
    g.stride = int32_t(tile_stride);
    g.offset = int32_t(tile_offset);
    const hipError_t e = launch_gather_tiles(g, static_cast<hipStream_t>(stream));
    (void)hipSetDevice(cur);
    HIP_TRY(e);
    return HEIFGPU_OK;
}

namespace {
std::mutex g_ipc_mu;
std::vector<std::pair<void *, void *>> g_ipc_open;  // (pointer returned, mapping base)
}  // namespace

int heifgpu_ipc_export(const void *dev_ptr, heifgpu_ipc_handle *out) {
    static_assert(sizeof(hipIpcMemHandle_t) == sizeof(out->handle), "hipIpcMemHandle_t is 64 bytes");
    if (!dev_ptr || !out) return fail(HEIFGPU_E_INVALID, "null argument");
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    HIP_TRY(hipMemGetAddressRange(&base, &size, const_cast<void *>(dev_ptr)));
    hipIpcMemHandle_t h;
    HIP_TRY(hipIpcGetMemHandle(&h, base));
    std::memcpy(out->handle, &h, sizeof(h));
    out->offset = uint64_t(static_cast<const uint8_t *>(dev_ptr) - static_cast<const uint8_t *>(base));
    return HEIFGPU_OK;
}

int heifgpu_ipc_open(int device, const heifgpu_ipc_handle *h, void **dev_ptr) {
    if (!h || !dev_ptr) return fail(HEIFGPU_E_INVALID, "null argument");
    *dev_ptr = nullptr;
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    HIP_TRY(hipSetDevice(device));
    hipIpcMemHandle_t mh;
    std::memcpy(&mh, h->handle, sizeof(mh));
    void *base = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&base, mh, hipIpcMemLazyEnablePeerAccess);
    (void)hipSetDevice(cur);
    HIP_TRY(e);
    *dev_ptr = static_cast<uint8_t *>(base) + h->offset;
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    g_ipc_open.emplace_back(*dev_ptr, base);
    return HEIFGPU_OK;
}

int heifgpu_ipc_close(void *dev_ptr) {
    void *base = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_ipc_mu);
        for (size_t i = 0; i < g_ipc_open.size(); ++i)
            if (g_ipc_open[i].first == dev_ptr) {
                base = g_ipc_open[i].second;
                g_ipc_open.erase(g_ipc_open.begin() + long(i));
                break;
            }
    }
    if (!base) return fail(HEIFGPU_E_INVALID, "not a pointer returned by heifgpu_ipc_open");
    HIP_TRY(hipIpcCloseMemHandle(base));
    return HEIFGPU_OK;
}

int heifgpu_image_get_info(const heifgpu_image *img, heifgpu_image_info *info) {
    if (!img || !info) return fail(HEIFGPU_E_INVALID, "null argument");
    const ParsedImage &p = img->img;
    const SequenceParameterSet &s = p.params[0].sps;
    std::memset(info, 0, sizeof(*info));
    info->width = p.out_width;
    info->height = p.out_height;
    info->chroma_format_idc = uint32_t(s.chroma_array_type());
    info->bit_depth = uint32_t(8 + s.bit_depth_luma_minus8);
    info->bytes_per_sample = info->bit_depth > 8 ? 2 : 1;
    info->grid_rows = p.rows;
    info->grid_cols = p.cols;
    info->tile_width = p.tile_width;
    info->tile_height = p.tile_height;
    info->num_tiles = uint32_t(p.tiles.size());
    info->rotation = p.rotation;
    info->ispe_width = p.ispe_width;
    info->ispe_height = p.ispe_height;
    info->coded_bytes = p.coded_bytes;
    info->primary_item_id = p.primary_item_id;
    info->num_thumbnails = p.num_thumbnails;
    info->matrix_coeffs = p.nclx ? p.nclx_matrix : uint32_t(s.matrix_coeffs);
    info->full_range = p.nclx ? p.nclx_full_range : (s.video_full_range_flag ? 1u : 0u);
    info->item_id = p.item_id;
    info->aux_item_id = p.aux_item_id;
    return HEIFGPU_OK;
}

int heifgpu_ycbcr_to_rgb(heifgpu_ctx *ctx, const heifgpu_image_info *info, const heifgpu_planes *in, void *rgb,
                         int32_t rgb_pitch, void *stream) {
    if (!ctx || !info || !in || !rgb || !in->plane[0]) return fail(HEIFGPU_E_INVALID, "invalid argument");
    if (info->chroma_format_idc > 3) return fail(HEIFGPU_E_INVALID, "chroma_format_idc");
    if (info->chroma_format_idc && (!in->plane[1] || !in->plane[2])) return fail(HEIFGPU_E_INVALID, "missing chroma plane");
    if (info->bit_depth < 8 || info->bit_depth > 16) return fail(HEIFGPU_E_INVALID, "bit depth");
    HIP_TRY(hipSetDevice(ctx->device));
    ColorArgs c{};
    for (int k = 0; k < 3; ++k) {
        c.plane[k] = reinterpret_cast<uint64_t>(in->plane[k]);
        c.pitch[k] = in->pitch[k];
    }
    c.rgb = reinterpret_cast<uint64_t>(rgb);
    c.rgb_pitch = rgb_pitch;
    c.w = int32_t(info->width);
    c.h = int32_t(info->height);
    c.rotation = int32_t(info->rotation & 3);
    c.out_w = (c.rotation & 1) ? c.h : c.w;
    c.out_h = (c.rotation & 1) ? c.w : c.h;
    if (rgb_pitch < 3 * c.out_w) return fail(HEIFGPU_E_INVALID, "rgb_pitch smaller than 3 * output width");
    c.chroma = int32_t(info->chroma_format_idc);
    c.shift = int32_t(info->bit_depth) - 8;
    color_coefs(info->matrix_coeffs, info->full_range != 0, c);
    HIP_TRY(launch_ycbcr_rgb(c, int(info->bytes_per_sample), static_cast<hipStream_t>(stream)));
    return HEIFGPU_OK;
}

void heifgpu_image_free(heifgpu_image *img) { delete img; }

int heifgpu_create(int device, heifgpu_ctx **out) {
    if (!out) return fail(HEIFGPU_E_INVALID, "null argument");
    *out = nullptr;
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(HEIFGPU_E_DEVICE, "no such HIP device");
    HIP_TRY(hipSetDevice(device));
    auto c = std::make_unique<heifgpu_ctx>();
    c->device = device;
    c->stream = stream_knobs_from_env();
    // parse and reconstruction streams at the same priority: with the parse
    // stream at the highest priority (HEIFGPU_PARSE_PRIORITY=1) k_transform
    // starves beside it and the bench measured 1 % lower (two A/B pairs,
    // 14909 / 14881 vs 15039 / 15058 Mpix/s)
    static const bool prio = [] {
        const char *e = std::getenv("HEIFGPU_PARSE_PRIORITY");
        return e && std::atoi(e) != 0;
    }();
    int least = 0, greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_TRY(hipStreamCreateWithPriority(&c->parse, hipStreamNonBlocking, prio ? greatest : least));
    // HEIFGPU_RECON_PRIORITY=1: the transform and reconstruction streams at the
    // highest priority instead (tuning knob; the recon stream sets the step)
    static const bool rprio = [] {
        const char *e = std::getenv("HEIFGPU_RECON_PRIORITY");
        return e && std::atoi(e) != 0;
    }();
    HIP_TRY(hipStreamCreateWithPriority(&c->xform, hipStreamNonBlocking, rprio ? greatest : least));
    HIP_TRY(hipStreamCreateWithPriority(&c->recon, hipStreamNonBlocking, rprio ? greatest : least));
    HIP_TRY(hipStreamCreateWithFlags(&c->upload, hipStreamNonBlocking));
    if (prep_stream_default()) HIP_TRY(hipStreamCreateWithFlags(&c->prep, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&c->fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->join, hipEventDisableTiming));
    for (auto &row : c->tev)
        for (auto &e : row) HIP_TRY(hipEventCreate(&e));
    *out = c.release();
    return HEIFGPU_OK;
}

void heifgpu_destroy(heifgpu_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    for (auto &row : ctx->tev)
        for (auto &e : row)
            if (e) (void)hipEventDestroy(e);
    if (ctx->fork) (void)hipEventDestroy(ctx->fork);
    if (ctx->join) (void)hipEventDestroy(ctx->join);
    if (ctx->parse) (void)hipStreamDestroy(ctx->parse);
    if (ctx->xform) (void)hipStreamDestroy(ctx->xform);
    if (ctx->recon) (void)hipStreamDestroy(ctx->recon);
    if (ctx->upload) (void)hipStreamDestroy(ctx->upload);
    if (ctx->prep) (void)hipStreamDestroy(ctx->prep);
    delete ctx;
}

int heifgpu_set_timing(heifgpu_ctx *ctx, int enable) {
    if (!ctx) return fail(HEIFGPU_E_INVALID, "null ctx");
    if (enable && !ctx->timing) {  // a fresh accumulation
        for (double &v : ctx->acc) v = 0.0;
        ctx->timed_calls = ctx->folded = 0;
    }
    ctx->timing = enable != 0;
    return HEIFGPU_OK;
}

int heifgpu_stage_times(heifgpu_ctx *ctx, float ms[6]) {
    if (!ctx || !ms) return fail(HEIFGPU_E_INVALID, "null argument");
    if (!ctx->timing) return fail(HEIFGPU_E_INVALID, "timing disabled");
    // mean per decode call over the timed calls since the previous query
    for (int i = 0; i < 6; ++i) ms[i] = 0.f;
    for (int c = ctx->folded; c < ctx->timed_calls; ++c) HIP_TRY(fold_timing(ctx, c % kTimingSlots));
    if (ctx->timed_calls)
        for (int i = 0; i < 6; ++i) ms[i] = float(ctx->acc[i] / ctx->timed_calls);
    for (double &v : ctx->acc) v = 0.0;
    ctx->timed_calls = ctx->folded = 0;
    return HEIFGPU_OK;
}

int heifgpu_batch_prepare_ex(heifgpu_ctx *ctx, const heifgpu_image *const *imgs, size_t n,
                             const heifgpu_batch_opts *opts, heifgpu_batch **inout) {
    if (!ctx || !imgs || !inout || n == 0) return fail(HEIFGPU_E_INVALID, "invalid argument");
    const uint32_t stride = opts && opts->tile_stride ? opts->tile_stride : 1u;
    const uint32_t offset = opts ? opts->tile_offset : 0u;
    if (offset >= stride) return fail(HEIFGPU_E_INVALID, "tile_offset must be below tile_stride");
    const uint32_t mode_req = opts ? opts->parse_mode : 0u;
    if (mode_req > HEIFGPU_PARSE_ROWS) return fail(HEIFGPU_E_INVALID, "parse_mode");
    if (mode_req == HEIFGPU_PARSE_ROWS)
        return fail(HEIFGPU_E_UNSUPPORTED, "HEIFGPU_PARSE_ROWS was removed in ABI 6 (DESIGN.md 5.9)");
    const int ppw_req = opts ? int(std::min<uint32_t>(opts->pics_per_wave, 64u)) : 0;
    if (*inout && (*inout)->device != ctx->device) return fail(HEIFGPU_E_INVALID, "batch belongs to another device");
    HIP_TRY(hipSetDevice(ctx->device));
    std::vector<const ParsedImage *> parsed;
    std::vector<heifgpu_image_info> infos;
    for (size_t i = 0; i < n; ++i) {
        if (!imgs[i]) return fail(HEIFGPU_E_INVALID, "null image");
        parsed.push_back(&imgs[i]->img);
        heifgpu_image_info info;
        heifgpu_image_get_info(imgs[i], &info);
        infos.push_back(info);
    }
    HostBatch hb;
    try {
        hb = build_batch(parsed.data(), n, stride, offset, /*defer_bits=*/true);
    } catch (const UnsupportedError &e) {
        return fail(HEIFGPU_E_UNSUPPORTED, e.what());
    } catch (const std::exception &e) {
        return fail(HEIFGPU_E_PARSE, e.what());
    }
    std::unique_ptr<heifgpu_batch> fresh;
    heifgpu_batch *b = *inout;
    if (!b) {
        fresh = std::make_unique<heifgpu_batch>();
        b = fresh.get();
        b->device = ctx->device;
        HIP_TRY(hipEventCreateWithFlags(&b->uploaded, hipEventDisableTiming));
        static const int pipeline = [] {
            const char *e = std::getenv("HEIFGPU_PIPELINE");
            return e ? std::atoi(e) : 3;
        }();
        // sets of parse outputs: the batch's own choice, else HEIFGPU_PIPELINE (default 3)
        const int sets = opts && opts->pipeline_sets ? int(opts->pipeline_sets) : pipeline;
        b->n_sets = sets <= 1 ? 1 : (sets >= 3 ? 3 : 2);
        for (int k = 0; k < b->n_sets; ++k) {
            HIP_TRY(hipEventCreateWithFlags(&b->set[k].parsed, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&b->set[k].transformed, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&b->set[k].recon_done, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&b->set[k].progreset, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&b->set[k].prepped, hipEventDisableTiming));
        }
        for (DescGen &g : b->gen) HIP_TRY(hipEventCreateWithFlags(&g.done, hipEventDisableTiming));
    }
    // A reloaded batch.  The staging buffer is rewritten only after the
    // previous load's copies (long finished in a double-buffered loop).  The
    // upload stream then waits for
    // - the parses in flight (they read bits / rbsp / subs / the parse order);
    // - the decodes of the load before the previous one, which read the
    //   descriptor generation this load overwrites;
    // not for the in-flight decodes' transform and reconstruction, which read
    // only their parse set, the other generation and the sample arena (that
    // one is ordered by the recon stream).
    // (unconditionally: a reload that failed may have issued copies from staging)
    HIP_TRY(hipEventSynchronize(b->uploaded));
    // The generation the last successful load did not use (not the
    // one of b->loaded, which a failed reload clears while gen[cur] still holds
    // the last good load, its in-flight decodes and their sticky status)
    const int gi = b->gen[b->cur].loaded ? b->cur ^ 1 : b->cur;
    DescGen &G = b->gen[gi];
    for (int k = 0; k < b->n_sets; ++k)
        if (b->set[k].pending) HIP_TRY(hipStreamWaitEvent(ctx->upload, b->set[k].parsed, 0));
    if (G.pending) HIP_TRY(hipStreamWaitEvent(ctx->upload, G.done, 0));
    std::vector<uint32_t> order;
    const int mode = parse_mode_for(int(mode_req), int(hb.pics.size()), hb.pics.data());
    const int solo_waves = solo_waves_for(hb.lane_rows);
    int parse_group = 1;
    if (mode == PARSE_SPREAD) {
        if (spread_parse_order(hb.pics.data(), int(hb.pics.size()), order) < 0)
            return fail(HEIFGPU_E_UNSUPPORTED, "spread parse: over 2^20 pictures or 4096 substreams per picture");
    } else {  // pictures dealt by payload size (r03: dealing by WPP critical path lost, 16.9 vs 17.0 Gpix/s)
        parse_group = lanes_parse_order(hb.pics.data(), int(hb.pics.size()), hb.lane_rows,
                                        mode == PARSE_SOLO ? 1 : ppw_req, order);
    }
    // spread parse: WPP neighbours in other waves (progress words,
    // context hand-off blocks, the job counter after the progress words)
    const bool cross_rows = mode == PARSE_SPREAD;
    const bool grows = (order.size() > b->porder.cap || hb.bits_size > b->bits.cap || hb.bits_size > b->set[0].rbsp.cap || hb.pics.size() > G.pics.cap ||
                                     hb.subs.size() > b->subs.cap || hb.seqs.size() > G.seqs.cap ||
                                     hb.sf.size() > G.sf.cap || n > G.outs.cap || hb.recon_bytes > b->recon.cap ||
                                     hb.resid_elems > b->set[0].resid.cap || hb.tu_n > b->set[0].tus.cap ||
                                     hb.coef_n > b->set[0].coefs.cap || hb.map_bytes > b->set[0].maps.cap ||
                                     hb.sao_n > b->set[0].sao.cap || 2 * size_t(hb.rows) > b->set[0].row_counts.cap ||
                                     hb.pics.size() > b->set[0].status.cap || hb.pics.size() > G.sticky.cap ||
                                     (cross_rows && (xprog_words(hb) > b->set[0].xprog.cap || hb.rows * CTX_PAD > b->xctx.cap)) ||
                                     (mode == PARSE_SPREAD && xntu_words(hb) > b->set[0].xntu.cap));
    if (grows) {  // reallocation: every decode of the old contents fully drained
        for (int k = 0; k < b->n_sets; ++k)
            if (b->set[k].pending) HIP_TRY(hipEventSynchronize(b->set[k].recon_done));
        HIP_TRY(hipStreamSynchronize(ctx->upload));
    }
    // A failure from here on leaves the batch unusable until a reload succeeds
    // (its arguments may point at freed arenas): `loaded` is set again last.
    b->loaded = false;
    G.loaded = false;  // its previous contents (two loads back) are overwritten from here on
    G.pic_image.clear();
    G.n_images = 0;
    if (fault_injected("prepare"))  // test hook: a reload that fails after touching the generation
        return fail(HEIFGPU_E_INVALID, "injected prepare failure (HEIFGPU_FAULT_INJECT=prepare)");
    // ---- device arenas (reused when large enough)
    HIP_TRY(b->bits.alloc(hb.bits_size));
    HIP_TRY(G.pics.alloc(hb.pics.size()));
    HIP_TRY(b->subs.alloc(hb.subs.size()));
    HIP_TRY(G.seqs.alloc(hb.seqs.size()));
    HIP_TRY(G.sf.alloc(hb.sf.size()));
    HIP_TRY(G.outs.alloc(n));
    HIP_TRY(G.sticky.alloc(hb.pics.size()));
    HIP_TRY(hipMemsetAsync(G.sticky.p, 0, hb.pics.size() * sizeof(uint32_t), ctx->upload));
    for (int k = 0; k < b->n_sets; ++k) {
        ParseSet &ps = b->set[k];
        HIP_TRY(ps.tus.alloc(hb.tu_n));
        HIP_TRY(ps.coefs.alloc(hb.coef_n));
        HIP_TRY(ps.row_counts.alloc(size_t(2) * hb.rows));
        HIP_TRY(ps.maps.alloc(hb.map_bytes));
        HIP_TRY(ps.sao.alloc(hb.sao_n));
        HIP_TRY(ps.status.alloc(hb.pics.size()));
        HIP_TRY(ps.resid.alloc(hb.resid_elems));  // (each decode zeroes its set's status before the parse)
        HIP_TRY(ps.rbsp.alloc(hb.bits_size));
        HIP_TRY(ps.rsubs.alloc(hb.subs.size()));
    }
    HIP_TRY(b->recon.alloc(hb.recon_bytes));
    HIP_TRY(b->porder.alloc(order.size()));
    if (cross_rows) {  // per-row WPP progress words (+ the job counter) and context hand-off blocks
        for (int k = 0; k < b->n_sets; ++k) {
            HIP_TRY(b->set[k].xprog.alloc(xprog_words(hb)));
            if (mode == PARSE_SPREAD) HIP_TRY(b->set[k].xntu.alloc(xntu_words(hb)));
        }
        HIP_TRY(b->xctx.alloc(std::max<size_t>(hb.rows, 1) * CTX_PAD));
    }
    // ---- one pinned staging image of every upload, copied asynchronously
    struct Seg {
        const void *src;
        size_t bytes;
        void *dst;
    };
    const Seg segs[] = {
        {nullptr, hb.bits_size, b->bits.p},  // the payload pieces, copied below
        {hb.pics.data(), hb.pics.size() * sizeof(PicDesc), G.pics.p},
        {hb.subs.data(), hb.subs.size() * sizeof(uint32_t), b->subs.p},
        {hb.seqs.data(), hb.seqs.size() * sizeof(SeqParams), G.seqs.p},
        {hb.sf.data(), hb.sf.size(), G.sf.p},
        {order.data(), order.size() * sizeof(uint32_t), b->porder.p},
    };
    size_t total = 0;
    for (const Seg &g : segs) total += (g.bytes + 255) & ~size_t(255);
    HIP_TRY(b->stage.reserve(total));
    {  // the bitstreams (most of the bytes) straight from the parsed images into staging, on a few threads
        uint8_t *dst = b->stage.p;
        const size_t np = hb.pieces.size();
        const size_t nt = std::min<size_t>(std::max(1u, std::min(16u, std::thread::hardware_concurrency())),
                                           (hb.bits_size >> 22) + 1);  // ~4 MB per thread at least
        std::atomic<size_t> next{0};
        auto copy = [&] {
            for (size_t i; (i = next.fetch_add(64)) < np;)
                for (size_t j = i; j < std::min(np, i + 64); ++j) {
                    const HostBatch::Piece &pc = hb.pieces[j];
                    std::memcpy(dst + pc.dst, pc.src, pc.len);
                    const size_t end = j + 1 < np ? hb.pieces[j + 1].dst : hb.bits_size;
                    std::memset(dst + pc.dst + pc.len, 0, end - pc.dst - pc.len);  // alignment padding
                }
        };
        std::vector<std::thread> pool;
        for (size_t t = 1; t < nt; ++t) pool.emplace_back(copy);
        copy();
        for (auto &th : pool) th.join();
        if (np == 0) std::memset(dst, 0, hb.bits_size);
    }
    size_t off = 0;
    for (const Seg &g : segs) {
        if (g.bytes) {
            if (g.src) std::memcpy(b->stage.p + off, g.src, g.bytes);
            HIP_TRY(hipMemcpyAsync(g.dst, b->stage.p + off, g.bytes, hipMemcpyHostToDevice, ctx->upload));
        }
        off += (g.bytes + 255) & ~size_t(255);
    }
    for (int k = 0; k < b->n_sets; ++k) HIP_TRY(hipMemsetAsync(b->set[k].rbsp.p, 0, hb.bits_size, ctx->upload));
    HIP_TRY(hipEventRecord(b->uploaded, ctx->upload));
    b->n_images = n;
    b->tile_stride = stride;
    b->tile_offset = offset;
    b->infos = std::move(infos);
    b->pic_image = hb.pic_image;
    G.pic_image = hb.pic_image;
    G.n_images = n;
    G.loaded = true;
    b->n_pics = int(hb.pics.size());
    b->cur = gi;
    b->loaded = true;
    BatchArgs &a = b->args;
    a = BatchArgs{};
    a.bits = b->bits.p;
    a.pics = G.pics.p;
    a.subs = b->subs.p;
    a.rbsp = nullptr;  // (per parse set: heifgpu_batch_decode)
    a.rsubs = nullptr;
    a.parse_order = b->porder.p;
    a.n_slots = int(order.size());
    a.parse_group = parse_group;
    a.seqs = G.seqs.p;
    a.sf = G.sf.p;
    a.outs = G.outs.p;
    a.recon = b->recon.p;
    a.n_pics = b->n_pics;
    a.max_width = hb.max_w;
    a.max_wctb = hb.max_wctb;
    a.max_rows = hb.max_rows;
    a.max_log2ctb = hb.max_log2ctb;
    a.lane_rows = hb.lane_rows;
    a.parse_mode = mode;
    a.solo_waves = solo_waves;
    a.xprog = nullptr;  // (per parse set: heifgpu_batch_decode)
    a.xctx = cross_rows ? b->xctx.p : nullptr;
    a.intra_stream = intra_stream_for(mode, int(hb.pics.size()), hb.has_assembly, ctx->stream) ? 1 : 0;
    a.xntu = nullptr;
    a.stream_patience_us = ctx->stream.patience_us;
    // rows wrap round the lanes (waves) of a picture: the WPP context staging
    a.wpp_ring = mode == PARSE_SOLO ? (hb.max_wpp_rows > solo_waves ? 1 : 0) : hb.wpp_ring;
    a.has_assembly = hb.has_assembly ? 1 : 0;
    a.total_rows = int(hb.rows);
    a.bytes_per_sample = hb.bps;
    a.chroma_format = hb.chroma;
    G.out_host.assign(n, OutImage{});
    if (fresh) *inout = fresh.release();
    return HEIFGPU_OK;
}

int heifgpu_batch_prepare(heifgpu_ctx *ctx, const heifgpu_image *const *imgs, size_t n, heifgpu_batch **out) {
    if (!out) return fail(HEIFGPU_E_INVALID, "invalid argument");
    *out = nullptr;
    const int rc = heifgpu_batch_prepare_ex(ctx, imgs, n, nullptr, out);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(ctx->upload));  // v1 semantics: uploaded on return
    return HEIFGPU_OK;
}

int heifgpu_batch_decode(heifgpu_ctx *ctx, heifgpu_batch *b, const heifgpu_planes *out, void *stream) {
    if (!ctx || !b || !out) return fail(HEIFGPU_E_INVALID, "invalid argument");
    if (b->device != ctx->device) return fail(HEIFGPU_E_INVALID, "batch belongs to another device");
    if (!b->loaded) return fail(HEIFGPU_E_INVALID, "batch not loaded (its last prepare failed)");
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the null stream, as in HIP
    HIP_TRY(hipSetDevice(ctx->device));
    DescGen &G = b->gen[b->cur];
    bool changed = false;
    for (size_t i = 0; i < b->n_images; ++i) {
        OutImage o{};
        for (int c = 0; c < 3; ++c) {
            o.plane[c] = reinterpret_cast<uint64_t>(out[i].plane[c]);
            o.pitch[c] = out[i].pitch[c];
        }
        if (!out[i].plane[0] || (b->infos[i].chroma_format_idc && (!out[i].plane[1] || !out[i].plane[2])))
            return fail(HEIFGPU_E_INVALID, "missing output plane");
        o.width = int32_t(b->infos[i].width);
        o.height = int32_t(b->infos[i].height);
        if (std::memcmp(&o, &G.out_host[i], sizeof(o)) != 0) {
            G.out_host[i] = o;
            changed = true;
        }
    }
    if (changed)
        HIP_TRY(hipMemcpyAsync(G.outs.p, G.out_host.data(), b->n_images * sizeof(OutImage), hipMemcpyHostToDevice, s));
    // parse set of this call
    const int k = b->next_set;
    b->next_set = (k + 1) % b->n_sets;
    b->last_set = k;
    ParseSet &ps = b->set[k];
    BatchArgs a = b->args;
    a.tus = ps.tus.p;
    a.coefs = ps.coefs.p;
    a.row_counts = ps.row_counts.p;
    a.maps = ps.maps.p;
    a.sao = ps.sao.p;
    a.status = ps.status.p;
    a.resid = ps.resid.p;
    a.rbsp = ps.rbsp.p;
    a.rsubs = ps.rsubs.p;
    if (a.parse_mode == PARSE_SPREAD) {
        a.xprog = ps.xprog.p;
        a.xjob = ps.xprog.p + a.total_rows;
        a.xntu = a.intra_stream ? ps.xntu.p : nullptr;
    }
    // bring-up knob: HEIFGPU_STAGES=k launches only the first k stages (in order, on the caller's stream)
    static const int max_stages = [] {
        const char *e = std::getenv("HEIFGPU_STAGES");
        return e ? std::atoi(e) : 5;
    }();
    if (max_stages < 5) {
        a.intra_stream = 0;  // (stages one after another: k_transform, then the plain k_intra)
        a.xntu = nullptr;
        HIP_TRY(hipStreamSynchronize(ctx->upload));
        HIP_TRY(hipStreamSynchronize(ctx->parse));
        HIP_TRY(hipStreamSynchronize(ctx->xform));
        HIP_TRY(hipStreamSynchronize(ctx->recon));
        HIP_TRY(hipMemsetAsync(ps.status.p, 0, size_t(b->n_pics) * sizeof(uint32_t), s));
        HIP_TRY(hipMemsetAsync(ps.row_counts.p, 0, size_t(2) * uint32_t(b->args.total_rows) * sizeof(uint32_t), s));
        HIP_TRY(launch_rbsp(a, s));
        hipError_t (*fns[5])(const BatchArgs &, hipStream_t) = {launch_parse, launch_transform, launch_intra,
                                                                launch_deblock, launch_sao_out};
        for (int i = 0; i < max_stages; ++i) HIP_TRY(fns[i](a, s));
        HIP_TRY(launch_status_fold(ps.status.p, G.sticky.p, b->n_pics, s));
        return HEIFGPU_OK;
    }
#if defined(HG_ABLATE)
    // measurement builds only (make variant VDEFS=-DHG_ABLATE): HEIFGPU_ABLATE bit i
    // drops reconstruction stage i (1 transform, 2 intra, 4 deblock, 8 sao): wrong
    // pixels, the co-run cost of each stage on the parse
    static const int ablate = [] {
        const char *e = std::getenv("HEIFGPU_ABLATE");
        return e ? std::atoi(e) : 0;
    }();
#else
    constexpr int ablate = 0;
#endif
    hipStream_t p = ctx->parse, r = ctx->recon;
    if (b->n_pics == 0) {  // a tile subset without pictures: nothing to decode
        return HEIFGPU_OK;
    }
    const bool t = ctx->timing;
    hipEvent_t *ev = nullptr;
    if (t) {  // this call's timing slot; the call that used it last is folded first
        const int slot = ctx->timed_calls % kTimingSlots;
        if (ctx->timed_calls - ctx->folded >= kTimingSlots) {
            HIP_TRY(fold_timing(ctx, slot));
            ++ctx->folded;
        }
        ev = ctx->tev[slot];
        ++ctx->timed_calls;
    }
    // k_rbsp (prep stream, or the parse stream itself): the batch's uploads, and
    // this set's previous reconstruction must be done with it.  It also zeroes
    // this set's status words and row counts (rows a stopped substream never
    // reaches keep zero TBs) and, streaming, the progress words, TU counts and
    // done words k_intra_stream polls from its start (launch_parse leaves them
    // alone in that mode).  On the prep stream it runs beside the previous
    // decode's parse, so the parse stream goes from one k_parse to the next.
    hipStream_t q = ctx->prep ? ctx->prep : p;
    HIP_TRY(hipStreamWaitEvent(q, b->uploaded, 0));
    if (ps.pending) HIP_TRY(hipStreamWaitEvent(q, ps.recon_done, 0));
    if (t) HIP_TRY(hipEventRecord(ev[0], q));
    HIP_TRY(launch_rbsp(a, q));
    if (a.intra_stream) HIP_TRY(hipEventRecord(ps.progreset, q));
    if (t) HIP_TRY(hipEventRecord(ev[1], q));
    if (q != p) {
        HIP_TRY(hipEventRecord(ps.prepped, q));
        HIP_TRY(hipStreamWaitEvent(p, ps.prepped, 0));
    }
    if (t) HIP_TRY(hipEventRecord(ev[9], p));
    HIP_TRY(launch_parse(a, p));
    if (t) HIP_TRY(hipEventRecord(ev[2], p));
    HIP_TRY(hipEventRecord(ps.parsed, p));
    HIP_TRY(hipEventRecord(ctx->fork, s));
    if (a.intra_stream) {
        // streaming (small batches): no k_transform; the
        // reconstruction starts beside this decode's parse and trails it
        HIP_TRY(hipStreamWaitEvent(r, ps.progreset, 0));
        if (t) {
            HIP_TRY(hipEventRecord(ev[3], r));
            HIP_TRY(hipEventRecord(ev[4], r));
        }
    } else {
        // transform stream (the recon stream with two sets): this set's parse
        hipStream_t x = b->n_sets >= 3 ? ctx->xform : r;
        HIP_TRY(hipStreamWaitEvent(x, ps.parsed, 0));
        if (t) HIP_TRY(hipEventRecord(ev[3], x));
        if (!(ablate & 1)) HIP_TRY(launch_transform(a, x));
        if (t) HIP_TRY(hipEventRecord(ev[4], x));
        HIP_TRY(hipEventRecord(ps.transformed, x));
        // recon stream: this set's transform, and the caller's prior work before the planes are written
        HIP_TRY(hipStreamWaitEvent(r, ps.transformed, 0));
    }
    if (t) HIP_TRY(hipEventRecord(ev[5], r));
    if (!(ablate & 2)) HIP_TRY(launch_intra(a, r));
    if (a.intra_stream) {
        // the second launch, after the parse: the pictures the first one gave up
        // on (none, unless the parse did not run beside it); the rest exit at once
        HIP_TRY(hipStreamWaitEvent(r, ps.parsed, 0));
        BatchArgs a2 = a;
        a2.stream_redo = 1;
        HIP_TRY(launch_intra(a2, r));
    }
    if (t) HIP_TRY(hipEventRecord(ev[6], r));
    if (!(ablate & 4)) HIP_TRY(launch_deblock(a, r));
    if (t) HIP_TRY(hipEventRecord(ev[7], r));
    HIP_TRY(hipStreamWaitEvent(r, ctx->fork, 0));
    if (!(ablate & 8)) HIP_TRY(launch_sao_out(a, r));
    if (t) HIP_TRY(hipEventRecord(ev[8], r));
    HIP_TRY(launch_status_fold(ps.status.p, G.sticky.p, b->n_pics, r));
    HIP_TRY(hipEventRecord(ps.recon_done, r));
    ps.pending = true;
    HIP_TRY(hipEventRecord(G.done, r));
    G.pending = true;
    HIP_TRY(hipEventRecord(ctx->join, r));
    HIP_TRY(hipStreamWaitEvent(s, ctx->join, 0));
    return HEIFGPU_OK;
}

int heifgpu_batch_parse_geometry(const heifgpu_batch *b, uint32_t *mode, uint32_t *workgroups,
                                 uint32_t *pics_per_wave, uint32_t *waves_per_workgroup) {
    if (!b || !b->loaded) return fail(HEIFGPU_E_INVALID, "invalid batch");
    const BatchArgs &a = b->args;
    const bool solo = a.parse_mode == PARSE_SOLO, lanes = a.parse_mode == PARSE_LANES;
    const uint32_t ppw = lanes ? uint32_t(std::max(1, a.parse_group)) : 1u;
    if (mode) *mode = uint32_t(a.parse_mode);
    if (workgroups) *workgroups = (uint32_t(a.n_slots) + ppw - 1) / ppw;
    if (pics_per_wave) *pics_per_wave = ppw;
    if (waves_per_workgroup) *waves_per_workgroup = solo ? uint32_t(a.solo_waves) : 1u;
    return HEIFGPU_OK;
}

int heifgpu_batch_status(heifgpu_ctx *ctx, heifgpu_batch *b, uint32_t *status, void *stream) {
    if (!ctx || !b) return fail(HEIFGPU_E_INVALID, "invalid argument");
    if (b->device != ctx->device) return fail(HEIFGPU_E_INVALID, "batch belongs to another device");
    if (!b->loaded) return fail(HEIFGPU_E_INVALID, "batch not loaded (its last prepare failed)");
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the null stream, as in HIP
    HIP_TRY(hipSetDevice(ctx->device));
    // every decode since the last query (or the load) ORed its status words
    // into the sticky array (k_status_fold after k_sao_out); read and clear it
    DescGen &G = b->gen[b->cur];
    std::vector<uint32_t> st(size_t(b->n_pics));
    if (!st.empty()) {
        HIP_TRY(hipMemcpyAsync(st.data(), G.sticky.p, st.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemsetAsync(G.sticky.p, 0, st.size() * sizeof(uint32_t), s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<uint32_t> per(b->n_images, 0);
    for (size_t p = 0; p < st.size(); ++p) per[b->pic_image[p]] |= st[p];
    bool bad = false;
    for (size_t i = 0; i < b->n_images; ++i) {
        if (status) status[i] = per[i];
        bad |= per[i] != 0;
    }
    return bad ? fail(HEIFGPU_E_DECODE, "one or more pictures failed the kernel bitstream checks") : HEIFGPU_OK;
}

// The load before the current one: decodes of it still in flight when the
// batch was reloaded fold their status into that load's generation, which
// heifgpu_batch_status (current load only) does not read.  This reads and
// clears it, per image of that load (errors must reach the
// caller, /root/reference/src/heic/decoder.rs:109-112).
int heifgpu_batch_status_previous(heifgpu_ctx *ctx, heifgpu_batch *b, uint32_t *status, size_t cap, size_t *n_prev,
                                  void *stream) {
    if (!ctx || !b || !n_prev) return fail(HEIFGPU_E_INVALID, "invalid argument");
    if (b->device != ctx->device) return fail(HEIFGPU_E_INVALID, "batch belongs to another device");
    *n_prev = 0;
    if (!b->loaded) return fail(HEIFGPU_E_INVALID, "batch not loaded (its last prepare failed)");
    DescGen &P = b->gen[b->cur ^ 1];
    if (!P.loaded || P.pic_image.empty()) return HEIFGPU_OK;  // no previous load
    *n_prev = P.n_images;
    if (!status) return HEIFGPU_OK;  // the size query: nothing read or cleared
    if (cap < P.n_images) return fail(HEIFGPU_E_INVALID, "status array smaller than the previous load");
    hipStream_t s = static_cast<hipStream_t>(stream);
    HIP_TRY(hipSetDevice(ctx->device));
    if (P.pending) HIP_TRY(hipStreamWaitEvent(s, P.done, 0));  // its last decode
    std::vector<uint32_t> st(P.pic_image.size());
    HIP_TRY(hipMemcpyAsync(st.data(), P.sticky.p, st.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemsetAsync(P.sticky.p, 0, st.size() * sizeof(uint32_t), s));
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<uint32_t> per(P.n_images, 0);
    for (size_t p = 0; p < st.size(); ++p) per[P.pic_image[p]] |= st[p];
    bool bad = false;
    for (size_t i = 0; i < P.n_images; ++i) {
        status[i] = per[i];
        bad |= per[i] != 0;
    }
    return bad ? fail(HEIFGPU_E_DECODE, "one or more pictures of the previous load failed the kernel bitstream checks")
               : HEIFGPU_OK;
}

int heifgpu_abi_version(void) { return HEIFGPU_ABI_VERSION; }

void heifgpu_batch_free(heifgpu_batch *b) {
    if (!b) return;
    (void)hipSetDevice(b->device);
    (void)hipDeviceSynchronize();  // in-flight parses / reconstructions of this batch
    delete b;
}

int heifgpu_decode_batch(heifgpu_ctx *ctx, const heifgpu_image *const *imgs, size_t n, const heifgpu_planes *out,
                         void *stream, uint32_t *status) {
    heifgpu_batch *b = nullptr;
    int rc = heifgpu_batch_prepare(ctx, imgs, n, &b);
    if (rc) return rc;
    rc = heifgpu_batch_decode(ctx, b, out, stream);
    if (!rc) rc = heifgpu_batch_status(ctx, b, status, stream);
    heifgpu_batch_free(b);
    return rc;
}

// ---------------------------------------------------------------- test hooks
size_t heifgpu_remove_emulation_prevention(const uint8_t *in, size_t n, uint8_t *out) {
    std::vector<uint8_t> v = RbspReader::remove_emulation_prevention(in, n);
    if (!v.empty()) std::memcpy(out, v.data(), v.size());
    return v.size();
}

int heifgpu_read_ue(const uint8_t *buf, size_t n, uint32_t *val) {
    try {
        RbspReader r(buf, n);
        *val = r.read_ue();
        return HEIFGPU_OK;
    } catch (const std::exception &e) {
        return fail(HEIFGPU_E_PARSE, e.what());
    }
}

int heifgpu_read_se(const uint8_t *buf, size_t n, int32_t *val) {
    try {
        RbspReader r(buf, n);
        *val = r.read_se();
        return HEIFGPU_OK;
    } catch (const std::exception &e) {
        return fail(HEIFGPU_E_PARSE, e.what());
    }
}

namespace {
struct VecBins {
    const uint8_t *b;
    int n, i = 0;
    bool under = false;
    int operator()() {
        if (i >= n) {
            under = true;
            return 0;
        }
        return b[i++] ? 1 : 0;
    }
};
}  // namespace

int heifgpu_bins_truncated_rice(const uint8_t *bins, int n, int c_max, int c_rice, int *used) {
    VecBins v{bins, n};
    uint32_t r = bin_truncated_rice(v, uint32_t(c_max), c_rice);
    if (used) *used = v.i;
    return v.under ? -1 : int(r);
}

int heifgpu_bins_chroma_pred_mode(const uint8_t *bins, int n, int *used) {
    VecBins v{bins, n};
    uint32_t r = bin_intra_chroma_pred_mode(v, v);
    if (used) *used = v.i;
    return v.under ? -1 : int(r);
}

int heifgpu_bins_coeff_abs_level_remaining(const uint8_t *bins, int n, int c_rice, int *used) {
    VecBins v{bins, n};
    uint32_t r = bin_coeff_abs_level_remaining(v, c_rice);
    if (used) *used = v.i;
    return (v.under || r == 0xffffffffu) ? -1 : int(r);
}

int heifgpu_bins_exp_golomb(const uint8_t *bins, int n, int k, int *used) {
    VecBins v{bins, n};
    uint32_t r = bin_exp_golomb(v, k);
    if (used) *used = v.i;
    return (v.under || r == 0xffffffffu) ? -1 : int(r);
}

int heifgpu_image_tile_params(const heifgpu_image *img, uint32_t tile, heifgpu_tile_params *o) {
    if (!img || !o) return fail(HEIFGPU_E_INVALID, "invalid argument");
    const ParsedImage &pi = img->img;
    if (tile >= pi.tiles.size()) return fail(HEIFGPU_E_INVALID, "tile index out of range");
    const TileJob &t = pi.tiles[tile];
    const SequenceParameterSet &sps = pi.params[t.param].sps;
    const PictureParameterSet &pps = pi.params[t.param].pps;
    const SliceSegmentHeader &sh = t.segs[0].sh;  // the picture's first slice segment
    std::memset(o, 0, sizeof(*o));
    o->nal_unit_type = t.segs[0].nal.nal_unit_type();
    o->slice_type = sh.slice_type;
    o->first_slice_segment_in_pic = sh.first_slice_segment_in_pic_flag;
    o->general_profile_idc = sps.general_profile_idc;
    o->general_level_idc = sps.general_level_idc;
    o->pic_width = sps.pic_width_in_luma_samples;
    o->pic_height = sps.pic_height_in_luma_samples;
    o->chroma_format_idc = sps.chroma_format_idc;
    o->bit_depth_luma = 8 + sps.bit_depth_luma_minus8;
    o->bit_depth_chroma = 8 + sps.bit_depth_chroma_minus8;
    o->log2_max_poc_lsb = sps.log2_max_pic_order_cnt_lsb;
    o->log2_min_cb = sps.log2_min_luma_coding_block_size;
    o->log2_ctb = sps.log2_ctb_size;
    o->log2_min_tb = sps.log2_min_tb_size;
    o->log2_max_tb = sps.log2_max_tb_size;
    o->max_th_depth_inter = sps.max_transform_hierarchy_depth_inter;
    o->max_th_depth_intra = sps.max_transform_hierarchy_depth_intra;
    o->scaling_list_enabled = sps.scaling_list_enabled_flag;
    o->amp = sps.amp_enabled_flag;
    o->sao = sps.sample_adaptive_offset_enabled_flag;
    o->pcm = sps.pcm_enabled_flag;
    o->num_short_term_ref_pic_sets = sps.num_short_term_ref_pic_sets;
    o->long_term_refs = sps.long_term_ref_pics_present_flag;
    o->temporal_mvp = sps.sps_temporal_mvp_enabled_flag;
    o->strong_intra_smoothing = sps.strong_intra_smoothing_enabled_flag;
    o->video_full_range = sps.video_full_range_flag;
    o->colour_primaries = sps.colour_primaries;
    o->transfer_characteristics = sps.transfer_characteristics;
    o->matrix_coeffs = sps.matrix_coeffs;
    o->init_qp = 26 + pps.init_qp_minus26;
    o->sign_data_hiding = pps.sign_data_hiding_enabled_flag;
    o->cabac_init_present = pps.cabac_init_present_flag;
    o->constrained_intra_pred = pps.constrained_intra_pred_flag;
    o->transform_skip = pps.transform_skip_enabled_flag;
    o->cu_qp_delta_enabled = pps.cu_qp_delta_enabled_flag;
    o->diff_cu_qp_delta_depth = pps.diff_cu_qp_delta_depth;
    o->cb_qp_offset = pps.pps_cb_qp_offset;
    o->cr_qp_offset = pps.pps_cr_qp_offset;
    o->slice_chroma_qp_offsets_present = pps.pps_slice_chroma_qp_offsets_present_flag;
    o->transquant_bypass = pps.transquant_bypass_enabled_flag;
    o->tiles_enabled = pps.tiles_enabled_flag;
    o->entropy_coding_sync = pps.entropy_coding_sync_enabled_flag;
    o->loop_filter_across_slices = pps.pps_loop_filter_across_slices_enabled_flag;
    o->deblocking_control_present = pps.deblocking_filter_control_present_flag;
    o->deblocking_override_enabled = pps.deblocking_filter_override_enabled_flag;
    o->deblocking_disabled = sh.slice_deblocking_filter_disabled_flag;
    o->beta_offset_div2 = sh.slice_beta_offset_div2;
    o->tc_offset_div2 = sh.slice_tc_offset_div2;
    o->log2_parallel_merge_level = pps.log2_parallel_merge_level;
    o->slice_sao_luma = sh.slice_sao_luma_flag;
    o->slice_sao_chroma = sh.slice_sao_chroma_flag;
    o->slice_qp_y = 26 + pps.init_qp_minus26 + sh.slice_qp_delta;
    o->num_entry_point_offsets = sh.num_entry_point_offsets;
    o->slice_data_raw_offset = int32_t(sh.slice_data_raw_offset);
    o->payload_bytes = int32_t(t.segs[0].payload_len);
    for (size_t i = 0; i < sh.entry_point_offset.size() && i < 64; ++i) o->entry_point_offset[i] = sh.entry_point_offset[i];
    return HEIFGPU_OK;
}

}  // extern "C"
