// rbsp.hip — k_rbsp: emulation-prevention removal for every picture of a
// batch (pipeline stage 0, ahead of k_parse_lanes).
//
// H.265 7.3.1.1 / 7.4.2: inside a NAL unit every 0x000003 is an
// emulation_prevention_three_byte.  The reference strips 00 00 03 → 00 00
// when the byte after the 03 is <= 3 or the 03 ends the NAL unit
// (src/hevc/rbsp_reader.rs:11-39, called once per NAL at
// src/heic/decoder.rs:139,160).  Position i of a payload is such a byte iff
// raw[i-2] == 0, raw[i-1] == 0, raw[i] == 3 and (i + 1 == len or
// raw[i+1] <= 3): neither zero can itself be a removed byte (those are 3s),
// so the sequential rule is a per-position predicate and the removal is a
// stream compaction.  The two bytes before the payload are the NAL header,
// whose second byte (nuh_temporal_id_plus1 >= 1) is never zero.
//
// The entry points of the slice header count raw bytes (7.4.7.1); each is
// remapped to its RBSP offset (raw offset minus the removed bytes before it)
// in `rsubs`, and the last entry of a picture becomes its RBSP length.
//
// One wave per picture, 16 bytes per lane per step (1 KiB per wave step,
// 16-byte coalesced loads and stores).  Emulation prevention is rare (2 bytes
// in the 1.7 MB of halfmoonbay), so a chunk without a 0x03 byte and no
// removal before it in its picture is copied with one 16-byte store; the
// others are compacted byte by byte.  Roofline: HBM, 2 bytes moved per
// payload byte.
#include "kernels.hpp"

namespace hg {

// This decode's per-picture words that start at zero, cleared here instead of
// by memsets on the parse stream (each of those waited ~5 ms for a slot behind
// the previous decode's k_transform, on the parse's critical path): the
// status word, the picture's row counts, its spread-parse progress words and,
// for k_intra_stream, its TU counts and done word.
__device__ inline void zero_outputs(const BatchArgs &a, int pic, int lane, int nl) {
    const PicDesc &pd = a.pics[pic];
    if (lane == 0) a.status[pic] = 0;
    if (pic == a.pic0 && lane == 0 && a.xjob) *a.xjob = 0;  // spread / rows parse: the job counter
    if (pd.flags & PD_ASSEMBLY) return;  // no rows of its own
    const SeqParams &sp = a.seqs[pd.seq];
    const int hctb = (sp.height + (1 << sp.log2_ctb) - 1) >> sp.log2_ctb;
    for (int i = lane; i < 2 * hctb; i += nl) a.row_counts[2 * (size_t)pd.row_off + i] = 0;
    if (a.xprog)  // spread parse: one progress word per row
        for (int i = lane; i < hctb; i += nl) a.xprog[pd.row_off + i] = 0;
    if (a.intra_stream && a.xntu) {
        for (int i = lane; i < hctb; i += nl) a.xntu[pd.row_off + i] = 0;
        if (lane == 0) a.xntu[a.total_rows + pic] = 0;
    }
}

#if defined(HG_HOST_EMU)
// host restatement of the kernel's result (tests only)
void emu_rbsp(const BatchArgs &a) {
    for (int p = a.pic0; p < a.pic0 + a.n_pics; ++p) {
        const PicDesc &pd = a.pics[p];
        const uint8_t *raw = a.bits + pd.bits_off;
        uint8_t *out = a.rbsp + pd.bits_off;
        const uint32_t len = pd.bits_len;
        std::vector<uint32_t> removed_before(len + 1, 0);
        uint32_t o = 0, r = 0;
        for (uint32_t i = 0; i < len; ++i) {
            removed_before[i] = r;
            const bool ep = raw[i] == 3 && i >= 2 && raw[i - 1] == 0 && raw[i - 2] == 0 && (i + 1 == len || raw[i + 1] <= 3);
            if (ep) ++r;
            else out[o++] = raw[i];
        }
        removed_before[len] = r;
        for (uint32_t s = 0; s <= pd.n_sub + (pd.flags >> PD_NMID_SHIFT); ++s) {
            const uint32_t e = a.subs[pd.sub_first + s] & SUB_OFFSET, fl = a.subs[pd.sub_first + s] & ~SUB_OFFSET;
            a.rsubs[pd.sub_first + s] = (e < len ? e - removed_before[e] : len - r) | fl;
        }
        zero_outputs(a, p, 0, 1);
    }
}
#else
namespace {

__device__ __forceinline__ uint32_t byte_of(const uint4 &q, int j) {
    const uint32_t w = j < 4 ? q.x : j < 8 ? q.y : j < 12 ? q.z : q.w;
    return (w >> ((j & 3) * 8)) & 0xffu;
}

// any byte of w equal to 3
__device__ __forceinline__ bool has3(uint32_t w) {
    const uint32_t x = w ^ 0x03030303u;
    return ((x - 0x01010101u) & ~x & 0x80808080u) != 0;
}

__device__ __forceinline__ int wave_excl_sum(int v, int lane, int &total) {
    int s = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(s, d, 64);
        if (lane >= d) s += t;
    }
    total = __shfl(s, 63, 64);
    return s - v;
}

}  // namespace

__global__ void __launch_bounds__(64) k_rbsp(BatchArgs a) {
#if !defined(HG_HOST_EMU) && HG_PARSE_SETPRIO > 0
    // on the parse stream right before k_parse, beside the previous decodes'
    // reconstruction: at the parse's issue priority, so the gap between two
    // parses is its own 0.25 ms and not 2 ms of issue lost to k_intra
    __builtin_amdgcn_s_setprio(HG_PARSE_SETPRIO);
#endif
    const int pic = a.pic0 + (int)blockIdx.x;
    const int lane = (int)threadIdx.x;
    const PicDesc &pd = a.pics[pic];
    const uint8_t *raw = a.bits + pd.bits_off;
    uint8_t *out = a.rbsp + pd.bits_off;
    const uint32_t len = pd.bits_len;
    const uint32_t nent = pd.n_sub + 1 + (pd.flags >> PD_NMID_SHIFT);  // (segment starts inside rows after the end entry)
    const uint32_t *subs = a.subs + pd.sub_first;
    uint32_t *rsubs = a.rsubs + pd.sub_first;
    uint32_t run = 0;  // bytes removed before this step
    for (uint32_t c0 = 0; c0 < len; c0 += 1024) {
        const uint32_t i0 = c0 + (uint32_t)lane * 16u;
        uint4 q = make_uint4(0, 0, 0, 0);
        uint32_t mask = 0;  // bit j: raw[i0 + j] is removed
        if (i0 < len) {
            // payloads are 64-byte aligned and the arena is padded, so the 16-byte
            // chunk and the dword after it are in bounds
            q = *reinterpret_cast<const uint4 *>(raw + i0);
            if (has3(q.x) || has3(q.y) || has3(q.z) || has3(q.w)) {
                const uint32_t pw = i0 ? *reinterpret_cast<const uint32_t *>(raw + i0 - 4) : 0xffffffffu;
                const uint32_t nw = *reinterpret_cast<const uint32_t *>(raw + i0 + 16);
                uint32_t p2 = (pw >> 16) & 0xffu, p1 = pw >> 24;
                for (int j = 0; j < 16; ++j) {
                    const uint32_t b = byte_of(q, j);
                    const uint32_t nb = j < 15 ? byte_of(q, j + 1) : (nw & 0xffu);
                    const uint32_t pos = i0 + (uint32_t)j;
                    if (b == 3 && p1 == 0 && p2 == 0 && pos < len && (pos + 1 == len || nb <= 3)) mask |= 1u << j;
                    p2 = p1;
                    p1 = b;
                }
            }
        }
        int total;
        const uint32_t ex = (uint32_t)wave_excl_sum(__popc(mask), lane, total);
        if (i0 < len) {
            const uint32_t sh = run + ex;
            if (sh == 0 && mask == 0) {
                *reinterpret_cast<uint4 *>(out + i0) = q;
            } else {
                for (int j = 0; j < 16; ++j) {
                    const uint32_t pos = i0 + (uint32_t)j;
                    if (pos < len && !((mask >> j) & 1u))
                        out[pos - sh - (uint32_t)__popc(mask & ((1u << j) - 1u))] = (uint8_t)byte_of(q, j);
                }
            }
        }
        // entry points inside this step: lane t of the chunk holding e knows the removals before e
        for (uint32_t g = 0; g < nent; g += 64) {
            const uint32_t idx = g + (uint32_t)lane;
            const uint32_t raw_e = idx < nent ? subs[idx] : 0xffffffffu;
            const uint32_t e = raw_e & SUB_OFFSET;  // the flags ride along (SP_ROW_SEGMENTS)
            const bool here = e >= c0 && e < c0 + 1024u && e < len;
            const int t = here ? (int)((e - c0) >> 4) : 0;
            const uint32_t ext = (uint32_t)__shfl((int)ex, t, 64);
            const uint32_t mt = (uint32_t)__shfl((int)mask, t, 64);
            if (here)
                rsubs[idx] = (e - (run + ext + (uint32_t)__popc(mt & ((1u << ((e - c0) & 15u)) - 1u)))) |
                             (raw_e & ~SUB_OFFSET);
        }
        run += (uint32_t)total;
    }
    // the RBSP length, and entries at or past the payload end (corrupt headers)
    for (uint32_t idx = (uint32_t)lane; idx < nent; idx += 64)
        if ((subs[idx] & SUB_OFFSET) >= len) rsubs[idx] = (len - run) | (subs[idx] & ~SUB_OFFSET);
    zero_outputs(a, pic, lane, 64);
}

hipError_t launch_rbsp(const BatchArgs &a, hipStream_t s) {
    if (a.n_pics <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rbsp, dim3(a.n_pics), dim3(64), 0, s, a);
    return hipGetLastError();
}
#endif

}  // namespace hg
