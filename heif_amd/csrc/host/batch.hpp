// batch.hpp — flattens parsed images into the device descriptor arrays of
// common/desc.hpp (shared by the HIP path and the host-emulation test build).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../common/desc.hpp"
#include "heic_image.hpp"

namespace hg {

struct HostBatch {
    std::vector<uint8_t> bits;  // every picture's payload, 64-byte aligned (+128 B tail), unless deferred
    // deferred bits (build_batch(..., defer_bits = true)): where each payload
    // goes in the bits arena, copied by the caller straight into its staging
    struct Piece {
        const uint8_t *src;
        size_t len, dst;
    };
    std::vector<Piece> pieces;
    size_t bits_size = 0;  // bytes of the bits arena
    std::vector<PicDesc> pics;
    std::vector<uint32_t> subs;
    std::vector<SeqParams> seqs;
    std::vector<uint8_t> sf;
    std::vector<uint32_t> pic_image;  // picture → image index
    uint64_t recon_bytes = 0, resid_elems = 0, map_bytes = 0, sao_n = 0, tu_n = 0, coef_n = 0;
    uint32_t rows = 0;
    int max_w = 0, max_wctb = 0, max_rows = 0, max_log2ctb = 4, bps = 0, chroma = -1;
    int lane_rows = 1, wpp_ring = 0;  // k_parse_lanes geometry (BatchArgs::lane_rows / wpp_ring)
    int max_wpp_rows = 0;             // CTB rows of the tallest WPP picture (k_parse_solo's context staging)
    bool has_assembly = false;        // some picture is a PD_ASSEMBLY (BatchArgs::has_assembly)
};

// Throws HeifError / UnsupportedError.  Only grid tiles k (row-major) with
// k % tile_stride == tile_offset become pictures (the single-image tile split
// across GPUs); the default takes every tile.
HostBatch build_batch(const ParsedImage *const *imgs, size_t n, uint32_t tile_stride = 1, uint32_t tile_offset = 0,
                      bool defer_bits = false);

}  // namespace hg
