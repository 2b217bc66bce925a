// heic_image.hpp — host half of HeicDecoder::decode (src/heic/decoder.rs:12-112).
#pragma once
#include <cstdint>
#include <vector>

#include "heif_reader.hpp"
#include "hevc_ps.hpp"

namespace hg {

struct ParamSet {
    std::vector<uint8_t> key;  // raw SPS ++ PPS NAL bytes (dedupe key)
    VideoParameterSet vps;
    SequenceParameterSet sps;
    PictureParameterSet pps;
    std::vector<int> col_bd, row_bd;  // HEVC tile boundaries in CTBs (one tile without tiles)
};

struct SliceSeg {
    // raw NAL payload after the 2-byte header (EP bytes kept): a view into ParsedImage::coded
    const uint8_t *payload = nullptr;
    size_t payload_len = 0;
    NalUnitHeader nal;
    SliceSegmentHeader sh;
};

struct TileJob {
    std::vector<SliceSeg> segs;  // the coded picture's slice segments in decoding order (one or more)
    int param = 0;
};

struct ParsedImage {
    // move-only: the tiles' payload views point into `coded`, whose buffer a move keeps
    ParsedImage() = default;
    ParsedImage(const ParsedImage &) = delete;
    ParsedImage &operator=(const ParsedImage &) = delete;
    ParsedImage(ParsedImage &&) = default;
    ParsedImage &operator=(ParsedImage &&) = default;
    std::vector<uint8_t> coded;  // the coded items' bytes, one copy (TileJob payloads point into it)
    std::vector<ParamSet> params;
    std::vector<TileJob> tiles;  // grid order (row-major)
    uint32_t primary_item_id = 0, ispe_width = 0, ispe_height = 0, rotation = 0, num_thumbnails = 0;
    uint32_t item_id = 0;      // the decoded image item (the primary unless asked otherwise)
    uint32_t aux_item_id = 0;  // first auxiliary image of the primary ('auxl'), 0 if none
    bool nclx = false;         // the item has an nclx colr (overrides the VUI colour description)
    uint32_t nclx_matrix = 0, nclx_full_range = 0;
    uint32_t rows = 1, cols = 1, out_width = 0, out_height = 0;
    uint32_t tile_width = 0, tile_height = 0, coded_bytes = 0;
};

// Throws HeifError (parse) or UnsupportedError (valid stream, tool outside this path).
// item_id 0 = the primary item (heic/decoder.rs:12-112); otherwise any coded
// image item, e.g. an auxiliary image found through ParsedImage::aux_item_id
ParsedImage parse_heic(const uint8_t *data, size_t len, uint32_t item_id = 0);

}  // namespace hg
