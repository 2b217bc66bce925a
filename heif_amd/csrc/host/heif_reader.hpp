// heif_reader.hpp — ISOBMFF / HEIF demux (host).
// Mirrors src/heif/reader.rs (HeifReader::read :59-83, get_item_data :33-57)
// and src/heif/grammar.rs (Heif::primary_item_id / item_info_by_item_id /
// hevc_configuration_record :25-50), fixing what the reference leaves open:
// idat (construction_method 1, reader.rs:42), multi-extent items (:47),
// index-preserving ipco (:460-463), 16-bit ipma indices (:496-500), infe v0/v1
// are skipped rather than panicking (:303), and the ImageGrid descriptor.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "rbsp.hpp"

namespace hg {

constexpr uint32_t fourcc(char a, char b, char c, char d) {
    return (uint32_t(uint8_t(a)) << 24) | (uint32_t(uint8_t(b)) << 16) | (uint32_t(uint8_t(c)) << 8) | uint32_t(uint8_t(d));
}

struct ItemExtent {
    uint64_t offset, length;
};

struct ItemInfo {
    uint32_t id = 0;
    uint32_t type = 0;         // 'hvc1', 'grid', 'Exif', ...
    bool hidden = false;
    int construction_method = 0;
    std::vector<ItemExtent> extents;
    std::vector<uint32_t> properties;  // 1-based ipco indices (essential bit stripped)
};

struct Property {
    uint32_t type = 0;
    size_t offset = 0, length = 0;  // payload within the file
};

struct ItemReference {
    uint32_t type = 0;  // 'dimg', 'thmb', 'cdsc', 'auxl', ...
    uint32_t from = 0;
    std::vector<uint32_t> to;
};

struct ImageGrid {
    uint32_t rows = 0, cols = 0, output_width = 0, output_height = 0;
};

struct Heif {
    const uint8_t *data = nullptr;
    size_t len = 0;
    uint32_t major_brand = 0;
    uint32_t primary_item_id = 0;
    std::vector<ItemInfo> items;
    std::vector<Property> properties;
    std::vector<ItemReference> references;
    size_t idat_offset = 0, idat_length = 0;

    const ItemInfo *item_info_by_item_id(uint32_t id) const;
    const Property *item_property(const ItemInfo &it, uint32_t type) const;
    std::vector<uint8_t> item_data(const ItemInfo &it) const;  // concatenated extents
    // the item's byte count (extents bounds-checked), appending its bytes to *out when out is set
    size_t item_data(const ItemInfo &it, std::vector<uint8_t> *out) const;
    std::vector<uint32_t> references_from(uint32_t type, uint32_t from) const;
    ImageGrid grid(const ItemInfo &it) const;
    // tests/libheif_comparison.rs:240-250: 'thmb' references pointing at the primary
    uint32_t num_thumbnails() const;
};

class HeifReader {
  public:
    HeifReader(const uint8_t *data, size_t len) : d_(data), n_(len) {}
    Heif read();  // throws HeifError

  private:
    const uint8_t *d_;
    size_t n_;
};

}  // namespace hg
