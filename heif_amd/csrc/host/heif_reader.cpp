// heif_reader.cpp — see heif_reader.hpp.
#include "heif_reader.hpp"

#include <cstring>

namespace hg {
namespace {

struct Cursor {
    const uint8_t *d;
    size_t end, pos;
    uint64_t be(int n) {
        if (n < 0 || n > 8 || pos + size_t(n) > end) throw HeifError("box payload overrun");
        uint64_t v = 0;
        for (int i = 0; i < n; ++i) v = (v << 8) | d[pos + i];
        pos += size_t(n);
        return v;
    }
    uint32_t u8() { return uint32_t(be(1)); }
    uint32_t u16() { return uint32_t(be(2)); }
    uint32_t u32() { return uint32_t(be(4)); }
};

struct BoxHeader {
    uint32_t type;
    size_t start, payload, end;  // box start, payload start, box end
};

// box header at pos within [.., limit)  (reader.rs:806-819)
BoxHeader box_at(const uint8_t *d, size_t limit, size_t pos) {
    if (pos + 8 > limit) throw HeifError("truncated box header");
    uint64_t size = (uint64_t(d[pos]) << 24) | (uint64_t(d[pos + 1]) << 16) | (uint64_t(d[pos + 2]) << 8) | d[pos + 3];
    uint32_t type = (uint32_t(d[pos + 4]) << 24) | (uint32_t(d[pos + 5]) << 16) | (uint32_t(d[pos + 6]) << 8) | d[pos + 7];
    size_t hdr = 8;
    if (size == 1) {
        if (pos + 16 > limit) throw HeifError("truncated largesize");
        size = 0;
        for (int i = 0; i < 8; ++i) size = (size << 8) | d[pos + 8 + i];
        hdr = 16;
    } else if (size == 0) {
        size = limit - pos;
    }
    if (size < hdr || pos + size > limit) throw HeifError("box size out of range");
    return {type, pos, pos + hdr, size_t(pos + size)};
}

template <class F>
void for_each_child(const uint8_t *d, size_t begin, size_t end, F &&f) {
    size_t p = begin;
    while (p < end) {
        BoxHeader b = box_at(d, end, p);
        f(b);
        p = b.end;
    }
}

ItemInfo &item_slot(Heif &h, uint32_t id) {
    for (auto &it : h.items)
        if (it.id == id) return it;
    h.items.emplace_back();
    h.items.back().id = id;
    return h.items.back();
}

}  // namespace

const ItemInfo *Heif::item_info_by_item_id(uint32_t id) const {
    for (auto &it : items)
        if (it.id == id) return &it;
    return nullptr;
}

const Property *Heif::item_property(const ItemInfo &it, uint32_t type) const {
    for (uint32_t idx : it.properties) {
        if (idx == 0 || idx > properties.size()) continue;
        if (properties[idx - 1].type == type) return &properties[idx - 1];
    }
    return nullptr;
}

size_t Heif::item_data(const ItemInfo &it, std::vector<uint8_t> *out) const {
    size_t total = 0;
    for (auto &e : it.extents) {
        const uint8_t *base;
        size_t limit;
        if (it.construction_method == 0) {
            base = data;
            limit = len;
        } else if (it.construction_method == 1) {
            base = data + idat_offset;
            limit = idat_length;
        } else {
            throw HeifError("unsupported construction_method " + std::to_string(it.construction_method));
        }
        // without overflow: offset and length are up to 64-bit file fields
        if (e.offset > limit || e.length > limit - e.offset) throw HeifError("item extent out of bounds");
        if (out) out->insert(out->end(), base + e.offset, base + e.offset + e.length);
        total += size_t(e.length);
    }
    return total;
}

std::vector<uint8_t> Heif::item_data(const ItemInfo &it) const {
    std::vector<uint8_t> out;
    item_data(it, &out);
    return out;
}

std::vector<uint32_t> Heif::references_from(uint32_t type, uint32_t from) const {
    for (auto &r : references)
        if (r.type == type && r.from == from) return r.to;
    return {};
}

ImageGrid Heif::grid(const ItemInfo &it) const {
    std::vector<uint8_t> g = item_data(it);
    if (g.size() < 8) throw HeifError("grid descriptor too short");
    int fl = (g[1] & 1) ? 4 : 2;
    if (g.size() < size_t(4 + 2 * fl)) throw HeifError("grid descriptor too short");
    ImageGrid r;
    r.rows = g[2] + 1u;
    r.cols = g[3] + 1u;
    for (int i = 0; i < fl; ++i) {
        r.output_width = (r.output_width << 8) | g[4 + i];
        r.output_height = (r.output_height << 8) | g[4 + fl + i];
    }
    return r;
}

uint32_t Heif::num_thumbnails() const {
    uint32_t n = 0;
    for (auto &r : references)
        if (r.type == fourcc('t', 'h', 'm', 'b'))
            for (uint32_t t : r.to)
                if (t == primary_item_id) ++n;
    return n;
}

Heif HeifReader::read() {
    Heif h;
    h.data = d_;
    h.len = n_;
    bool have_ftyp = false, have_meta = false;
    size_t iloc_b = 0, iloc_e = 0, ipma_b = 0, ipma_e = 0;
    for_each_child(d_, 0, n_, [&](const BoxHeader &top) {
        if (top.type == fourcc('f', 't', 'y', 'p')) {
            have_ftyp = true;
            Cursor c{d_, top.end, top.payload};
            h.major_brand = c.u32();
        } else if (top.type == fourcc('m', 'e', 't', 'a')) {
            have_meta = true;
            if (top.payload + 4 > top.end || d_[top.payload] != 0) throw HeifError("meta box version != 0");
            for_each_child(d_, top.payload + 4, top.end, [&](const BoxHeader &b) {
                Cursor c{d_, b.end, b.payload};
                switch (b.type) {
                case fourcc('p', 'i', 't', 'm'): {
                    int v = int(c.u8());
                    c.be(3);
                    h.primary_item_id = v == 0 ? c.u16() : c.u32();
                    break;
                }
                case fourcc('i', 'i', 'n', 'f'): {
                    int v = int(c.u8());
                    c.be(3);
                    c.be(v == 0 ? 2 : 4);
                    for_each_child(d_, c.pos, b.end, [&](const BoxHeader &e) {
                        if (e.type != fourcc('i', 'n', 'f', 'e')) return;
                        Cursor ec{d_, e.end, e.payload};
                        int ev = int(ec.u8());
                        uint32_t flags = uint32_t(ec.be(3));
                        if (ev < 2) return;  // infe v0/v1 carry no item_type (reader.rs:303 panics)
                        uint32_t id = ev == 2 ? ec.u16() : ec.u32();
                        ec.u16();  // item_protection_index
                        ItemInfo &it = item_slot(h, id);
                        it.type = ec.u32();
                        it.hidden = (flags & 1) != 0;
                    });
                    break;
                }
                case fourcc('i', 'r', 'e', 'f'): {
                    int v = int(c.u8());
                    c.be(3);
                    for_each_child(d_, c.pos, b.end, [&](const BoxHeader &r) {
                        Cursor rc{d_, r.end, r.payload};
                        ItemReference ref;
                        ref.type = r.type;
                        ref.from = v == 0 ? rc.u16() : rc.u32();
                        uint32_t cnt = rc.u16();
                        for (uint32_t k = 0; k < cnt; ++k) ref.to.push_back(v == 0 ? rc.u16() : rc.u32());
                        h.references.push_back(std::move(ref));
                    });
                    break;
                }
                case fourcc('i', 'p', 'r', 'p'):
                    for_each_child(d_, b.payload, b.end, [&](const BoxHeader &p) {
                        if (p.type == fourcc('i', 'p', 'c', 'o')) {
                            // every child keeps its slot so 1-based ipma indices stay valid
                            for_each_child(d_, p.payload, p.end, [&](const BoxHeader &prop) {
                                h.properties.push_back({prop.type, prop.payload, prop.end - prop.payload});
                            });
                        } else if (p.type == fourcc('i', 'p', 'm', 'a')) {
                            ipma_b = p.payload;
                            ipma_e = p.end;
                        }
                    });
                    break;
                case fourcc('i', 'l', 'o', 'c'):
                    iloc_b = b.payload;
                    iloc_e = b.end;
                    break;
                case fourcc('i', 'd', 'a', 't'):
                    h.idat_offset = b.payload;
                    h.idat_length = b.end - b.payload;
                    break;
                default:
                    break;  // hdlr, dinf, ...
                }
            });
        }
    });
    if (!have_ftyp) throw HeifError("missing ftyp box");
    if (!have_meta) throw HeifError("missing required meta box");
    if (iloc_e) {  // reader.rs:632-704
        Cursor c{d_, iloc_e, iloc_b};
        int v = int(c.u8());
        c.be(3);
        uint32_t t = c.u8();
        int off_sz = int(t >> 4), len_sz = int(t & 15);
        t = c.u8();
        int base_sz = int(t >> 4), idx_sz = (v == 1 || v == 2) ? int(t & 15) : 0;
        uint32_t count = v < 2 ? c.u16() : c.u32();
        for (uint32_t i = 0; i < count; ++i) {
            uint32_t id = v < 2 ? c.u16() : c.u32();
            ItemInfo &it = item_slot(h, id);
            it.construction_method = (v == 1 || v == 2) ? int(c.u16() & 15) : 0;
            c.u16();  // data_reference_index
            uint64_t base = c.be(base_sz);
            uint32_t ne = c.u16();
            it.extents.clear();
            for (uint32_t k = 0; k < ne; ++k) {
                if (idx_sz) c.be(idx_sz);
                uint64_t o = c.be(off_sz), l = c.be(len_sz);
                if (o > UINT64_MAX - base) throw HeifError("iloc extent offset overflows");
                it.extents.push_back({base + o, l});
            }
        }
    }
    if (ipma_e) {  // reader.rs:475-513 (full 15-bit index when flags & 1)
        Cursor c{d_, ipma_e, ipma_b};
        int v = int(c.u8());
        uint32_t flags = uint32_t(c.be(3));
        uint32_t count = c.u32();
        for (uint32_t i = 0; i < count; ++i) {
            uint32_t id = v < 1 ? c.u16() : c.u32();
            uint32_t na = c.u8();
            ItemInfo &it = item_slot(h, id);
            for (uint32_t k = 0; k < na; ++k) it.properties.push_back((flags & 1) ? (c.u16() & 0x7fffu) : (c.u8() & 0x7fu));
        }
    }
    return h;
}

}  // namespace hg
