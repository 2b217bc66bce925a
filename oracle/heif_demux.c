/*
 * heif_demux.c — oracle ISOBMFF/HEIF demux (TEST INFRASTRUCTURE ONLY).
 *
 * Restates the box walk of src/heif/reader.rs (read :59-83, meta :100-156,
 * iinf/infe :282-374, iref :376-422, iprp/ipco/ipma :424-513, hvcC :570-630,
 * iloc :632-704) plus what the reference lacks (construction_method 1 / idat,
 * multi-extent items, index-preserving ipco, the ImageGrid descriptor of
 * ISO/IEC 23008-12 6.6.2.3).
 */
#include "oracle_internal.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint32_t be16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
static uint32_t be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static uint64_t bev(const uint8_t *p, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 8) | p[i];
    return v;
}

typedef struct {
    const uint8_t *d;
    size_t n, pos;
    int err;
} cur_t;

static uint64_t rd(cur_t *c, int nbytes) {
    if (c->pos + (size_t)nbytes > c->n) { c->err = 1; return 0; }
    uint64_t v = bev(c->d + c->pos, nbytes);
    c->pos += nbytes;
    return v;
}

/* box header: returns payload [start,end) and type */
static int box_hdr(const uint8_t *d, size_t n, size_t pos, uint32_t *type, size_t *pstart, size_t *pend) {
    if (pos + 8 > n) return -1;
    uint64_t size = be32(d + pos);
    *type = be32(d + pos + 4);
    size_t hdr = 8;
    if (size == 1) {
        if (pos + 16 > n) return -1;
        size = bev(d + pos + 8, 8);
        hdr = 16;
    } else if (size == 0) {
        size = n - pos;
    }
    if (size < hdr || pos + size > n) return -1;
    *pstart = pos + hdr;
    *pend = pos + size;
    return 0;
}

#define FOURCC(a, b, c, d) (((uint32_t)(a) << 24) | ((uint32_t)(b) << 16) | ((uint32_t)(c) << 8) | (uint32_t)(d))

static void parse_iloc(const uint8_t *d, size_t s, size_t e, heif_file *f) {
    cur_t c = {d, e, s, 0};
    int version = (int)rd(&c, 1);
    rd(&c, 3);
    int t = (int)rd(&c, 1);
    int offset_size = t >> 4, length_size = t & 15;
    t = (int)rd(&c, 1);
    int base_offset_size = t >> 4, index_size = (version == 1 || version == 2) ? (t & 15) : 0;
    uint32_t count = version < 2 ? (uint32_t)rd(&c, 2) : (uint32_t)rd(&c, 4);
    for (uint32_t i = 0; i < count && !c.err; i++) {
        heif_item *it = NULL;
        uint32_t id = version < 2 ? (uint32_t)rd(&c, 2) : (uint32_t)rd(&c, 4);
        for (int k = 0; k < f->n_items; k++)
            if (f->items[k].id == id) it = &f->items[k];
        int cm = 0;
        if (version == 1 || version == 2) cm = (int)(rd(&c, 2) & 15);
        rd(&c, 2); /* data_reference_index */
        uint64_t base = rd(&c, base_offset_size);
        int ext = (int)rd(&c, 2);
        if (it) { it->construction_method = cm; it->n_extents = 0; }
        for (int x = 0; x < ext && !c.err; x++) {
            if (index_size) rd(&c, index_size);
            uint64_t off = rd(&c, offset_size);
            uint64_t len = rd(&c, length_size);
            if (off > UINT64_MAX - base) c.err = 1; /* base_offset + extent_offset wraps */
            if (it && it->n_extents < HEIF_MAX_EXTENTS) {
                it->ext_off[it->n_extents] = base + off;
                it->ext_len[it->n_extents] = len;
                it->n_extents++;
            }
        }
    }
}

static void parse_ipma(const uint8_t *d, size_t s, size_t e, heif_file *f) {
    cur_t c = {d, e, s, 0};
    int version = (int)rd(&c, 1);
    uint32_t flags = (uint32_t)rd(&c, 3);
    uint32_t count = (uint32_t)rd(&c, 4);
    for (uint32_t i = 0; i < count && !c.err; i++) {
        uint32_t id = version < 1 ? (uint32_t)rd(&c, 2) : (uint32_t)rd(&c, 4);
        int na = (int)rd(&c, 1);
        heif_item *it = NULL;
        for (int k = 0; k < f->n_items; k++)
            if (f->items[k].id == id) it = &f->items[k];
        for (int a = 0; a < na && !c.err; a++) {
            uint32_t idx;
            if (flags & 1) idx = (uint32_t)rd(&c, 2) & 0x7fff;
            else idx = (uint32_t)rd(&c, 1) & 0x7f;
            if (it && it->n_props < HEIF_MAX_PROPS) it->props[it->n_props++] = idx;
        }
    }
}

static heif_item *find_or_add(heif_file *f, uint32_t id) {
    for (int k = 0; k < f->n_items; k++)
        if (f->items[k].id == id) return &f->items[k];
    if (f->n_items >= HEIF_MAX_ITEMS) return NULL;
    heif_item *it = &f->items[f->n_items++];
    memset(it, 0, sizeof(*it));
    it->id = id;
    return it;
}

int heif_parse(const uint8_t *d, size_t n, heif_file *f) {
    memset(f, 0, sizeof(*f));
    f->data = d;
    f->len = n;
    size_t pos = 0;
    int have_meta = 0;
    while (pos < n) {
        uint32_t type;
        size_t s, e;
        if (box_hdr(d, n, pos, &type, &s, &e)) return oracle_fail("bad top-level box");
        if (type == FOURCC('m', 'e', 't', 'a')) {
            have_meta = 1;
            size_t p = s + 4; /* full box */
            while (p < e) {
                uint32_t t2;
                size_t s2, e2;
                if (box_hdr(d, e, p, &t2, &s2, &e2)) return oracle_fail("bad meta child");
                if (t2 == FOURCC('p', 'i', 't', 'm')) {
                    f->primary = d[s2] == 0 ? be16(d + s2 + 4) : be32(d + s2 + 4);
                } else if (t2 == FOURCC('i', 'i', 'n', 'f')) {
                    size_t q = s2 + 4 + (d[s2] == 0 ? 2 : 4);
                    while (q < e2) {
                        uint32_t t3;
                        size_t s3, e3;
                        if (box_hdr(d, e2, q, &t3, &s3, &e3)) return oracle_fail("bad infe");
                        if (t3 == FOURCC('i', 'n', 'f', 'e')) {
                            int v = d[s3];
                            if (v >= 2) {
                                uint32_t id = v == 2 ? be16(d + s3 + 4) : be32(d + s3 + 4);
                                size_t tp = s3 + 4 + (v == 2 ? 2 : 4) + 2;
                                heif_item *it = find_or_add(f, id);
                                if (it) {
                                    it->type = be32(d + tp);
                                    it->hidden = d[s3 + 3] & 1;
                                }
                            }
                        }
                        q = e3;
                    }
                } else if (t2 == FOURCC('i', 'r', 'e', 'f')) {
                    int v = d[s2];
                    size_t q = s2 + 4;
                    while (q < e2) {
                        uint32_t t3;
                        size_t s3, e3;
                        if (box_hdr(d, e2, q, &t3, &s3, &e3)) return oracle_fail("bad iref");
                        cur_t c = {d, e3, s3, 0};
                        uint32_t from = v == 0 ? (uint32_t)rd(&c, 2) : (uint32_t)rd(&c, 4);
                        int cnt = (int)rd(&c, 2);
                        if (f->n_refs < HEIF_MAX_REFS) {
                            heif_ref *r = &f->refs[f->n_refs++];
                            r->type = t3;
                            r->from = from;
                            r->n_to = 0;
                            for (int k = 0; k < cnt && !c.err; k++) {
                                uint32_t to = v == 0 ? (uint32_t)rd(&c, 2) : (uint32_t)rd(&c, 4);
                                if (r->n_to < HEIF_MAX_TO) r->to[r->n_to++] = to;
                            }
                        }
                        q = e3;
                    }
                } else if (t2 == FOURCC('i', 'p', 'r', 'p')) {
                    size_t q = s2;
                    while (q < e2) {
                        uint32_t t3;
                        size_t s3, e3;
                        if (box_hdr(d, e2, q, &t3, &s3, &e3)) return oracle_fail("bad iprp");
                        if (t3 == FOURCC('i', 'p', 'c', 'o')) {
                            size_t r = s3;
                            while (r < e3) {
                                uint32_t t4;
                                size_t s4, e4;
                                if (box_hdr(d, e3, r, &t4, &s4, &e4)) return oracle_fail("bad ipco");
                                if (f->n_props < HEIF_MAX_PROPS_TOTAL) {
                                    /* index-preserving: every child gets a slot */
                                    heif_prop *pp = &f->props[f->n_props++];
                                    pp->type = t4;
                                    pp->off = s4;
                                    pp->len = e4 - s4;
                                }
                                r = e4;
                            }
                        } else if (t3 == FOURCC('i', 'p', 'm', 'a')) {
                            /* items may be declared after; parse ipma later */
                            f->ipma_s = s3;
                            f->ipma_e = e3;
                        }
                        q = e3;
                    }
                } else if (t2 == FOURCC('i', 'l', 'o', 'c')) {
                    f->iloc_s = s2;
                    f->iloc_e = e2;
                } else if (t2 == FOURCC('i', 'd', 'a', 't')) {
                    f->idat_off = s2;
                    f->idat_len = e2 - s2;
                }
                p = e2;
            }
        }
        pos = e;
    }
    if (!have_meta) return oracle_fail("missing meta box");
    if (f->iloc_e) parse_iloc(d, f->iloc_s, f->iloc_e, f);
    if (f->ipma_e) parse_ipma(d, f->ipma_s, f->ipma_e, f);
    return 0;
}

heif_item *heif_item_by_id(heif_file *f, uint32_t id) {
    for (int k = 0; k < f->n_items; k++)
        if (f->items[k].id == id) return &f->items[k];
    return NULL;
}

const heif_prop *heif_item_prop(heif_file *f, heif_item *it, uint32_t type) {
    for (int k = 0; k < it->n_props; k++) {
        uint32_t idx = it->props[k];
        if (idx == 0 || (int)idx > f->n_props) continue;
        if (f->props[idx - 1].type == type) return &f->props[idx - 1];
    }
    return NULL;
}

/* Item payload: returns a malloc'd concatenation of extents (cm 0 → file
 * offsets, cm 1 → idat offsets). */
uint8_t *heif_item_data(heif_file *f, heif_item *it, size_t *len) {
    size_t total = 0;
    for (int x = 0; x < it->n_extents; x++) total += (size_t)it->ext_len[x];
    uint8_t *buf = (uint8_t *)malloc(total ? total : 1);
    size_t w = 0;
    for (int x = 0; x < it->n_extents; x++) {
        uint64_t off = it->ext_off[x], ln = it->ext_len[x];
        const uint8_t *src;
        if (it->construction_method == 0) {
            if (off > f->len || ln > f->len - off) { free(buf); oracle_fail("extent out of range"); return NULL; }
            src = f->data + off;
        } else if (it->construction_method == 1) {
            if (off > f->idat_len || ln > f->idat_len - off) { free(buf); oracle_fail("idat extent out of range"); return NULL; }
            src = f->data + f->idat_off + off;
        } else {
            free(buf);
            oracle_fail("unsupported construction_method");
            return NULL;
        }
        memcpy(buf + w, src, ln);
        w += ln;
    }
    *len = total;
    return buf;
}

int heif_grid_tiles(heif_file *f, uint32_t grid_id, uint32_t *tiles, int max) {
    for (int r = 0; r < f->n_refs; r++) {
        heif_ref *rf = &f->refs[r];
        if (rf->type == FOURCC('d', 'i', 'm', 'g') && rf->from == grid_id) {
            int n = rf->n_to < max ? rf->n_to : max;
            for (int k = 0; k < n; k++) tiles[k] = rf->to[k];
            return n;
        }
    }
    return 0;
}

int oracle_read_meta(const uint8_t *data, size_t len, oracle_meta *out) {
    heif_file *f = (heif_file *)calloc(1, sizeof(heif_file));
    memset(out, 0, sizeof(*out));
    if (heif_parse(data, len, f)) { free(f); return -1; }
    out->primary_item_id = f->primary;
    heif_item *pi = heif_item_by_id(f, f->primary);
    if (!pi) { free(f); return oracle_fail("primary item not found"); }
    const heif_prop *ispe = heif_item_prop(f, pi, FOURCC('i', 's', 'p', 'e'));
    if (ispe) {
        out->ispe_width = be32(data + ispe->off + 4);
        out->ispe_height = be32(data + ispe->off + 8);
    }
    const heif_prop *irot = heif_item_prop(f, pi, FOURCC('i', 'r', 'o', 't'));
    out->rotation = irot ? (data[irot->off] & 3) : 0;
    if (out->rotation == 1 || out->rotation == 3) {
        out->width = out->ispe_height;
        out->height = out->ispe_width;
    } else {
        out->width = out->ispe_width;
        out->height = out->ispe_height;
    }
    for (int r = 0; r < f->n_refs; r++)
        if (f->refs[r].type == FOURCC('t', 'h', 'm', 'b'))
            for (int k = 0; k < f->refs[r].n_to; k++)
                if (f->refs[r].to[k] == f->primary) out->num_thumbnails++;
    /* SPS bit depths of the first hvcC (as the reference does,
     * heif/grammar.rs:38-49), parsed properly */
    heif_item *coded = pi;
    if (pi->type == FOURCC('g', 'r', 'i', 'd')) {
        uint32_t tiles[1];
        if (heif_grid_tiles(f, pi->id, tiles, 1) == 1) coded = heif_item_by_id(f, tiles[0]);
        size_t gl;
        uint8_t *g = heif_item_data(f, pi, &gl);
        if (g && gl >= 8) {
            int fl = (g[1] & 1) ? 4 : 2;
            out->is_grid = 1;
            out->grid_rows = g[2] + 1u;
            out->grid_cols = g[3] + 1u;
            out->out_width = (uint32_t)bev(g + 4, fl);
            out->out_height = (uint32_t)bev(g + 4 + fl, fl);
        }
        free(g);
        out->num_tiles = out->grid_rows * out->grid_cols;
    }
    if (coded) {
        const heif_prop *hv = heif_item_prop(f, coded, FOURCC('h', 'v', 'c', 'C'));
        if (hv) {
            hevc_ps ps;
            if (hevc_parse_hvcc(data + hv->off, hv->len, &ps) == 0) {
                out->luma_bits = (uint32_t)ps.sps.bit_depth_y;
                out->chroma_bits = (uint32_t)ps.sps.bit_depth_c;
                out->chroma_format_idc = (uint32_t)ps.sps.chroma_format_idc;
                out->tile_width = (uint32_t)ps.sps.out_w;
                out->tile_height = (uint32_t)ps.sps.out_h;
            }
        }
    }
    if (!out->is_grid) {
        out->out_width = out->ispe_width;
        out->out_height = out->ispe_height;
        out->num_tiles = 1;
    }
    free(f);
    return 0;
}

int oracle_list_tiles(const uint8_t *data, size_t len, uint32_t *off, uint32_t *ln, int max,
                      uint32_t *hvcc_off, uint32_t *hvcc_len) {
    return oracle_list_item_tiles(data, len, 0, off, ln, max, hvcc_off, hvcc_len);
}

/* First auxiliary image of the primary item: an 'auxl' reference whose
 * target list holds the primary (heif/grammar.rs:202-207 parses these). */
uint32_t oracle_aux_item(const uint8_t *data, size_t len) {
    heif_file *f = (heif_file *)calloc(1, sizeof(heif_file));
    uint32_t id = 0;
    if (heif_parse(data, len, f) == 0)
        for (int r = 0; r < f->n_refs && !id; r++)
            if (f->refs[r].type == FOURCC('a', 'u', 'x', 'l'))
                for (int k = 0; k < f->refs[r].n_to; k++)
                    if (f->refs[r].to[k] == f->primary) id = f->refs[r].from;
    free(f);
    return id;
}

int oracle_list_item_tiles(const uint8_t *data, size_t len, uint32_t item_id, uint32_t *off, uint32_t *ln, int max,
                           uint32_t *hvcc_off, uint32_t *hvcc_len) {
    heif_file *f = (heif_file *)calloc(1, sizeof(heif_file));
    if (heif_parse(data, len, f)) { free(f); return -1; }
    heif_item *pi = heif_item_by_id(f, item_id ? item_id : f->primary);
    if (!pi) { free(f); return oracle_fail("no such item"); }
    uint32_t ids[HEIF_MAX_TO];
    int n;
    if (pi->type == FOURCC('g', 'r', 'i', 'd')) n = heif_grid_tiles(f, pi->id, ids, HEIF_MAX_TO);
    else { ids[0] = pi->id; n = 1; }
    int w = 0;
    for (int k = 0; k < n && w < max; k++) {
        heif_item *it = heif_item_by_id(f, ids[k]);
        if (!it || it->construction_method != 0 || it->n_extents != 1) { free(f); return oracle_fail("tile layout"); }
        off[w] = (uint32_t)it->ext_off[0];
        ln[w] = (uint32_t)it->ext_len[0];
        if (k == 0) {
            const heif_prop *hv = heif_item_prop(f, it, FOURCC('h', 'v', 'c', 'C'));
            if (!hv) { free(f); return oracle_fail("no hvcC"); }
            *hvcc_off = (uint32_t)hv->off;
            *hvcc_len = (uint32_t)hv->len;
        }
        w++;
    }
    free(f);
    return w;
}
