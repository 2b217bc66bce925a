/* heifgpu_caller.c — a plain C host of the C ABI (include/heifgpu.h), built
 * with gcc by tests/test_c_caller.py: the seam a Rust or C maintainer binds
 * in place of the serial tile loop of src/heic/decoder.rs:114-119.
 *
 *   heifgpu_caller FILE             parse -> info -> tile_params -> parse_many,
 *                                   checked against halfmoonbay's values
 *                                   (tests/libheif_comparison.rs:9-112)
 *   heifgpu_caller FILE --decode OUT
 *                                   also decodes on device 0 (heifgpu_decode_batch),
 *                                   then again as two tile subsets gathered into one
 *                                   image (heifgpu_batch_prepare_ex + heifgpu_gather_tiles),
 *                                   and writes Y, Cb, Cr of both decodes to OUT
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "heifgpu.h"

#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (!(cond)) {                                     \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                  \
            fprintf(stderr, " (%s)\n", heifgpu_last_error()); \
            exit(1);                                       \
        }                                                  \
    } while (0)

static unsigned char *read_file(const char *path, size_t *n) {
    FILE *f = fopen(path, "rb");
    CHECK(f != NULL, "open %s", path);
    fseek(f, 0, SEEK_END);
    long len = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char *buf = (unsigned char *)malloc((size_t)len);
    CHECK(fread(buf, 1, (size_t)len, f) == (size_t)len, "read %s", path);
    fclose(f);
    *n = (size_t)len;
    return buf;
}

typedef struct {
    void *dev[3];
    size_t bytes[3];
    heifgpu_planes planes;
} DevPlanes;

static void alloc_planes(DevPlanes *p, const heifgpu_image_info *info) {
    const int cw = (int)(info->width + 1) / 2, ch = (int)(info->height + 1) / 2;
    const int w[3] = {(int)info->width, cw, cw}, h[3] = {(int)info->height, ch, ch};
    for (int c = 0; c < 3; ++c) {
        p->bytes[c] = (size_t)w[c] * (size_t)h[c] * info->bytes_per_sample;
        CHECK(hipMalloc(&p->dev[c], p->bytes[c]) == hipSuccess, "hipMalloc");
        CHECK(hipMemset(p->dev[c], 0, p->bytes[c]) == hipSuccess, "hipMemset");
        p->planes.plane[c] = p->dev[c];
        p->planes.pitch[c] = w[c] * (int)info->bytes_per_sample;
    }
}

static void write_planes(FILE *f, const DevPlanes *p) {
    for (int c = 0; c < 3; ++c) {
        void *host = malloc(p->bytes[c]);
        CHECK(hipMemcpy(host, p->dev[c], p->bytes[c], hipMemcpyDeviceToHost) == hipSuccess, "hipMemcpy");
        CHECK(fwrite(host, 1, p->bytes[c], f) == p->bytes[c], "write");
        free(host);
    }
}

int main(int argc, char **argv) {
    CHECK(argc >= 2, "usage: heifgpu_caller FILE [--decode OUT]");
    CHECK(HEIFGPU_ABI_VERSION == 6, "ABI version");
    CHECK(heifgpu_abi_version() == HEIFGPU_ABI_VERSION, "library ABI %d, header %d", heifgpu_abi_version(),
          HEIFGPU_ABI_VERSION);
    CHECK(sizeof(heifgpu_batch_opts) == 20, "heifgpu_batch_opts is %zu bytes", sizeof(heifgpu_batch_opts));
    CHECK(sizeof(heifgpu_image_info) == 80, "heifgpu_image_info is %zu bytes", sizeof(heifgpu_image_info));
    size_t n = 0;
    unsigned char *data = read_file(argv[1], &n);

    heifgpu_image *img = NULL;
    CHECK(heifgpu_image_parse(data, n, &img) == HEIFGPU_OK && img, "heifgpu_image_parse");
    heifgpu_image_info info;
    memset(&info, 0xab, sizeof(info));
    CHECK(heifgpu_image_get_info(img, &info) == HEIFGPU_OK, "heifgpu_image_get_info");
    /* tests/libheif_comparison.rs:102-111 and SURVEY Appendix A */
    CHECK(info.ispe_width == 4032 && info.ispe_height == 3024, "ispe %ux%u", info.ispe_width, info.ispe_height);
    CHECK(info.width == 4032 && info.height == 3024, "size");
    CHECK(info.bit_depth == 8 && info.chroma_format_idc == 1 && info.bytes_per_sample == 1, "format");
    CHECK(info.primary_item_id == 49 && info.item_id == 49 && info.num_thumbnails == 0, "primary");
    CHECK(info.rotation == 3, "irot");
    CHECK(info.grid_rows == 6 && info.grid_cols == 8 && info.num_tiles == 48, "grid");
    CHECK(info.tile_width == 512 && info.tile_height == 512, "tile size");
    CHECK(info.coded_bytes == 1704187, "coded bytes %u", info.coded_bytes);
    CHECK(info.matrix_coeffs == 6 && info.full_range == 1, "colour");
    CHECK(info.aux_item_id == 52, "aux item %u", info.aux_item_id);

    heifgpu_tile_params tp;
    CHECK(heifgpu_image_tile_params(img, 0, &tp) == HEIFGPU_OK, "tile_params");
    CHECK(tp.pic_width == 512 && tp.pic_height == 512 && tp.log2_ctb == 5 && tp.log2_min_cb == 3, "sps");
    CHECK(tp.init_qp == 15 && tp.slice_qp_y == 15 && tp.entropy_coding_sync == 1, "pps / slice");
    CHECK(tp.num_entry_point_offsets == 15 && tp.entry_point_offset[0] == 136 && tp.entry_point_offset[14] == 78,
          "entry points");
    CHECK(heifgpu_image_tile_params(img, 48, &tp) == HEIFGPU_E_INVALID, "tile 48 must be out of range");

    const uint8_t *many[3] = {data, data, (const uint8_t *)"junk"};
    size_t lens[3] = {n, n, 4};
    heifgpu_image *imgs[3];
    int rcs[3];
    CHECK(heifgpu_image_parse_many(many, lens, 3, 2, imgs, rcs) == HEIFGPU_E_PARSE, "parse_many error code");
    CHECK(imgs[0] && imgs[1] && !imgs[2] && rcs[0] == 0 && rcs[1] == 0 && rcs[2] == HEIFGPU_E_PARSE, "parse_many");
    heifgpu_image_free(imgs[0]);
    heifgpu_image_free(imgs[1]);
    printf("host ABI ok: %ux%u grid %ux%u, %u tiles\n", info.width, info.height, info.grid_rows, info.grid_cols,
           info.num_tiles);

    if (argc >= 4 && strcmp(argv[2], "--decode") == 0) {
        heifgpu_ctx *ctx = NULL;
        CHECK(heifgpu_create(0, &ctx) == HEIFGPU_OK, "heifgpu_create");
        DevPlanes full, part[2], merged;
        alloc_planes(&full, &info);
        uint32_t status = 0xffffffffu;
        const heifgpu_image *one[1] = {img};
        CHECK(heifgpu_decode_batch(ctx, one, 1, &full.planes, NULL, &status) == HEIFGPU_OK && status == 0,
              "heifgpu_decode_batch (status %u)", status);
        /* the same image as two tile subsets (one per GPU in a split; one device here), then gathered */
        alloc_planes(&merged, &info);
        for (uint32_t g = 0; g < 2; ++g) {
            alloc_planes(&part[g], &info);
            heifgpu_batch *b = NULL;
            heifgpu_batch_opts o = {2, g, g ? HEIFGPU_PARSE_LANES : HEIFGPU_PARSE_SOLO, 0, g ? 2u : 0u};
            CHECK(heifgpu_batch_prepare_ex(ctx, one, 1, &o, &b) == HEIFGPU_OK, "prepare_ex");
            CHECK(heifgpu_batch_decode(ctx, b, &part[g].planes, NULL) == HEIFGPU_OK, "batch_decode");
            CHECK(heifgpu_batch_status(ctx, b, &status, NULL) == HEIFGPU_OK && status == 0, "batch_status");
            heifgpu_batch_free(b);
            CHECK(heifgpu_gather_tiles(&info, &merged.planes, &part[g].planes, 2, g, NULL) == HEIFGPU_OK, "gather");
        }
        CHECK(hipDeviceSynchronize() == hipSuccess, "sync");
        FILE *f = fopen(argv[3], "wb");
        CHECK(f != NULL, "open %s", argv[3]);
        write_planes(f, &full);
        write_planes(f, &merged);
        fclose(f);
        heifgpu_destroy(ctx);
        printf("decode ok\n");
    }
    heifgpu_image_free(img);
    free(data);
    return 0;
}
