/* oracle_cli.c — debugging driver for the CPU oracle (TEST INFRASTRUCTURE ONLY).
 * usage: oracle_cli file.heic [out.yuv]   (writes 8-bit planar Y, Cb, Cr) */
#include "oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <time.h>

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s file.heic [out.yuv]\n", argv[0]); return 2; }
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror("open"); return 2; }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char *buf = malloc((size_t)n);
    if (fread(buf, 1, (size_t)n, f) != (size_t)n) { perror("read"); return 2; }
    fclose(f);
    oracle_meta m;
    if (oracle_read_meta(buf, (size_t)n, &m)) { fprintf(stderr, "meta: %s\n", oracle_last_error()); return 1; }
    printf("meta: ispe %ux%u rot %u -> %ux%u bits %u/%u thumbs %u grid %ux%u out %ux%u tiles %u\n", m.ispe_width,
           m.ispe_height, m.rotation, m.width, m.height, m.luma_bits, m.chroma_bits, m.num_thumbnails, m.grid_rows,
           m.grid_cols, m.out_width, m.out_height, m.num_tiles);
    static oracle_substream_check ck[4096];
    int nck = 0;
    oracle_image img;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int rc = oracle_decode_heic(buf, (size_t)n, &img, ck, 4096, &nck);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    double ms = (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_nsec - t0.tv_nsec) / 1e6;
    int bad = 0;
    for (int i = 0; i < nck; i++)
        if (!ck[i].term_ok || ck[i].raw_start != ck[i].raw_entry) {
            if (bad < 10)
                printf("substream tile %u sub %u: start %u entry %u term_ok %u\n", ck[i].tile, ck[i].substream,
                       ck[i].raw_start, ck[i].raw_entry, ck[i].term_ok);
            bad++;
        }
    printf("decode rc=%d (%s) in %.1f ms; substreams %d, bad %d\n", rc, rc ? oracle_last_error() : "ok", ms, nck, bad);
    if (rc) return 1;
    if (argc > 2) {
        FILE *o = fopen(argv[2], "wb");
        for (int c = 0; c < 3; c++)
            for (size_t i = 0; i < (size_t)img.pw[c] * img.ph[c]; i++) fputc(img.plane[c][i] & 255, o);
        fclose(o);
        printf("wrote %ux%u yuv420p to %s\n", img.width, img.height, argv[2]);
    }
    oracle_image_free(&img);
    return bad ? 1 : 0;
}
