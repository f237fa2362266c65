/* TEST-ONLY sanitizer driver: the oracle restatements (oracle/*.c) built with
 * -fsanitize=address,undefined and run over every file named on the command line:
 *   .jpg -> or_nj_decode (and the trace), then or_tje_encode q1..3 and or_jpeg_encode 420/444 of
 *           the decoded pixels; .hdr -> or_hdr_decode; every decoded RGB image also goes through
 *           the PNG colour choice, filters and zlib encode.
 * The reference's two UB idioms (signed left shifts in the IDCT, jpeg_dec.h:352,397; bits <<
 * (32 - n) with n = 0, jpeg_enc.h:627) are restated with defined operations; UBSan checks that
 * they stay so. Exit status 0 = no sanitizer report (-fno-sanitize-recover=all aborts). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/oracle.h"

static uint8_t* slurp(const char* path, int64_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    *n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t* b = (uint8_t*)malloc(*n > 0 ? *n : 1);
    if (*n > 0 && fread(b, 1, (size_t)*n, f) != (size_t)*n) { free(b); b = NULL; }
    fclose(f);
    return b;
}

static void png_path(const uint8_t* px, int w, int h, int d) {
    or_png_mode m;
    if (!or_png_choose(px, w, h, d, &m)) return;
    const int64_t n = or_png_filtered_size(w, h, &m);
    uint8_t* f = (uint8_t*)malloc(n > 0 ? n : 1);
    or_png_filter(px, w, h, d, &m, f);
    free(f);
    uint8_t* png = NULL;
    int64_t sz = 0;
    if (or_png_encode(px, w, h, d, 6, &png, &sz)) or_free(png);
}

int main(int argc, char** argv) {
    int files = 0;
    for (int a = 1; a < argc; ++a) {
        int64_t n = 0;
        uint8_t* data = slurp(argv[a], &n);
        if (!data) { fprintf(stderr, "cannot read %s\n", argv[a]); return 2; }
        const size_t L = strlen(argv[a]);
        if (L > 4 && !strcmp(argv[a] + L - 4, ".hdr")) {
            float* out = NULL;
            int w = 0, h = 0, rows = 0;
            or_hdr_decode(data, n, &out, &w, &h, &rows);
            or_free(out);
        } else {
            uint8_t* px = NULL;
            int w = 0, h = 0, c = 0;
            static int16_t coef[64 * 70000];
            static int32_t dc[70000];
            or_trace t = {0, coef, dc, 70000};
            const int code = or_nj_decode(data, n, &px, &w, &h, &c, &t);
            if (code == 0 && px && c == 3 && (int64_t)w * h <= 4096 * 4096) {
                for (int q = 1; q <= 3; ++q) {
                    uint8_t* o = NULL;
                    int64_t ol = 0;
                    if (or_tje_encode(q, w, h, 3, px, &o, &ol)) or_free(o);
                }
                for (int s = 0; s < 2; ++s) {
                    uint8_t* o = NULL;
                    int64_t ol = 0;
                    if (or_jpeg_encode(90, s ? 420 : 444, w, h, 3, px, &o, &ol)) or_free(o);
                }
                if ((int64_t)w * h <= 1024 * 1024) png_path(px, w, h, 3);
            }
            or_free(px);
        }
        free(data);
        ++files;
    }
    printf("sanitized %d files\n", files);
    return 0;
}
