/* TEST INFRASTRUCTURE ONLY -- the parity checker for the PNG encode path.
 *
 * CPU restatement of what lodepng (reference png_encoder.cpp, lodepng 20230410) decides and
 * filters for png_encoder::saveToFile (png_encoder.cpp:4474-4486: RGB8 for d == 3, else RGBA8,
 * lodepng defaults: auto_convert, LFS_MINSUM, filter_palette_zero):
 *   or_png_choose  -- lodepng_compute_color_stats (:3357-3543) + auto_choose_color (:3552-3616)
 *   or_png_filter  -- lodepng_convert/rgba8ToPixel (:2781-2835, addColorBits :2706-2714),
 *                     preProcessScanlines row padding (:4160-4180) and filter() (:3935-3983,
 *                     filterScanline :3820-3865, paethPredictor :3621-3631)
 *   or_png_encode  -- the PNG container (signature, IHDR :3723, PLTE :3742, tRNS :3763, IDAT,
 *                     IEND) around a zlib stream.
 * png_encoder.cpp includes libpng's png.h, which this image lacks, so the reference is
 * unbuildable here; colour choice and filter bytes are pinned by data/test.png (palette, filter 0,
 * SURVEY.md §8(c)) and the restated rules. The deflate itself is NOT a restatement: lodepng's
 * LZ77/package-merge coder is replaced here by the system zlib (compress2) as a size proxy and
 * CPU baseline; the parity contract for IDAT is "inflates to the identical filtered stream".
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "oracle.h"

enum { LCT_GREY = 0, LCT_RGB = 2, LCT_PALETTE = 3, LCT_GREY_ALPHA = 4, LCT_RGBA = 6 };

static unsigned required_bits(unsigned v) {  // getValueRequiredBits (:3349-3355)
    if (v == 0 || v == 255) return 1;
    if (v % 17 == 0) return v % 85 == 0 ? 2 : 4;
    return 8;
}

/* Distinct-colour set in first-seen order, capped at 257 (the ColorTree use of :3496-3512). */
typedef struct {
    uint32_t key[1024];
    int16_t idx[1024];
    int n;
} ColorSet;
static int cs_find(const ColorSet* s, uint32_t c) {
    uint32_t h = (c * 2654435761u) >> 22;
    for (;; h = (h + 1) & 1023) {
        if (s->idx[h] < 0) return -1 - (int)h;
        if (s->key[h] == c) return s->idx[h];
    }
}

int or_png_choose(const uint8_t* px, int w, int h, int d, or_png_mode* m) {
    if (!px || w <= 0 || h <= 0 || (d != 3 && d != 4) || !m) return 0;
    memset(m, 0, sizeof *m);
    const int64_t np = (int64_t)w * h;
    ColorSet* cs = (ColorSet*)malloc(sizeof(ColorSet));
    if (!cs) return 0;
    memset(cs->idx, 0xFF, sizeof cs->idx);
    cs->n = 0;
    unsigned colored = 0, alpha = 0, key = 0, bits = 1, numcolors = 0;
    unsigned kr = 0, kg = 0, kb = 0;
    uint8_t pal[256 * 4];
    /* RGB8 input cannot have alpha (lodepng_can_have_alpha :2653): alpha_done from the start.
     * bits_done = bits >= bpp (24/32) never holds for 8-bit RGB(A) input, so the scan never
     * stops early and every pixel is visited (:3462-3516). */
    const int alpha_done0 = d == 3;
    int alpha_done = alpha_done0, numcolors_done = 0;
    for (int64_t i = 0; i < np; ++i) {
        const uint8_t* p = px + i * d;
        const unsigned r = p[0], g = p[1], b = p[2], a = d == 4 ? p[3] : 255;
        if (bits < 8) {
            const unsigned q = required_bits(r);
            if (q > bits) bits = q;
        }
        if (!colored && (r != g || r != b)) {
            colored = 1;
            if (bits < 8) bits = 8;
        }
        if (!alpha_done) {
            const unsigned matchkey = r == kr && g == kg && b == kb;
            if (a != 255 && (a != 0 || (key && !matchkey))) {
                alpha = 1;
                key = 0;
                alpha_done = 1;
                if (bits < 8) bits = 8;
            } else if (a == 0 && !alpha && !key) {
                key = 1;
                kr = r;
                kg = g;
                kb = b;
            } else if (a == 255 && key && matchkey) {
                alpha = 1;
                key = 0;
                alpha_done = 1;
                if (bits < 8) bits = 8;
            }
        }
        if (!numcolors_done) {
            const uint32_t c = (uint32_t)r | (uint32_t)g << 8 | (uint32_t)b << 16 | (uint32_t)a << 24;
            const int f = cs_find(cs, c);
            if (f < 0) {
                const int slot = -1 - f;
                cs->key[slot] = c;
                cs->idx[slot] = (int16_t)numcolors;
                if (numcolors < 256) memcpy(pal + numcolors * 4, (uint8_t[4]){(uint8_t)r, (uint8_t)g, (uint8_t)b, (uint8_t)a}, 4);
                ++numcolors;
                numcolors_done = numcolors >= 257;
            }
        }
    }
    if (key && !alpha) {  // :3518-3528
        for (int64_t i = 0; i < np; ++i) {
            const uint8_t* p = px + i * d;
            const unsigned a = d == 4 ? p[3] : 255;
            if (a != 0 && p[0] == kr && p[1] == kg && p[2] == kb) {
                alpha = 1;
                key = 0;
                if (bits < 8) bits = 8;
            }
        }
    }
    free(cs);
    const unsigned k16r = kr + (kr << 8), k16g = kg + (kg << 8), k16b = kb + (kb << 8);  // :3531-3533

    /* auto_choose_color (:3552-3616) */
    if (key && np <= 16) {
        alpha = 1;
        key = 0;
        if (bits < 8) bits = 8;
    }
    const unsigned gray_ok = !colored;
    if (!gray_ok && bits < 8) bits = 8;
    const unsigned n = numcolors;
    const unsigned palettebits = n <= 2 ? 1 : (n <= 4 ? 2 : (n <= 16 ? 4 : 8));
    unsigned palette_ok = n <= 256 && bits <= 8 && n != 0;
    if ((uint64_t)np < (uint64_t)n * 2) palette_ok = 0;
    if (gray_ok && !alpha && bits <= palettebits) palette_ok = 0;
    if (palette_ok) {
        m->colortype = LCT_PALETTE;
        m->bitdepth = (int)palettebits;
        m->npal = (int)n;
        memcpy(m->pal, pal, n * 4);
    } else {
        m->bitdepth = (int)bits;
        m->colortype = alpha ? (gray_ok ? LCT_GREY_ALPHA : LCT_RGBA) : (gray_ok ? LCT_GREY : LCT_RGB);
        if (key) {
            const unsigned mask = (1u << m->bitdepth) - 1u;
            m->key_defined = 1;
            m->key_r = (int)(k16r & mask);
            m->key_g = (int)(k16g & mask);
            m->key_b = (int)(k16b & mask);
        }
    }
    return 1;
}

static int mode_bpp(const or_png_mode* m) {
    const int ch = m->colortype == LCT_RGB ? 3 : m->colortype == LCT_RGBA ? 4 : m->colortype == LCT_GREY_ALPHA ? 2 : 1;
    return ch * m->bitdepth;
}

int64_t or_png_linebytes(int w, const or_png_mode* m) { return ((int64_t)w * mode_bpp(m) + 7) / 8; }

int64_t or_png_filtered_size(int w, int h, const or_png_mode* m) { return (int64_t)h * (1 + or_png_linebytes(w, m)); }

/* Converted, row-padded scanline y (lodepng_convert + addPaddingBits). */
static void convert_row(const uint8_t* px, int w, int d, const or_png_mode* m, int y, uint8_t* row, int64_t lb) {
    memset(row, 0, (size_t)lb);
    const uint8_t* src = px + (int64_t)y * w * d;
    for (int x = 0; x < w; ++x) {
        const uint8_t* p = src + (int64_t)x * d;
        const uint8_t r = p[0], g = p[1], b = p[2], a = d == 4 ? p[3] : 255;
        switch (m->colortype) {
            case LCT_RGBA: memcpy(row + 4 * x, (uint8_t[4]){r, g, b, a}, 4); break;
            case LCT_RGB: memcpy(row + 3 * x, (uint8_t[3]){r, g, b}, 3); break;
            case LCT_GREY_ALPHA: row[2 * x] = r; row[2 * x + 1] = a; break;
            default: {
                unsigned v;
                if (m->colortype == LCT_GREY) {
                    v = m->bitdepth == 8 ? r : ((unsigned)r >> (8 - m->bitdepth)) & ((1u << m->bitdepth) - 1u);
                } else {  // palette index (color_tree_get)
                    v = 0;
                    for (int k = 0; k < m->npal; ++k)
                        if (m->pal[4 * k] == r && m->pal[4 * k + 1] == g && m->pal[4 * k + 2] == b && m->pal[4 * k + 3] == a) {
                            v = (unsigned)k;
                            break;
                        }
                }
                if (m->bitdepth == 8) row[x] = (uint8_t)v;
                else {
                    const int per = 8 / m->bitdepth;  // MSB-first packing (addColorBits)
                    row[x / per] |= (uint8_t)(v << (m->bitdepth * (per - 1 - x % per)));
                }
            }
        }
    }
}

static uint8_t paeth(uint8_t a, uint8_t b, uint8_t c) {  // paethPredictor (:3621-3631)
    short pa = (short)abs(b - c), pb = (short)abs(a - c), pc = (short)abs(a + b - c - c);
    if (pb < pa) { a = b; pa = pb; }
    return pc < pa ? c : a;
}

static void filter_row(uint8_t* out, const uint8_t* s, const uint8_t* prev, int64_t n, int bw, int type) {
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t left = i >= bw ? s[i - bw] : 0, up = prev ? prev[i] : 0, ul = (prev && i >= bw) ? prev[i - bw] : 0;
        uint8_t pred = 0;
        switch (type) {
            case 1: pred = left; break;
            case 2: pred = up; break;
            case 3: pred = (uint8_t)((left + up) >> 1); break;
            case 4: pred = paeth(left, up, ul); break;
            default: pred = 0;
        }
        out[i] = (uint8_t)(s[i] - pred);
    }
}

int or_png_filter(const uint8_t* px, int w, int h, int d, const or_png_mode* m, uint8_t* out) {
    const int64_t lb = or_png_linebytes(w, m);
    const int bw = (mode_bpp(m) + 7) / 8;
    const int zero = m->colortype == LCT_PALETTE || m->bitdepth < 8;  // filter_palette_zero
    uint8_t* cur = (uint8_t*)malloc((size_t)lb + 1);
    uint8_t* prv = (uint8_t*)malloc((size_t)lb + 1);
    uint8_t* att = (uint8_t*)malloc((size_t)lb * 5 + 1);
    if (!cur || !prv || !att) { free(cur); free(prv); free(att); return 0; }
    for (int y = 0; y < h; ++y) {
        convert_row(px, w, d, m, y, cur, lb);
        const uint8_t* prev = y ? prv : NULL;
        uint8_t* o = out + (int64_t)y * (lb + 1);
        int best = 0;
        if (zero) {
            filter_row(att, cur, prev, lb, bw, 0);
        } else {
            uint64_t smallest = 0;
            for (int t = 0; t < 5; ++t) {
                uint8_t* a = att + (int64_t)t * lb;
                filter_row(a, cur, prev, lb, bw, t);
                uint64_t sum = 0;
                for (int64_t x = 0; x < lb; ++x) sum += t == 0 ? a[x] : (a[x] < 128 ? a[x] : 255u - a[x]);
                if (t == 0 || sum < smallest) { best = t; smallest = sum; }
            }
        }
        o[0] = (uint8_t)best;
        memcpy(o + 1, att + (int64_t)best * lb, (size_t)lb);
        uint8_t* t = prv; prv = cur; cur = t;
    }
    free(cur); free(prv); free(att);
    return 1;
}

static void be32(uint8_t* p, uint32_t v) { p[0] = v >> 24; p[1] = v >> 16; p[2] = v >> 8; p[3] = v; }

static uint8_t* put_chunk(uint8_t* o, const char* type, const uint8_t* data, uint32_t n) {
    be32(o, n);
    memcpy(o + 4, type, 4);
    if (n) memcpy(o + 8, data, n);
    be32(o + 8 + n, (uint32_t)crc32(0, o + 4, n + 4));
    return o + 12 + n;
}

int or_png_encode(const uint8_t* px, int w, int h, int d, int zlevel, uint8_t** out, int64_t* size) {
    or_png_mode m;
    if (!or_png_choose(px, w, h, d, &m)) return 0;
    const int64_t fs = or_png_filtered_size(w, h, &m);
    uint8_t* filt = (uint8_t*)malloc((size_t)fs);
    if (!filt || !or_png_filter(px, w, h, d, &m, filt)) { free(filt); return 0; }
    uLongf zn = compressBound((uLong)fs);
    uint8_t* z = (uint8_t*)malloc(zn);
    if (!z || compress2(z, &zn, filt, (uLong)fs, zlevel) != Z_OK) { free(filt); free(z); return 0; }
    free(filt);
    uint8_t* o = (uint8_t*)malloc(zn + 2048);
    if (!o) { free(z); return 0; }
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    memcpy(o, sig, 8);
    uint8_t ihdr[13];
    be32(ihdr, (uint32_t)w);
    be32(ihdr + 4, (uint32_t)h);
    ihdr[8] = (uint8_t)m.bitdepth;
    ihdr[9] = (uint8_t)m.colortype;
    ihdr[10] = ihdr[11] = ihdr[12] = 0;
    uint8_t* p = put_chunk(o + 8, "IHDR", ihdr, 13);
    uint8_t tr[256];
    uint32_t ntr = 0;
    if (m.colortype == LCT_PALETTE) {
        uint8_t pl[768];
        for (int i = 0; i < m.npal; ++i) memcpy(pl + 3 * i, m.pal + 4 * i, 3);
        p = put_chunk(p, "PLTE", pl, (uint32_t)m.npal * 3);
        ntr = (uint32_t)m.npal;
        while (ntr && m.pal[4 * (ntr - 1) + 3] == 255) --ntr;
        for (uint32_t i = 0; i < ntr; ++i) tr[i] = m.pal[4 * i + 3];
    } else if (m.key_defined && m.colortype == LCT_GREY) {
        tr[0] = (uint8_t)(m.key_r >> 8); tr[1] = (uint8_t)m.key_r; ntr = 2;
    } else if (m.key_defined && m.colortype == LCT_RGB) {
        const int k[3] = {m.key_r, m.key_g, m.key_b};
        for (int i = 0; i < 3; ++i) { tr[2 * i] = (uint8_t)(k[i] >> 8); tr[2 * i + 1] = (uint8_t)k[i]; }
        ntr = 6;
    }
    if (ntr) p = put_chunk(p, "tRNS", tr, ntr);
    p = put_chunk(p, "IDAT", z, (uint32_t)zn);
    p = put_chunk(p, "IEND", NULL, 0);
    free(z);
    *out = o;
    *size = p - o;
    return 1;
}
