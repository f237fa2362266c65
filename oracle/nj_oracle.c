/*
 * nj_oracle.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Reentrant CPU restatement of the NanoJPEG 1.3.5 decoder that ImageCodecs
 * vendors as /root/reference/jpeg_dec.h.  Organisation differs on purpose (an
 * explicit context, a canonical Huffman lookup instead of the 64K direct table),
 * but every observable result -- return code, dimensions, pixel bytes -- follows
 * the reference line by line as cited.  All intermediate integer arithmetic uses
 * wrap-around 32-bit semantics, matching what the reference compiles to.
 */
#include "oracle.h"

#include <limits.h>
#include <stdlib.h>
#include <string.h>

#define OR_FINISHED 6 /* jpeg_dec.h:124 (__NJ_FINISHED, internal) */

typedef int32_t i32;
typedef uint32_t u32;

/* wrap-around helpers: the reference's int arithmetic (incl. `x << k` on negatives,
 * jpeg_dec.h:352,397) as executed on two's-complement hardware */
static inline i32 wadd(i32 a, i32 b) { return (i32)((u32)a + (u32)b); }
static inline i32 wsub(i32 a, i32 b) { return (i32)((u32)a - (u32)b); }
static inline i32 wmul(i32 a, i32 b) { return (i32)((u32)a * (u32)b); }
static inline i32 wshl(i32 a, int k) { return (i32)((u32)a << k); }

static inline uint8_t clamp_u8(i32 v) { return v < 0 ? 0 : (v > 255 ? 255 : (uint8_t)v); } /* :339-341 */

/* natural index of the k-th zig-zag coefficient (jpeg_dec.h:334-337) */
static const uint8_t kDezigzag[64] = {
     0,  1,  8, 16,  9,  2,  3, 10, 17, 24, 32, 25, 18, 11,  4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,  6,  7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63 };

/* Canonical form of one DHT table. A table NanoJPEG never saw is all-invalid
 * (its vlctab stays zeroed by njInit, jpeg_dec.h:868-870). */
typedef struct {
    uint8_t count[17];   /* codes per length 1..16                           */
    uint8_t symbol[256]; /* symbols in code order (jpeg_dec.h:600-607)       */
    u32 bound[17];       /* left-justified 16-bit upper bound after length L */
    int first[17];       /* index in symbol[] of the first length-L code     */
} or_huff;

typedef struct {
    int id, hs, vs;      /* cid, ssx, ssy        (jpeg_dec.h:302-311) */
    int w, h, stride;
    int tq, dc_tab, ac_tab;
    i32 pred;
    uint8_t* plane;
} or_comp;

typedef struct {
    /* byte cursor: nj.pos / nj.size / nj.length (jpeg_dec.h:315-317) */
    const uint8_t* at;
    int avail;
    int seg;
    int status; /* nj.error */
    int W, H, nc;
    int mbw, mbh, mbx_px, mby_px;
    or_comp c[3];
    uint8_t q[4][64];
    or_huff huff[4];
    int restart;
    uint8_t* rgb;
    /* bit reader (jpeg_dec.h:326) */
    u32 acc;
    int nacc;
    or_trace* trace;
} or_ctx;

/* ---- cursor helpers: njSkip / njDecodeLength / njSkipMarker (jpeg_dec.h:500-521) ---- */
static void cur_skip(or_ctx* d, int n) {
    d->at += n;
    d->avail -= n;
    d->seg -= n;
    if (d->avail < 0) d->status = OR_SYNTAX_ERROR;
}
static int be16(const uint8_t* p) { return (p[0] << 8) | p[1]; }
static void seg_open(or_ctx* d) {
    if (d->avail < 2) { d->status = OR_SYNTAX_ERROR; return; }
    d->seg = be16(d->at);
    if (d->seg > d->avail) { d->status = OR_SYNTAX_ERROR; return; }
    cur_skip(d, 2);
}
static void seg_skip_whole(or_ctx* d) { seg_open(d); cur_skip(d, d->seg); }

/* ---- SOF0 (jpeg_dec.h:523-575) ---- */
static void read_sof(or_ctx* d) {
    seg_open(d);
    if (d->status) return;
    if (d->seg < 9) { d->status = OR_SYNTAX_ERROR; return; }
    if (d->at[0] != 8) { d->status = OR_UNSUPPORTED; return; }
    d->H = be16(d->at + 1);
    d->W = be16(d->at + 3);
    if (d->W == 0 || d->H == 0) { d->status = OR_SYNTAX_ERROR; return; }
    d->nc = d->at[5];
    cur_skip(d, 6);
    if (d->nc != 1 && d->nc != 3) { d->status = OR_UNSUPPORTED; return; }
    if (d->seg < d->nc * 3) { d->status = OR_SYNTAX_ERROR; return; }
    int hmax = 0, vmax = 0;
    for (int i = 0; i < d->nc; ++i) {
        or_comp* c = &d->c[i];
        c->id = d->at[0];
        c->hs = d->at[1] >> 4;
        if (!c->hs) { d->status = OR_SYNTAX_ERROR; return; }
        if (c->hs & (c->hs - 1)) { d->status = OR_UNSUPPORTED; return; }
        c->vs = d->at[1] & 15;
        if (!c->vs) { d->status = OR_SYNTAX_ERROR; return; }
        if (c->vs & (c->vs - 1)) { d->status = OR_UNSUPPORTED; return; }
        c->tq = d->at[2];
        if (c->tq & 0xFC) { d->status = OR_SYNTAX_ERROR; return; }
        cur_skip(d, 3);
        if (c->hs > hmax) hmax = c->hs;
        if (c->vs > vmax) vmax = c->vs;
    }
    if (d->nc == 1) { d->c[0].hs = d->c[0].vs = hmax = vmax = 1; }
    d->mbx_px = hmax << 3;
    d->mby_px = vmax << 3;
    d->mbw = (d->W + d->mbx_px - 1) / d->mbx_px;
    d->mbh = (d->H + d->mby_px - 1) / d->mby_px;
    for (int i = 0; i < d->nc; ++i) {
        or_comp* c = &d->c[i];
        c->w = (d->W * c->hs + hmax - 1) / hmax;
        c->h = (d->H * c->vs + vmax - 1) / vmax;
        c->stride = (d->mbw * c->hs) << 3;
        if ((c->w < 3 && c->hs != hmax) || (c->h < 3 && c->vs != vmax)) { d->status = OR_UNSUPPORTED; return; }
        int64_t bytes = (int64_t)c->stride * ((int64_t)(d->mbh * c->vs) << 3);
        free(c->plane); /* a repeated SOF re-allocates (the reference leaks the old plane) */
        c->plane = (bytes > INT_MAX) ? NULL : (uint8_t*)calloc((size_t)bytes, 1);
        if (!c->plane) { d->status = OR_OUT_OF_MEM; return; }
    }
    if (d->nc == 3) {
        int64_t bytes = (int64_t)d->W * d->H * d->nc;
        free(d->rgb);
        d->rgb = (bytes > INT_MAX) ? NULL : (uint8_t*)malloc((size_t)bytes);
        if (!d->rgb) { d->status = OR_OUT_OF_MEM; return; }
    }
    cur_skip(d, d->seg);
}

/* ---- DHT (jpeg_dec.h:577-616): keep the canonical counts + symbols ---- */
static void read_dht(or_ctx* d) {
    seg_open(d);
    if (d->status) return;
    while (d->seg >= 17) {
        int tc = d->at[0];
        if (tc & 0xEC) { d->status = OR_SYNTAX_ERROR; return; }
        if (tc & 0x02) { d->status = OR_UNSUPPORTED; return; }
        or_huff* t = &d->huff[(tc | (tc >> 3)) & 3];
        uint8_t cnt[17];
        cnt[0] = 0;
        for (int L = 1; L <= 16; ++L) cnt[L] = d->at[L];
        cur_skip(d, 17);
        memset(t, 0, sizeof(*t));
        int32_t room = 65536; /* `remain` */
        int nsym = 0;
        for (int L = 1; L <= 16; ++L) {
            if (!cnt[L]) continue;
            if (d->seg < cnt[L]) { d->status = OR_SYNTAX_ERROR; return; }
            room -= cnt[L] << (16 - L);
            if (room < 0) { d->status = OR_SYNTAX_ERROR; return; }
            for (int i = 0; i < cnt[L]; ++i) t->symbol[nsym + i] = d->at[i];
            nsym += cnt[L];
            t->count[L] = cnt[L];
            cur_skip(d, cnt[L]);
        }
        /* bounds of the sequential left-justified fill */
        u32 edge = 0;
        int idx = 0;
        for (int L = 1; L <= 16; ++L) {
            t->first[L] = idx;
            edge += (u32)t->count[L] << (16 - L);
            idx += t->count[L];
            t->bound[L] = edge;
        }
    }
    if (d->seg) d->status = OR_SYNTAX_ERROR;
}

/* ---- DQT (jpeg_dec.h:618-633) ---- */
static void read_dqt(or_ctx* d) {
    seg_open(d);
    if (d->status) return;
    while (d->seg >= 65) {
        int id = d->at[0];
        if (id & 0xFC) { d->status = OR_SYNTAX_ERROR; return; }
        memcpy(d->q[id], d->at + 1, 64);
        cur_skip(d, 65);
    }
    if (d->seg) d->status = OR_SYNTAX_ERROR;
}

/* ---- DRI (jpeg_dec.h:635-641) ---- */
static void read_dri(or_ctx* d) {
    seg_open(d);
    if (d->status) return;
    if (d->seg < 2) { d->status = OR_SYNTAX_ERROR; return; }
    d->restart = be16(d->at);
    cur_skip(d, d->seg);
}

/* ---- bit reader: njShowBits/njSkipBits/njGetBits/njByteAlign (jpeg_dec.h:447-498) ----
 * Past the end of data, and after FF D9, the stream reads as 0xFF bytes. FF 00 and
 * FF FF yield one FF data byte; FF Dn pushes both bytes; any other FF xx (or an FF
 * that is the final byte) flags a syntax error. */
static void bits_fill(or_ctx* d, int want) {
    while (d->nacc < want) {
        if (d->avail <= 0) {
            d->acc = (d->acc << 8) | 0xFFu;
            d->nacc += 8;
            continue;
        }
        uint8_t b = *d->at++;
        d->avail--;
        d->acc = (d->acc << 8) | b;
        d->nacc += 8;
        if (b != 0xFF) continue;
        if (!d->avail) { d->status = OR_SYNTAX_ERROR; continue; }
        uint8_t m = *d->at++;
        d->avail--;
        if (m == 0x00 || m == 0xFF) continue;
        if (m == 0xD9) { d->avail = 0; continue; }
        if ((m & 0xF8) == 0xD0) { d->acc = (d->acc << 8) | m; d->nacc += 8; }
        else d->status = OR_SYNTAX_ERROR;
    }
}
static int bits_peek(or_ctx* d, int n) {
    if (!n) return 0;
    bits_fill(d, n);
    return (int)((d->acc >> (d->nacc - n)) & ((1u << n) - 1u));
}
static void bits_drop(or_ctx* d, int n) {
    if (d->nacc < n) bits_fill(d, n);
    d->nacc -= n;
}
static int bits_take(or_ctx* d, int n) {
    int v = bits_peek(d, n);
    bits_drop(d, n);
    return v;
}

/* Huffman symbol + magnitude (njGetVLC, jpeg_dec.h:643-656). Returns 0 and sets the
 * error when the 16-bit window matches no code; *sym is then left untouched. */
static int read_vlc(or_ctx* d, const or_huff* t, int* sym) {
    u32 win = (u32)bits_peek(d, 16);
    int L = 1;
    while (L <= 16 && win >= t->bound[L]) ++L;
    if (L > 16) { d->status = OR_SYNTAX_ERROR; return 0; }
    u32 lo = L > 1 ? t->bound[L - 1] : 0u;
    int s = t->symbol[t->first[L] + (int)((win - lo) >> (16 - L))];
    bits_drop(d, L);
    if (sym) *sym = s;
    int nb = s & 15;
    if (!nb) return 0;
    int v = bits_take(d, nb);
    if (v < (1 << (nb - 1))) v = wadd(v, wadd(wshl(-1, nb), 1));
    return v;
}

/* ---- integer IDCT (jpeg_dec.h:343-442), including both zero-AC shortcuts whose
 * tests use the shifted values exactly as written ---- */
enum { C1 = 2841, C2 = 2676, C3 = 2408, C5 = 1609, C6 = 1108, C7 = 565 };

static void idct_row(i32* r) {
    i32 a4 = wshl(r[4], 11);
    if (!(a4 | r[6] | r[2] | r[1] | r[7] | r[5] | r[3])) {
        i32 v = wshl(r[0], 3);
        for (int i = 0; i < 8; ++i) r[i] = v;
        return;
    }
    i32 s0 = wadd(wshl(r[0], 11), 128), s1 = a4, s2 = r[6], s3 = r[2];
    i32 s4 = r[1], s5 = r[7], s6 = r[5], s7 = r[3], t;
    t = wmul(C7, wadd(s4, s5));
    s4 = wadd(t, wmul(C1 - C7, s4));
    s5 = wsub(t, wmul(C1 + C7, s5));
    t = wmul(C3, wadd(s6, s7));
    s6 = wsub(t, wmul(C3 - C5, s6));
    s7 = wsub(t, wmul(C3 + C5, s7));
    t = wadd(s0, s1);
    s0 = wsub(s0, s1);
    s1 = wmul(C6, wadd(s3, s2));
    s2 = wsub(s1, wmul(C2 + C6, s2));
    s3 = wadd(s1, wmul(C2 - C6, s3));
    s1 = wadd(s4, s6);
    s4 = wsub(s4, s6);
    s6 = wadd(s5, s7);
    s5 = wsub(s5, s7);
    s7 = wadd(t, s3);
    t = wsub(t, s3);
    s3 = wadd(s0, s2);
    s0 = wsub(s0, s2);
    s2 = wadd(wmul(181, wadd(s4, s5)), 128) >> 8;
    s4 = wadd(wmul(181, wsub(s4, s5)), 128) >> 8;
    r[0] = wadd(s7, s1) >> 8;
    r[1] = wadd(s3, s2) >> 8;
    r[2] = wadd(s0, s4) >> 8;
    r[3] = wadd(t, s6) >> 8;
    r[4] = wsub(t, s6) >> 8;
    r[5] = wsub(s0, s4) >> 8;
    r[6] = wsub(s3, s2) >> 8;
    r[7] = wsub(s7, s1) >> 8;
}

static void idct_col(const i32* k, uint8_t* px, int stride) {
    i32 a4 = wshl(k[32], 8);
    if (!(a4 | k[48] | k[16] | k[8] | k[56] | k[40] | k[24])) {
        uint8_t v = clamp_u8(wadd((wadd(k[0], 32) >> 6), 128));
        for (int i = 0; i < 8; ++i) px[i * stride] = v;
        return;
    }
    i32 s0 = wadd(wshl(k[0], 8), 8192), s1 = a4, s2 = k[48], s3 = k[16];
    i32 s4 = k[8], s5 = k[56], s6 = k[40], s7 = k[24], t;
    t = wadd(wmul(C7, wadd(s4, s5)), 4);
    s4 = wadd(t, wmul(C1 - C7, s4)) >> 3;
    s5 = wsub(t, wmul(C1 + C7, s5)) >> 3;
    t = wadd(wmul(C3, wadd(s6, s7)), 4);
    s6 = wsub(t, wmul(C3 - C5, s6)) >> 3;
    s7 = wsub(t, wmul(C3 + C5, s7)) >> 3;
    t = wadd(s0, s1);
    s0 = wsub(s0, s1);
    s1 = wadd(wmul(C6, wadd(s3, s2)), 4);
    s2 = wsub(s1, wmul(C2 + C6, s2)) >> 3;
    s3 = wadd(s1, wmul(C2 - C6, s3)) >> 3;
    s1 = wadd(s4, s6);
    s4 = wsub(s4, s6);
    s6 = wadd(s5, s7);
    s5 = wsub(s5, s7);
    s7 = wadd(t, s3);
    t = wsub(t, s3);
    s3 = wadd(s0, s2);
    s0 = wsub(s0, s2);
    s2 = wadd(wmul(181, wadd(s4, s5)), 128) >> 8;
    s4 = wadd(wmul(181, wsub(s4, s5)), 128) >> 8;
    const i32 out[8] = { wadd(s7, s1), wadd(s3, s2), wadd(s0, s4), wadd(t, s6),
                         wsub(t, s6),  wsub(s0, s4), wsub(s3, s2), wsub(s7, s1) };
    for (int i = 0; i < 8; ++i) px[i * stride] = clamp_u8(wadd(out[i] >> 14, 128));
}

/* ---- one 8x8 block (njDecodeBlock, jpeg_dec.h:658-676) ---- */
static void decode_block(or_ctx* d, or_comp* c, uint8_t* px) {
    i32 k[64];
    memset(k, 0, sizeof(k));
    const uint8_t* q = d->q[c->tq];
    int16_t* tc = NULL;
    if (d->trace && d->trace->nblocks < d->trace->cap_blocks) {
        tc = d->trace->coef + (int64_t)d->trace->nblocks * 64;
        memset(tc, 0, 64 * sizeof(int16_t));
    }
    c->pred = wadd(c->pred, read_vlc(d, &d->huff[c->dc_tab], NULL));
    k[0] = wmul(c->pred, q[0]);
    if (tc) d->trace->dc[d->trace->nblocks] = c->pred;
    int sym = 0, pos = 0;
    do {
        int v = read_vlc(d, &d->huff[c->ac_tab], &sym);
        if (!sym) break; /* EOB */
        if (!(sym & 0x0F) && sym != 0xF0) { d->status = OR_SYNTAX_ERROR; goto done; }
        pos += (sym >> 4) + 1;
        if (pos > 63) { d->status = OR_SYNTAX_ERROR; goto done; }
        k[kDezigzag[pos]] = wmul(v, q[pos]);
        if (tc) tc[kDezigzag[pos]] = (int16_t)v;
    } while (pos < 63);
    for (int r = 0; r < 64; r += 8) idct_row(&k[r]);
    for (int x = 0; x < 8; ++x) idct_col(&k[x], px + x, c->stride);
done:
    if (tc) d->trace->nblocks++;
}

/* ---- SOS + entropy-coded segment (njDecodeScan, jpeg_dec.h:678-718) ---- */
static void read_scan(or_ctx* d) {
    seg_open(d);
    if (d->status) return;
    if (d->seg < 4 + 2 * d->nc) { d->status = OR_SYNTAX_ERROR; return; }
    if (d->at[0] != d->nc) { d->status = OR_UNSUPPORTED; return; }
    cur_skip(d, 1);
    for (int i = 0; i < d->nc; ++i) {
        or_comp* c = &d->c[i];
        if (d->at[0] != c->id) { d->status = OR_SYNTAX_ERROR; return; }
        if (d->at[1] & 0xEE) { d->status = OR_SYNTAX_ERROR; return; }
        c->dc_tab = d->at[1] >> 4;
        c->ac_tab = (d->at[1] & 1) | 2;
        cur_skip(d, 2);
    }
    if (d->at[0] || d->at[1] != 63 || d->at[2]) { d->status = OR_UNSUPPORTED; return; }
    cur_skip(d, d->seg);
    int left = d->restart, expect = 0;
    for (int my = 0; my < d->mbh || (d->mbh == 0 && my == 0); ++my) {
        for (int mx = 0; mx < d->mbw || (d->mbw == 0 && mx == 0); ++mx) {
            for (int i = 0; i < d->nc; ++i) {
                or_comp* c = &d->c[i];
                for (int by = 0; by < c->vs; ++by)
                    for (int bx = 0; bx < c->hs; ++bx) {
                        int64_t off = ((int64_t)(my * c->vs + by) * c->stride + mx * c->hs + bx) << 3;
                        decode_block(d, c, c->plane + off);
                        if (d->status) return;
                    }
            }
            int last = (mx + 1 >= d->mbw) && (my + 1 >= d->mbh);
            if (last) goto finished;
            if (d->restart && !(--left)) {
                d->nacc &= 0xF8;
                int m = bits_take(d, 16);
                if ((m & 0xFFF8) != 0xFFD0 || (m & 7) != expect) { d->status = OR_SYNTAX_ERROR; return; }
                expect = (expect + 1) & 7;
                left = d->restart;
                for (int i = 0; i < 3; ++i) d->c[i].pred = 0;
            }
        }
    }
finished:
    d->status = OR_FINISHED;
}

/* ---- bicubic chroma doubling (jpeg_dec.h:720-791) ---- */
static inline uint8_t cf(i32 x) { return clamp_u8(wadd(x, 64) >> 7); }
static inline uint8_t tap2(int a, int b) { return cf(139 * a - 11 * b); }
static inline uint8_t tap3x(int a, int b, int c) { return cf(104 * a + 27 * b - 3 * c); }
static inline uint8_t tap3a(int a, int b, int c) { return cf(28 * a + 109 * b - 9 * c); }
static inline uint8_t tap4(int a, int b, int c, int e) { return cf(-9 * a + 111 * b + 29 * c - 3 * e); }

static void double_width(or_ctx* d, or_comp* c) {
    const int w = c->w, ow = w << 1;
    uint8_t* out = (uint8_t*)malloc((size_t)ow * c->h);
    if (!out) { d->status = OR_OUT_OF_MEM; return; }
    for (int y = 0; y < c->h; ++y) {
        const uint8_t* s = c->plane + (int64_t)y * c->stride;
        uint8_t* o = out + (int64_t)y * ow;
        o[0] = tap2(s[0], s[1]);
        o[1] = tap3x(s[0], s[1], s[2]);
        o[2] = tap3a(s[0], s[1], s[2]);
        for (int x = 0; x < w - 3; ++x) {
            o[2 * x + 3] = tap4(s[x], s[x + 1], s[x + 2], s[x + 3]);
            o[2 * x + 4] = tap4(s[x + 3], s[x + 2], s[x + 1], s[x]);
        }
        /* right edge taps come from the END OF THE STRIDE, not of the width (:752-756) */
        const uint8_t* e = s + c->stride;
        o[ow - 3] = tap3a(e[-1], e[-2], e[-3]);
        o[ow - 2] = tap3x(e[-1], e[-2], e[-3]);
        o[ow - 1] = tap2(e[-1], e[-2]);
    }
    free(c->plane);
    c->plane = out;
    c->w = ow;
    c->stride = ow;
}

static void double_height(or_ctx* d, or_comp* c) {
    const int w = c->w, h = c->h, s = c->stride;
    uint8_t* out = (uint8_t*)malloc((size_t)w * h * 2);
    if (!out) { d->status = OR_OUT_OF_MEM; return; }
    for (int x = 0; x < w; ++x) {
        const uint8_t* col = c->plane + x;
        uint8_t* o = out + x;
#define ROW(r) col[(int64_t)(r) * s]
        o[0] = tap2(ROW(0), ROW(1));
        o[(int64_t)w] = tap3x(ROW(0), ROW(1), ROW(2));
        o[(int64_t)2 * w] = tap3a(ROW(0), ROW(1), ROW(2));
        for (int r = 1; r <= h - 3; ++r) {
            o[(int64_t)(2 * r + 1) * w] = tap4(ROW(r - 1), ROW(r), ROW(r + 1), ROW(r + 2));
            o[(int64_t)(2 * r + 2) * w] = tap4(ROW(r + 2), ROW(r + 1), ROW(r), ROW(r - 1));
        }
        o[(int64_t)(2 * h - 3) * w] = tap3a(ROW(h - 1), ROW(h - 2), ROW(h - 3));
        o[(int64_t)(2 * h - 2) * w] = tap3x(ROW(h - 1), ROW(h - 2), ROW(h - 3));
        o[(int64_t)(2 * h - 1) * w] = tap2(ROW(h - 1), ROW(h - 2));
#undef ROW
    }
    free(c->plane);
    c->plane = out;
    c->h = h << 1;
    c->stride = w;
}

/* ---- upsample to full size, then colour convert (njConvert, jpeg_dec.h:817-866) ---- */
static void finish_image(or_ctx* d) {
    for (int i = 0; i < d->nc; ++i) {
        or_comp* c = &d->c[i];
        while (c->w < d->W || c->h < d->H) {
            if (c->w < d->W) double_width(d, c);
            if (d->status) return;
            if (c->h < d->H) double_height(d, c);
            if (d->status) return;
        }
        if (c->w < d->W || c->h < d->H) { d->status = OR_INTERNAL_ERR; return; }
    }
    if (d->nc == 3) {
        uint8_t* o = d->rgb;
        for (int y = 0; y < d->H; ++y) {
            const uint8_t* py = d->c[0].plane + (int64_t)y * d->c[0].stride;
            const uint8_t* pb = d->c[1].plane + (int64_t)y * d->c[1].stride;
            const uint8_t* pr = d->c[2].plane + (int64_t)y * d->c[2].stride;
            for (int x = 0; x < d->W; ++x) {
                i32 Y = py[x] << 8, cb = pb[x] - 128, cr = pr[x] - 128;
                *o++ = clamp_u8((Y + 359 * cr + 128) >> 8);
                *o++ = clamp_u8((Y - 88 * cb - 183 * cr + 128) >> 8);
                *o++ = clamp_u8((Y + 454 * cb + 128) >> 8);
            }
        }
    }
    /* gray: stride removal happens when copying out (jpeg_dec.h:854-865) */
}

static void ctx_release(or_ctx* d) {
    for (int i = 0; i < 3; ++i) free(d->c[i].plane);
    free(d->rgb);
}

int or_nj_decode(const uint8_t* jpeg, int64_t size, uint8_t** out, int* w, int* h, int* ncomp,
                 or_trace* trace) {
    *out = NULL;
    *w = *h = *ncomp = 0;
    or_ctx* d = (or_ctx*)calloc(1, sizeof(or_ctx));
    if (!d) return OR_OUT_OF_MEM;
    d->trace = trace;
    if (trace) trace->nblocks = 0;
    d->at = jpeg;
    d->avail = (int)(size & 0x7FFFFFFF);
    int rc;
    if (d->avail < 2 || jpeg[0] != 0xFF || jpeg[1] != 0xD8) { rc = OR_NO_JPEG; goto out; }
    cur_skip(d, 2);
    while (!d->status) {
        if (d->avail < 2 || d->at[0] != 0xFF) { rc = OR_SYNTAX_ERROR; goto out; }
        cur_skip(d, 2);
        int m = d->at[-1];
        if (m == 0xC0) read_sof(d);
        else if (m == 0xC4) read_dht(d);
        else if (m == 0xDB) read_dqt(d);
        else if (m == 0xDD) read_dri(d);
        else if (m == 0xDA) read_scan(d);
        else if (m == 0xFE || (m & 0xF0) == 0xE0) seg_skip_whole(d);
        else { rc = OR_UNSUPPORTED; goto out; }
    }
    if (d->status != OR_FINISHED) { rc = d->status; goto out; }
    d->status = OR_OK;
    finish_image(d);
    rc = d->status;
    if (rc == OR_OK) {
        *w = d->W;
        *h = d->H;
        *ncomp = d->nc == 1 ? 1 : 3; /* observable via njIsColor (jpeg_dec.h:912) */
        int64_t n = (int64_t)d->W * d->H * d->nc; /* njGetImageSize (jpeg_dec.h:914) */
        if (n > 0) {
            uint8_t* buf = (uint8_t*)malloc((size_t)n);
            if (!buf) { rc = OR_OUT_OF_MEM; goto out; }
            if (d->nc == 3) memcpy(buf, d->rgb, (size_t)n);
            else
                for (int y = 0; y < d->H; ++y)
                    memcpy(buf + (int64_t)y * d->W, d->c[0].plane + (int64_t)y * d->c[0].stride, (size_t)d->W);
            *out = buf;
        }
    }
out:
    ctx_release(d);
    free(d);
    return rc;
}

void or_free(void* p) { free(p); }
