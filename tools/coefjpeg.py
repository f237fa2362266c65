"""Baseline JPEG writer from quantized coefficients (test-fixture tool, not product, not oracle).

PIL/libjpeg-turbo writes only what a real DCT of real pixels produces. Some decoder paths are
only reached by streams no pixel encoder emits, yet NanoJPEG decodes them deterministically
(jpeg_dec.h:658-676 does not bound coefficients): dequantized AC values in the thousands (the
IDCT's 32-bit corners), Huffman tables with 13-16-bit codes in the hot loop, or tables whose
long codes overflow the decoder's second-level pool. This module writes such streams from
coefficient arrays: SOI, DQT, SOF0, DHT, [DRI], SOS, the entropy-coded segment with FF00
stuffing and RSTn markers, EOI (ITU T.81 Annex B/F; the layout NanoJPEG parses,
jpeg_dec.h:523-718).

    write(w, h, comps, qt, blocks, huff="std"|"optimal"|dict, restart=0) -> bytes

comps: [(hs, vs, tq), ...] (1 or 3); qt: {id: 64 values in zig-zag order}; blocks: per
component an int array [by, bx, 64] of quantized coefficients in zig-zag order, covering the
MCU-padded component (by = mbh * vs, bx = mbw * hs). DC entries are absolute (the writer codes
differences, predictors reset at each restart).
"""
from __future__ import annotations

import numpy as np

# Annex K.3 standard tables (bits[1..16], values)
STD_DC_L = ([0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0], list(range(12)))
STD_DC_C = ([0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0], list(range(12)))
STD_AC_L = ([0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7D], [
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07,
    0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xA1, 0x08, 0x23, 0x42, 0xB1, 0xC1, 0x15, 0x52, 0xD1, 0xF0,
    0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0A, 0x16, 0x17, 0x18, 0x19, 0x1A, 0x25, 0x26, 0x27, 0x28,
    0x29, 0x2A, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3A, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49,
    0x4A, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5A, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69,
    0x6A, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7A, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89,
    0x8A, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9A, 0xA2, 0xA3, 0xA4, 0xA5, 0xA6, 0xA7,
    0xA8, 0xA9, 0xAA, 0xB2, 0xB3, 0xB4, 0xB5, 0xB6, 0xB7, 0xB8, 0xB9, 0xBA, 0xC2, 0xC3, 0xC4, 0xC5,
    0xC6, 0xC7, 0xC8, 0xC9, 0xCA, 0xD2, 0xD3, 0xD4, 0xD5, 0xD6, 0xD7, 0xD8, 0xD9, 0xDA, 0xE1, 0xE2,
    0xE3, 0xE4, 0xE5, 0xE6, 0xE7, 0xE8, 0xE9, 0xEA, 0xF1, 0xF2, 0xF3, 0xF4, 0xF5, 0xF6, 0xF7, 0xF8,
    0xF9, 0xFA])
STD_AC_C = ([0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77], [
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71,
    0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xA1, 0xB1, 0xC1, 0x09, 0x23, 0x33, 0x52, 0xF0,
    0x15, 0x62, 0x72, 0xD1, 0x0A, 0x16, 0x24, 0x34, 0xE1, 0x25, 0xF1, 0x17, 0x18, 0x19, 0x1A, 0x26,
    0x27, 0x28, 0x29, 0x2A, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3A, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48,
    0x49, 0x4A, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5A, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68,
    0x69, 0x6A, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7A, 0x82, 0x83, 0x84, 0x85, 0x86, 0x87,
    0x88, 0x89, 0x8A, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9A, 0xA2, 0xA3, 0xA4, 0xA5,
    0xA6, 0xA7, 0xA8, 0xA9, 0xAA, 0xB2, 0xB3, 0xB4, 0xB5, 0xB6, 0xB7, 0xB8, 0xB9, 0xBA, 0xC2, 0xC3,
    0xC4, 0xC5, 0xC6, 0xC7, 0xC8, 0xC9, 0xCA, 0xD2, 0xD3, 0xD4, 0xD5, 0xD6, 0xD7, 0xD8, 0xD9, 0xDA,
    0xE2, 0xE3, 0xE4, 0xE5, 0xE6, 0xE7, 0xE8, 0xE9, 0xEA, 0xF2, 0xF3, 0xF4, 0xF5, 0xF6, 0xF7, 0xF8,
    0xF9, 0xFA])


def _category(v: int) -> int:
    return int(abs(int(v))).bit_length()


def _codes(bits, vals):
    """Canonical code table (Annex C): symbol -> (code, length)."""
    out, code, k = {}, 0, 0
    for L in range(1, 17):
        for _ in range(bits[L - 1]):
            out[vals[k]] = (code, L)
            code += 1
            k += 1
        code <<= 1
    return out


def optimal_table(freq: dict) -> tuple[list, list]:
    """Length-limited (16-bit) Huffman table from symbol frequencies (Annex K.2, the procedure
    libjpeg's jpeg_gen_optimal_table follows; one reserved all-ones codeword)."""
    f = [0] * 257
    for s, c in freq.items():
        f[s] = int(c)
    f[256] = 1  # reserved: no code of all 1 bits
    codesize = [0] * 257
    others = [-1] * 257
    while True:
        c1, v = -1, 1 << 62
        for i in range(257):
            if f[i] and f[i] <= v:
                v, c1 = f[i], i
        c2, v = -1, 1 << 62
        for i in range(257):
            if f[i] and f[i] <= v and i != c1:
                v, c2 = f[i], i
        if c2 < 0:
            break
        f[c1] += f[c2]
        f[c2] = 0
        codesize[c1] += 1
        while others[c1] >= 0:
            c1 = others[c1]
            codesize[c1] += 1
        others[c1] = c2
        codesize[c2] += 1
        while others[c2] >= 0:
            c2 = others[c2]
            codesize[c2] += 1
    bits = [0] * 33
    for i in range(257):
        if codesize[i]:
            bits[codesize[i]] += 1
    for i in range(32, 16, -1):  # limit to 16 bits (K.3)
        while bits[i] > 0:
            j = i - 2
            while bits[j] == 0:
                j -= 1
            bits[i] -= 2
            bits[i - 1] += 1
            bits[j + 1] += 2
            bits[j] -= 1
    i = 16
    while bits[i] == 0:
        i -= 1
    bits[i] -= 1  # drop the reserved code
    vals = [s for L in range(1, 33) for s in range(256) if codesize[s] == L]
    return bits[1:17], vals


def skewed_table(symbols: list, short: int = 2) -> tuple[list, list]:
    """A valid table whose first `short` symbols get short codes and all others 15-16-bit codes
    (the decoder's long-code paths in the hot loop)."""
    n = len(symbols)
    bits = [0] * 16
    for k in range(min(short, n)):
        bits[k + 1] += 1  # lengths 2, 3, ...
    rest = n - min(short, n)
    # the remaining prefix space below 2^-(short+1) is split into 15- and 16-bit codes
    n15 = min(rest // 2, (1 << (15 - short - 1)) - 1)
    bits[14] += n15
    bits[15] += rest - n15
    return bits, list(symbols)


class _Bits:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, code: int, length: int):
        if length == 0:
            return
        self.acc = (self.acc << length) | (code & ((1 << length) - 1))
        self.n += length
        while self.n >= 8:
            self.n -= 8
            b = (self.acc >> self.n) & 0xFF
            self.out.append(b)
            if b == 0xFF:
                self.out.append(0)
        self.acc &= (1 << self.n) - 1

    def flush(self):  # pad with 1-bits (Annex F.1.2.3)
        if self.n:
            self.put((1 << (8 - self.n)) - 1, 8 - self.n)


def _mcu_blocks(comps, mbw, mbh):
    """NanoJPEG's block order (jpeg_dec.h:696-702): per MCU, per component, sby, sbx."""
    for my in range(mbh):
        for mx in range(mbw):
            for ci, (hs, vs, _) in enumerate(comps):
                for sby in range(vs):
                    for sbx in range(hs):
                        yield my * mbw + mx, ci, my * vs + sby, mx * hs + sbx


def _block_symbols(zz, pred):
    """Yield ('dc'|'ac', symbol, extra_bits, n_extra) for one block (F.1.2.1-2)."""
    d = int(zz[0]) - pred
    s = _category(d)
    yield "dc", s, (d if d >= 0 else d + (1 << s) - 1), s
    last = 0
    for k in range(63, 0, -1):
        if zz[k]:
            last = k
            break
    run = 0
    for k in range(1, last + 1):
        v = int(zz[k])
        if v == 0:
            run += 1
            continue
        while run > 15:
            yield "ac", 0xF0, 0, 0
            run -= 16
        s = _category(v)
        if s > 15:
            raise ValueError("AC magnitude beyond 15 bits")
        yield "ac", (run << 4) | s, (v if v >= 0 else v + (1 << s) - 1), s
        run = 0
    if last != 63:
        yield "ac", 0x00, 0, 0


def write(w: int, h: int, comps, qt: dict, blocks, huff="std", restart: int = 0, app0: bool = True) -> bytes:
    nc = len(comps)
    hmax = max(c[0] for c in comps)
    vmax = max(c[1] for c in comps)
    mbw = (w + 8 * hmax - 1) // (8 * hmax)
    mbh = (h + 8 * vmax - 1) // (8 * vmax)
    for ci, (hs, vs, _) in enumerate(comps):
        assert blocks[ci].shape == (mbh * vs, mbw * hs, 64), (blocks[ci].shape, mbh * vs, mbw * hs)
    # table id per component: 0 luma, 1 chroma (Annex K convention)
    tid = [0 if ci == 0 else 1 for ci in range(nc)]
    ntab = 2 if nc > 1 else 1
    seq = list(_mcu_blocks(comps, mbw, mbh))
    if isinstance(huff, dict):
        tabs = huff
    elif huff == "std":
        tabs = {("dc", 0): STD_DC_L, ("ac", 0): STD_AC_L, ("dc", 1): STD_DC_C, ("ac", 1): STD_AC_C}
    elif huff == "optimal":
        freq = {}
        pred = [0] * nc
        lastm = -1
        for m, ci, by, bx in seq:
            if restart and m != lastm and m % restart == 0:
                pred = [0] * nc
            lastm = m
            zz = blocks[ci][by, bx]
            for kind, sym, _, _ in _block_symbols(zz, pred[ci]):
                fr = freq.setdefault((kind, tid[ci]), {})
                fr[sym] = fr.get(sym, 0) + 1
            pred[ci] = int(zz[0])
        tabs = {k: optimal_table(v) for k, v in freq.items()}
    else:
        raise ValueError(huff)
    codes = {k: _codes(*v) for k, v in tabs.items()}

    o = bytearray(b"\xff\xd8")
    if app0:
        o += b"\xff\xe0\x00\x10JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00"
    for q, tab in sorted(qt.items()):
        o += b"\xff\xdb\x00\x43" + bytes([q]) + bytes(int(x) for x in tab)
    o += b"\xff\xc0" + (8 + 3 * nc).to_bytes(2, "big") + b"\x08" + h.to_bytes(2, "big") + w.to_bytes(2, "big")
    o += bytes([nc])
    for ci, (hs, vs, tq) in enumerate(comps):
        o += bytes([ci + 1, (hs << 4) | vs, tq])
    for (kind, t), (bits, vals) in sorted(tabs.items()):
        body = bytes([(0 if kind == "dc" else 0x10) | t]) + bytes(bits) + bytes(vals)
        o += b"\xff\xc4" + (2 + len(body)).to_bytes(2, "big") + body
    if restart:
        o += b"\xff\xdd\x00\x04" + restart.to_bytes(2, "big")
    o += b"\xff\xda" + (6 + 2 * nc).to_bytes(2, "big") + bytes([nc])
    for ci in range(nc):
        o += bytes([ci + 1, (tid[ci] << 4) | tid[ci]])
    o += b"\x00\x3f\x00"
    bw = _Bits()
    pred = [0] * nc
    lastm = -1
    rst = 0
    for m, ci, by, bx in seq:
        if m != lastm:
            if restart and m and m % restart == 0:
                bw.flush()
                bw.out += bytes([0xFF, 0xD0 + (rst & 7)])
                rst += 1
                pred = [0] * nc
            lastm = m
        zz = blocks[ci][by, bx]
        for kind, sym, extra, n in _block_symbols(zz, pred[ci]):
            c, L = codes[(kind, tid[ci])][sym]
            bw.put(c, L)
            bw.put(extra, n)
        pred[ci] = int(zz[0])
    bw.flush()
    o += bw.out + b"\xff\xd9"
    return bytes(o)


def sampling_comps(s: str):
    return {"gray": [(1, 1, 0)], "444": [(1, 1, 0), (1, 1, 1), (1, 1, 1)], "420": [(2, 2, 0), (1, 1, 1), (1, 1, 1)],
            "422": [(2, 1, 0), (1, 1, 1), (1, 1, 1)]}[s]


def empty_blocks(w: int, h: int, comps):
    hmax = max(c[0] for c in comps)
    vmax = max(c[1] for c in comps)
    mbw = (w + 8 * hmax - 1) // (8 * hmax)
    mbh = (h + 8 * vmax - 1) // (8 * vmax)
    return [np.zeros((mbh * vs, mbw * hs, 64), np.int32) for (hs, vs, _) in comps]
