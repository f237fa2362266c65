"""OpenEXR writer for test fixtures (single part, scanline or tiled with one level, mipmap or ripmap
levels; NONE / RLE / ZIPS / ZIP / PIZ compression; HALF / FLOAT / UINT channels). TEST
INFRASTRUCTURE: it makes the inputs the EXR tests decode -- no EXR library is importable here, so
the files are written from the format as tinyexr reads it (/root/reference/tinyexr.h: header
attributes :4441-4801, offset table :6077-6169, scanline chunks :5412-5496, tiles and levels
:4950-5161, :5616-5802, RLE / ZIP byte transforms :1424-1760, PIZ as CompressPiz :3109-3226 writes
it: range LUT :3045-3099, wavelet wav2Encode :1885-1989, Huffman hufCompress :2949-2977).

Knobs for corrupt variants (`raw_chunks`, `offsets`, attribute overrides) let the tests build
files that tinyexr rejects at each check."""
import struct
import zlib

import numpy as np

UINT, HALF, FLOAT = 0, 1, 2
NONE, RLE, ZIPS, ZIP, PIZ = 0, 1, 2, 3, 4
LINES = {NONE: 1, RLE: 1, ZIPS: 1, ZIP: 16, PIZ: 32}
_DT = {UINT: "<u4", HALF: "<f2", FLOAT: "<f4"}


def pixel_type(a):
    a = np.asarray(a)
    if a.dtype == np.float16:
        return HALF
    if a.dtype == np.float32:
        return FLOAT
    if a.dtype == np.uint32:
        return UINT
    raise ValueError(a.dtype)


def attr(name, typ, value: bytes) -> bytes:
    return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(value)) + value


def chlist(chans) -> bytes:
    out = b""
    for name, pt in chans:
        out += name.encode() + b"\0" + struct.pack("<iB3xii", pt, 0, 1, 1)
    return out + b"\0"


def rle_compress(raw: bytes) -> bytes:
    """OpenEXR's rleCompress (tinyexr.h:1537-1581)."""
    out = bytearray()
    n = len(raw)
    rs, re_ = 0, 1
    while rs < n:
        while re_ < n and raw[rs] == raw[re_] and re_ - rs - 1 < 127:
            re_ += 1
        if re_ - rs >= 3:
            out.append((re_ - rs - 1) & 0xFF)
            out.append(raw[rs])
            rs = re_
        else:
            while (re_ < n and ((re_ + 1 >= n or raw[re_] != raw[re_ + 1]) or (re_ + 2 >= n or raw[re_ + 1] != raw[re_ + 2]))
                   and re_ - rs < 127):
                re_ += 1
            out.append((rs - re_) & 0xFF)
            out += raw[rs:re_]
            rs = re_
        re_ += 1
    return bytes(out)


def _split_predict(raw: bytes) -> bytes:
    """The encode side of the RLE / ZIP byte transform: even bytes then odd bytes, then deltas."""
    a = np.frombuffer(raw, np.uint8)
    t = np.concatenate([a[0::2], a[1::2]]).astype(np.int32)
    d = t.copy()
    d[1:] = (t[1:] - t[:-1] + 128 + 256) & 0xFF
    return d.astype(np.uint8).tobytes()


# ------------------------------------------------------------------------------------------ PIZ
def _wenc14(a, b):
    as_ = (a.astype(np.int32) ^ 0x8000) - 0x8000
    bs = (b.astype(np.int32) ^ 0x8000) - 0x8000
    ms = (as_ + bs) >> 1
    ds = as_ - bs
    return (ms & 0xFFFF).astype(np.uint16), (ds & 0xFFFF).astype(np.uint16)


def _wenc16(a, b):
    ao = (a.astype(np.int32) + 32768) & 0xFFFF
    b = b.astype(np.int32)
    m = (ao + b) >> 1
    d = ao - b
    m = np.where(d < 0, (m + 32768) & 0xFFFF, m)
    return m.astype(np.uint16), (d & 0xFFFF).astype(np.uint16)


def wav2_encode(buf, j, nx, ox, ny, oy, mx):
    """wav2Encode (tinyexr.h:1885-1989) in place, one vector op per level part (disjoint groups)."""
    wenc = _wenc14 if mx < (1 << 14) else _wenc16
    n = min(nx, ny)
    p, p2 = 1, 2
    while p2 <= n:
        K, J = nx // p2, ny // p2
        xs = np.arange(K) * (ox * p2)
        ys = np.arange(J) * (oy * p2)
        if K and J:
            b = (j + ys[:, None] + xs[None, :]).ravel()
            p01, p10 = b + ox * p, b + oy * p
            p11 = p10 + ox * p
            i00, i01 = wenc(buf[b], buf[p01])
            i10, i11 = wenc(buf[p10], buf[p11])
            buf[b], buf[p10] = wenc(i00, i10)
            buf[p01], buf[p11] = wenc(i01, i11)
        if nx & p and J:
            b = j + ys + K * ox * p2
            i00, buf[b + oy * p] = wenc(buf[b], buf[b + oy * p])
            buf[b] = i00
        if ny & p and K:
            b = j + J * oy * p2 + xs
            i00, buf[b + ox * p] = wenc(buf[b], buf[b + ox * p])
            buf[b] = i00
        p = p2
        p2 <<= 1


def _huf_lengths(freq):
    """Huffman code lengths for the symbols with freq > 0 (a heap merge; tinyexr's
    hufBuildEncTable differs only in tie-breaking, which changes codes, not validity)."""
    import heapq
    syms = [i for i in np.nonzero(freq)[0]]
    lengths = {int(i): 0 for i in syms}
    if len(syms) == 1:
        lengths[int(syms[0])] = 1
        return lengths
    heap = [(int(freq[i]), k, [int(i)]) for k, i in enumerate(syms)]
    heapq.heapify(heap)
    k = len(heap)
    while len(heap) > 1:
        f1, _, a = heapq.heappop(heap)
        f2, _, b = heapq.heappop(heap)
        for x in a + b:
            lengths[x] += 1
        heapq.heappush(heap, (f1 + f2, k, a + b))
        k += 1
    assert max(lengths.values()) <= 58
    return lengths


def huf_compress(raw):
    """hufCompress (tinyexr.h:2949-2977): 20-byte header {im, iM, table length, nBits, 0}, the
    packed code-length table (hufPackEncTable :2420-2460), the codes (hufEncode :2679-2721, runs of
    a symbol as symbol + run code + 8-bit count when shorter, sendCode :2656-2673)."""
    raw = np.asarray(raw, np.uint16)
    if raw.size == 0:
        return b""
    freq = np.bincount(raw, minlength=65537).astype(np.int64)
    im = int(np.nonzero(freq)[0][0])
    iM = int(np.nonzero(freq)[0][-1]) + 1  # the run-length pseudo-symbol
    freq[iM] = 1
    lens = _huf_lengths(freq)
    hcode = [0] * 65537  # (a list: the loops below walk up to 64 Ki entries per chunk)
    for sym, ln in lens.items():
        hcode[sym] = ln
    # hufCanonicalCodeTable (:2181-2220)
    n = [0] * 59
    for ln in hcode[im:iM + 1]:
        n[int(ln)] += 1
    n[0] += 65537 - (iM + 1 - im)
    c = 0
    for i in range(58, 0, -1):
        nc = (c + n[i]) >> 1
        n[i] = c
        c = nc
    codes = {}
    for sym in range(im, iM + 1):
        ln = int(hcode[sym])
        if ln:
            codes[sym] = (n[ln], ln)
            n[ln] += 1
    # table
    acc, nb, out = 0, 0, bytearray()

    def put(nbits, v):
        nonlocal acc, nb
        acc = (acc << nbits) | v
        nb += nbits
        while nb >= 8:
            nb -= 8
            out.append((acc >> nb) & 0xFF)
        acc &= (1 << nb) - 1

    sym = im
    while sym <= iM:
        ln = int(hcode[sym])
        if ln == 0:
            run = 1
            while sym < iM and run < 255 + 6 and hcode[sym + 1] == 0:
                sym += 1
                run += 1
            if run >= 2:
                if run >= 6:
                    put(6, 63)
                    put(8, run - 6)
                else:
                    put(6, 59 + run - 2)
                sym += 1
                continue
        put(6, ln)
        sym += 1
    if nb:
        out.append((acc << (8 - nb)) & 0xFF)
    table = bytes(out)
    # codes
    acc, nb, out = 0, 0, bytearray()
    total = 0
    rlc = codes[iM]

    def send(s, cs):
        nonlocal total
        code, ln = codes[s]
        if ln + rlc[1] + 8 < ln * cs:
            put(ln, code)
            put(rlc[1], rlc[0])
            put(8, cs)
            total += ln + rlc[1] + 8
        else:
            for _ in range(cs + 1):
                put(ln, code)
            total += ln * (cs + 1)

    vals = raw.tolist()
    s, cs = vals[0], 0
    for v in vals[1:]:
        if v == s and cs < 255:
            cs += 1
        else:
            send(s, cs)
            cs = 0
        s = v
    send(s, cs)
    if nb:
        out.append((acc << (8 - nb)) & 0xFF)
    return struct.pack("<IIIII", im, iM, len(table), total, 0) + table + bytes(out)


def piz_compress(raw: bytes, chans, width, lines) -> bytes:
    """CompressPiz (tinyexr.h:3109-3226) of one chunk's pixel bytes (line-interleaved)."""
    us = np.frombuffer(raw, np.uint16)
    sizes = [1 if pt == HALF else 2 for _, pt in chans]
    planes, o = [[] for _ in chans], 0
    for _ in range(lines):
        for c, sz in enumerate(sizes):
            planes[c].append(us[o:o + width * sz])
            o += width * sz
    tmp = np.concatenate([np.concatenate(p) if p else np.zeros(0, np.uint16) for p in planes]).astype(np.uint16)
    bitmap = np.zeros(8192, np.uint8)
    np.bitwise_or.at(bitmap, tmp >> 3, (1 << (tmp & 7)).astype(np.uint8))
    bitmap[0] &= 0xFE
    nz = np.nonzero(bitmap)[0]
    mn, mx = (int(nz[0]), int(nz[-1])) if len(nz) else (8191, 0)
    bits = np.unpackbits(bitmap, bitorder="little").astype(bool)
    bits[0] = True
    lut = np.zeros(65536, np.uint16)
    lut[bits] = np.arange(int(bits.sum()), dtype=np.uint16)
    max_value = int(bits.sum()) - 1
    tmp = lut[tmp]
    st = 0
    for sz in sizes:
        for j in range(sz):
            wav2_encode(tmp, st + j, width, sz, lines, width * sz, max_value)
        st += width * lines * sz
    out = struct.pack("<HH", mn, mx)
    if mn <= mx:
        out += bitmap[mn:mx + 1].tobytes()
    h = huf_compress(tmp)
    out += struct.pack("<i", len(h)) + h
    return raw if len(out) >= len(raw) else out  # (Issue 40)


def compress(raw: bytes, comp: int, chans=None, width=0, lines=0) -> bytes:
    if comp == NONE:
        return raw
    if comp == PIZ:
        return piz_compress(raw, chans, width, lines)
    if comp == RLE:
        c = rle_compress(_split_predict(raw))
    elif comp in (ZIP, ZIPS):
        c = zlib.compress(_split_predict(raw), 6)
    else:
        raise ValueError(comp)
    return raw if len(c) >= len(raw) else c  # (tinyexr Issue 40: stored raw when not smaller)


def block_bytes(chans, arrays, y0, y1, x0, x1) -> bytes:
    """Pixel data of rows y0..y1-1, columns x0..x1-1: per line, per channel, the samples."""
    out = bytearray()
    for y in range(y0, y1):
        for (name, pt), a in zip(chans, arrays):
            out += np.ascontiguousarray(a[y, x0:x1]).astype(_DT[pt]).tobytes()
    return bytes(out)


def _level_size(top, level, rounding):  # LevelSize (tinyexr.h:4967-4979)
    ls = top >> level
    if rounding == 1 and (ls << level) < top:
        ls += 1
    return max(ls, 1)


def _log2(x, rounding):  # FloorLog2 / CeilLog2 (:5582-5614)
    y = r = 0
    while x > 1:
        r |= x & 1
        y += 1
        x >>= 1
    return y + (r if rounding == 1 else 0)


def levels_of(w, h, mode, rounding):
    """The (lx, ly) levels of a tiled image in offset-table order (InitTileOffsets :5758-5802)."""
    if mode == 0:
        return [(0, 0)]
    if mode == 1:
        n = _log2(max(w, h), rounding) + 1
        return [(l, l) for l in range(n)]
    nx, ny = _log2(w, rounding) + 1, _log2(h, rounding) + 1
    return [(lx, ly) for ly in range(ny) for lx in range(nx)]


def write_exr(channels, compression=ZIP, tiles=None, line_order=0, origin=(0, 0), sort=True, attrs=None,
              raw_chunks=None, offsets=None, chunk_line=None, version_flags=None, extra_attrs=b"",
              drop=(), levels=0, rounding=0):
    """channels: list of (name, HxW array) -- dtype float16 / float32 / uint32 picks the pixel type.
    tiles: None (scanline) or (tile_w, tile_h); levels: 0 one level, 1 mipmap, 2 ripmap (level
    (lx, ly) holds the image sampled every 2^lx columns / 2^ly rows, edge-padded to its size);
    rounding: 0 down, 1 up. origin: dataWindow min. raw_chunks(i, bytes) -> bytes may replace chunk
    i's payload; offsets(list) -> list may edit the offset table; chunk_line(i, y) -> y may change
    a scanline chunk's line number; drop: required attribute names to leave out."""
    if sort:
        channels = sorted(channels, key=lambda c: c[0])
    chans = [(n, pixel_type(a)) for n, a in channels]
    arrays = [np.asarray(a) for _, a in channels]
    h, w = arrays[0].shape
    x0, y0 = origin
    box = struct.pack("<iiii", x0, y0, x0 + w - 1, y0 + h - 1)
    a = {
        "channels": attr("channels", "chlist", chlist(chans)),
        "compression": attr("compression", "compression", bytes([compression])),
        "dataWindow": attr("dataWindow", "box2i", box),
        "displayWindow": attr("displayWindow", "box2i", box),
        "lineOrder": attr("lineOrder", "lineOrder", bytes([line_order])),
        "pixelAspectRatio": attr("pixelAspectRatio", "float", struct.pack("<f", 1.0)),
        "screenWindowCenter": attr("screenWindowCenter", "v2f", struct.pack("<ff", 0.0, 0.0)),
        "screenWindowWidth": attr("screenWindowWidth", "float", struct.pack("<f", 1.0)),
    }
    if tiles:
        a["tiles"] = attr("tiles", "tiledesc", struct.pack("<IIB", tiles[0], tiles[1], levels | (rounding << 4)))
    for k, v in (attrs or {}).items():
        a[k] = v
    header = b"".join(v for k, v in a.items() if k not in drop) + extra_attrs + b"\0"
    flags = version_flags if version_flags is not None else (0x2 if tiles else 0)
    head = bytes([0x76, 0x2F, 0x31, 0x01, 2, flags, 0, 0]) + header
    chunks = []
    if tiles:
        tw, th = tiles
        for lx, ly in levels_of(w, h, levels, rounding):
            lw, lh = _level_size(w, lx, rounding), _level_size(h, ly, rounding)
            la = [np.ascontiguousarray(a[::1 << ly, ::1 << lx][:lh, :lw]) for a in arrays]
            la = [np.pad(a, ((0, lh - a.shape[0]), (0, lw - a.shape[1])), mode="edge") for a in la]
            nty, ntx = -(-lh // th), -(-lw // tw)
            for ty in range(nty):
                for tx in range(ntx):
                    x1, y1 = min(lw, tx * tw + tw), min(lh, ty * th + th)
                    raw = block_bytes(chans, la, ty * th, y1, tx * tw, x1)
                    data = compress(raw, compression, chans, x1 - tx * tw, y1 - ty * th)
                    if raw_chunks:
                        data = raw_chunks(len(chunks), data)
                    chunks.append(struct.pack("<iiiii", tx, ty, lx, ly, len(data)) + data)
    else:
        n = LINES[compression]
        for k in range(-(-h // n)):
            raw = block_bytes(chans, arrays, k * n, min(h, k * n + n), 0, w)
            data = compress(raw, compression, chans, w, min(h, k * n + n) - k * n)
            if raw_chunks:
                data = raw_chunks(k, data)
            yl = y0 + k * n
            if chunk_line:
                yl = chunk_line(k, yl)
            chunks.append(struct.pack("<ii", yl, len(data)) + data)
    base = len(head) + 8 * len(chunks)
    offs, pos = [], base
    order = list(range(len(chunks)))
    if line_order == 1 and not tiles:
        order = order[::-1]  # DECREASING_Y: chunks stored bottom-up, the table stays by chunk index
    placed = {}
    for k in order:
        placed[k] = pos
        pos += len(chunks[k])
    offs = [placed[k] for k in range(len(chunks))]
    if offsets:
        offs = offsets(offs)
    body = b"".join(chunks[k] for k in order)
    return head + b"".join(struct.pack("<Q", o) for o in offs) + body
