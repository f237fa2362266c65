"""TEST-ONLY oracle: a Python restatement of tinyexr's LoadEXRFromMemory (/root/reference/tinyexr.h
:6645-6860) for single-part scanline and tiled images (one level, mipmap or ripmap levels), NONE /
RLE / ZIPS / ZIP / PIZ compression. Only tests/ may import it; libicx never does.

PINNED to the reference: tinyexr.h compiles here in place through its own documented zlib route
(TINYEXR_USE_MINIZ 0 with the system <zlib.h>, tinyexr.h:109-112, 664-671; oracle/ref/ref_exr_tu.cc,
`make -C oracle ref`), and tests/test_exr_oracle.py checks this module against that build on every
fixture and on seeded damage (codes and every float the reference defines; tests/exrref.py). For
NONE / RLE / PIZ chunks and all header and offset logic the inflate library is not on the path;
ZIP / ZIPS go through zlib in both, standing in for the reference's un-vendored miniz (both are
RFC 1950 / 1951 decoders that check the Adler-32: a valid stream inflates to the same bytes). PIZ
is tinyexr's own code (its build has TINYEXR_USE_PIZ 1, :126-128, which codecs.cpp:27-29 does not
override).

What it returns where tinyexr's result is undefined or out of this build's scope (the GPU path
does the same):
* rows / tile pixels no chunk wrote are 0.0 (tinyexr: uninitialised malloc memory; the manifest
  lists them per fixture, "ref_undefined_rows", from the reference build); a NONE
  chunk whose block index lies past the image (chunkCount > lines: tinyexr writes outside its
  buffer) is a decode failure (INVALID_DATA);
* bytes a damaged PIZ chunk makes the decoder read past the end of the file are 0 (tinyexr reads
  the memory after its buffer); a tile-offset reconstruction that walks before the file fails;
* PXR24 / B44 / ZFP -> UNSUPPORTED_FORMAT; a tile size of 0 -> INVALID_DATA (tinyexr divides by
  it). The multi-part and deep version bits are NOT rejected (LoadEXRFromMemory decodes such a
  file as one part; only LoadEXR refuses them, :6268-6270): they change only how
  ReconstructTileOffsets walks the chunks.
"""
import struct
import zlib

import numpy as np

SUCCESS = 0
INVALID_MAGIC_NUMBER = -1
INVALID_EXR_VERSION = -2
INVALID_ARGUMENT = -3
INVALID_DATA = -4
UNSUPPORTED_FORMAT = -8
INVALID_HEADER = -9
UNSUPPORTED_FEATURE = -10

UINT, HALF, FLOAT = 0, 1, 2
NONE, RLE, ZIPS, ZIP, PIZ = 0, 1, 2, 3, 4
SIZE = {UINT: 4, HALF: 2, FLOAT: 4}
THRESH = 1024 * 8192  # TINYEXR_DIMENSION_THRESHOLD (:3628)
INT_MAX = 2**31 - 1


def _w32(x):  # two's-complement int32 wrap-around
    return ((x + 2**31) % 2**32) - 2**31


def _i32(b, o):
    return struct.unpack_from("<i", b, o)[0]


def parse_header(buf):
    """ParseEXRVersionFromMemory (:8927-8982) + ParseEXRHeader (:4441-4801) + ConvertHeader
    (:4804-4940). Returns (code, info dict)."""
    n = len(buf)
    if n < 8:
        return INVALID_DATA, None
    if buf[:4] != bytes([0x76, 0x2F, 0x31, 0x01]):
        return INVALID_MAGIC_NUMBER, None
    if buf[4] != 2:
        return INVALID_EXR_VERSION, None
    tiled_v = bool(buf[5] & 2)
    multipart = bool(buf[5] & 0x10)
    non_image = bool(buf[5] & 0x8)
    info = dict(channels=[], dw=(0, 0, 0, 0), line_order=0, compression=None, tiled=0, tile=(-1, -1), tile_mode=-1,
                tile_round=-1, chunk_count=0, name="", type="", multipart=multipart, non_image=non_image)
    have = set()
    p, size = 8, n - 8
    ret = SUCCESS
    for _ in range(1024):  # TINYEXR_MAX_HEADER_ATTRIBUTES
        if size == 0:
            ret = INVALID_DATA
            break
        if buf[p] == 0:
            size -= 1
            break
        # ReadAttribute (:1069-1135)
        seg = buf[p:p + size]
        z = seg.find(b"\0")
        if z < 0:
            ret = INVALID_DATA
            break
        name = seg[:z].decode("latin-1")
        rest = seg[z + 1:]
        z2 = rest.find(b"\0")
        if z2 < 0:
            ret = INVALID_DATA
            break
        typ = rest[:z2].decode("latin-1")
        rest = rest[z2 + 1:]
        if len(rest) < 4:
            ret = INVALID_DATA
            break
        dlen = struct.unpack_from("<I", rest, 0)[0]
        if dlen == 0:
            if typ != "string":
                ret = INVALID_DATA
                break
            data = b"\0"
            msize = z + 1 + z2 + 1 + 4
        else:
            if len(rest) - 4 < dlen:
                ret = INVALID_DATA
                break
            data = rest[4:4 + dlen]
            msize = z + 1 + z2 + 1 + 4 + dlen
        p += msize
        size -= msize
        if (tiled_v or multipart or non_image) and name == "tiles":
            if len(data) != 9:
                ret = INVALID_DATA
                break
            xs, ys = struct.unpack_from("<II", data, 0)
            if xs > INT_MAX or ys > INT_MAX:
                ret = UNSUPPORTED_FORMAT
                break
            info["tile"] = (xs, ys)
            info["tile_mode"] = data[8] & 3
            info["tile_round"] = (data[8] >> 4) & 1
            info["tiled"] = 1
        elif name == "compression":
            c = data[0]
            if c > PIZ:
                ret = UNSUPPORTED_FORMAT  # "Unknown compression type" / ZFP not built (:4568-4601)
                break
            info["compression"] = c
            have.add("compression")
        elif name == "channels":
            ok, chans = _read_channels(data)
            chans = info["channels"] + chans  # (ReadChannelInfo appends: :1268)
            if not ok or not chans:
                ret = INVALID_DATA
                break
            info["channels"] = chans
            have.add("channels")
        elif name in ("dataWindow", "displayWindow"):
            if len(data) >= 16:
                if name == "dataWindow":
                    info["dw"] = struct.unpack_from("<iiii", data, 0)
                have.add(name)
        elif name == "lineOrder":
            if len(data) >= 1:
                info["line_order"] = data[0]
                have.add(name)
        elif name in ("pixelAspectRatio", "screenWindowWidth"):
            if len(data) >= 4:
                have.add(name)
        elif name == "screenWindowCenter":
            if len(data) >= 8:
                have.add(name)
        elif name == "chunkCount":
            if len(data) >= 4:
                info["chunk_count"] = _i32(data, 0)
        elif name in ("name", "type"):
            if data and data[0]:
                s = data.split(b"\0")[0].decode("latin-1")
                info[name] = s
                have.add(name)
    if ret == SUCCESS:
        need = {"compression", "channels", "lineOrder", "displayWindow", "dataWindow", "pixelAspectRatio",
                "screenWindowWidth", "screenWindowCenter"}
        if multipart or non_image:
            need |= {"name", "type"}
        if need - have:
            ret = INVALID_HEADER
    # ConvertHeader's type checks run whatever ParseEXRHeader returned (:6621-6637)
    t = info["type"]
    if (t == "scanlineimage" and info["tiled"]) or (t in ("tiledimage", "deeptile") and not info["tiled"]):
        ret = INVALID_HEADER
    info["header_len"] = (n - 8) - size
    return ret, info


def _read_channels(data):
    """ReadChannelInfo (:1226-1272)."""
    chans = []
    p = 0
    while True:
        if p >= len(data):
            return False, chans  # (data.at past the end throws in tinyexr)
        if data[p] == 0:
            break
        z = data.find(b"\0", p)
        if z < 0:
            return False, chans
        name = data[p:z].decode("latin-1")
        p = z + 1
        if p + 16 >= len(data):
            return False, chans
        pt = _i32(data, p)
        chans.append((name, pt))
        p += 16
    return True, chans


def _zip(src, dst_len):
    """DecompressZip (:1424-1503): raw when the sizes are equal; else mz_uncompress, then the
    predictor and the even / odd reorder over the bytes it produced."""
    if dst_len == len(src):
        return bytes(src)
    d = zlib.decompressobj()
    try:
        t = d.decompress(bytes(src), dst_len)
    except zlib.error:
        return None
    if d.unconsumed_tail or not d.eof:  # output past dst_len (MZ_BUF_ERROR) / stream not ended
        return None
    return _unpredict(t, dst_len)


def _rle(src, dst_len):
    """DecompressRle (:1696-1760) + rleUncompress (:1589-1619)."""
    if dst_len == len(src):
        return bytes(src)
    if len(src) <= 2:
        return None
    out = bytearray()
    i, inlen, maxlen = 0, len(src), dst_len
    while inlen > 0:
        c = struct.unpack_from("b", src, i)[0]
        i += 1
        if c < 0:
            cnt = -c
            inlen -= cnt + 1
            maxlen -= cnt
            if maxlen < 0 or inlen < 0:
                return None
            out += src[i:i + cnt]
            i += cnt
        else:
            inlen -= 2
            maxlen -= c + 1
            if maxlen < 0 or inlen < 0:
                return None
            out += bytes([src[i]]) * (c + 1)
            i += 1
    if len(out) != dst_len:
        return None
    return _unpredict(bytes(out), dst_len)


def _unpredict(t, dst_len):
    a = np.frombuffer(t, np.uint8).astype(np.int64)
    if len(a):
        a = (a[0] + np.concatenate([[0], np.cumsum(a[1:] - 128)])) & 0xFF
    a = a.astype(np.uint8)
    m = len(a)
    half = (m + 1) // 2
    out = np.zeros(dst_len, np.uint8)  # (the rest of tinyexr's zero-initialised outBuf)
    out[0:m:2] = a[:half]
    out[1:m:2] = a[half:m]
    return out.tobytes()


# ---------------------------------------------------------------------------------------- PIZ
# tinyexr builds PIZ in by default (TINYEXR_USE_PIZ 1, tinyexr.h:126-128) and codecs.cpp:27-29
# does not turn it off. DecompressPiz (:3228-3375) = range-compression bitmap and LUT
# (:3042-3099), the 16-bit Huffman decoder (hufUncompress :2979-3036, hufUnpackEncTable
# :2466-2519, hufCanonicalCodeTable :2181-2220, hufBuildDecTable :2548-2632, hufDecode :2804-2920)
# and the 2D Haar wavelet (wav2Decode :1995-2109). Restated with tinyexr's quirks: hufUncompress's
# result (and so every Huffman failure) is ignored by DecompressPiz -- what was decoded before a
# failure is kept, the rest of the buffer is zeros -- and a failed table unpack leaves its raw
# code lengths in place, which the decoder then uses. Bytes past the end of the file read as 0
# (tinyexr reads whatever memory follows the buffer there; only damaged files get that far).
HUF_ENCSIZE = (1 << 16) + 1
HUF_DECBITS = 14
HUF_DECMASK = (1 << HUF_DECBITS) - 1
SHORT_ZEROCODE_RUN, LONG_ZEROCODE_RUN = 59, 63
SHORTEST_LONG_RUN = 2 + LONG_ZEROCODE_RUN - SHORT_ZEROCODE_RUN
BITMAP_SIZE = 1 << 13
M64 = (1 << 64) - 1


def _s64(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def _s32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >> 31 else x


def _cdiv(a, b):  # C integer division (toward zero)
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


class _Buf:
    """The file as tinyexr's pointers see it: bytes past its end read as 0."""

    def __init__(self, b):
        self.b = b

    def __getitem__(self, i):
        return self.b[i] if 0 <= i < len(self.b) else 0

    def u32(self, i):
        return self[i] | self[i + 1] << 8 | self[i + 2] << 16 | self[i + 3] << 24


def _huf_unpack(F, p0, ni, im, iM):
    """hufUnpackEncTable (:2466-2519): (ok, hcode, end). On failure hcode keeps the raw code
    lengths read so far (no canonical codes) and the pointer stays at p0."""
    hcode = [0] * HUF_ENCSIZE
    p, c, lc = p0, 0, 0

    def bits(n):
        nonlocal p, c, lc
        while lc < n:
            c = ((c << 8) | F[p]) & M64
            p += 1
            lc += 8
        lc -= n
        return (c >> lc) & ((1 << n) - 1)

    while im <= iM:
        if p - p0 >= ni:
            return False, hcode, p0
        ln = hcode[im] = bits(6)
        if ln == LONG_ZEROCODE_RUN:
            if p - p0 > ni:
                return False, hcode, p0
            zerun = bits(8) + SHORTEST_LONG_RUN
            if im + zerun > iM + 1:
                return False, hcode, p0
            for _ in range(zerun):
                hcode[im] = 0
                im += 1
            im -= 1
        elif ln >= SHORT_ZEROCODE_RUN:
            zerun = ln - SHORT_ZEROCODE_RUN + 2
            if im + zerun > iM + 1:
                return False, hcode, p0
            for _ in range(zerun):
                hcode[im] = 0
                im += 1
            im -= 1
        im += 1
    _huf_canonical(hcode)
    return True, hcode, p


def _huf_canonical(hcode):
    """hufCanonicalCodeTable (:2181-2220): code lengths -> length | code << 6."""
    n = [0] * 59
    for h in hcode:
        n[h] += 1
    c = 0
    for i in range(58, 0, -1):
        nc = (c + n[i]) >> 1
        n[i] = c
        c = nc
    for i, ln in enumerate(hcode):
        if ln > 0:
            hcode[i] = (ln | (n[ln] << 6)) & M64
            n[ln] += 1


def _huf_build_dec(hcode, im, iM):
    """hufBuildDecTable (:2548-2632): {entry: (len, lit)} for short codes and {entry: [symbols]}
    for long ones, as far as the build gets before its first failure (which is ignored)."""
    short, longs = {}, {}
    while im <= iM:
        h = hcode[im]
        c = _s64(h) >> 6
        ln = h & 63
        if c >> ln:
            return short, longs
        if ln > HUF_DECBITS:
            e = c >> (ln - HUF_DECBITS)
            if e in short:
                return short, longs
            longs.setdefault(e, []).append(im)
        elif ln:
            e0 = c << (HUF_DECBITS - ln)
            for e in range(e0, e0 + (1 << (HUF_DECBITS - ln))):
                if e in short or e in longs:
                    return short, longs
                short[e] = (ln, im)
        im += 1
    return short, longs


def _huf_decode(hcode, short, longs, F, p0, ni, rlc, no, out):
    """hufDecode (:2804-2920) into the list `out` (ushorts); what it wrote stays on failure."""
    c, lc, i = 0, 0, p0
    ie = p0 + _cdiv(ni + 7, 8)

    def getcode(po):
        nonlocal c, lc, i
        if po == rlc:
            if lc < 8:
                if i >= ie:
                    return False
                c = ((c << 8) | F[i]) & M64
                i += 1
                lc += 8
            lc -= 8
            cs = (_s64(c) >> lc) & 0xFF
            if len(out) + cs > no or len(out) < 1:
                return False
            out.extend([out[-1]] * cs)
        elif len(out) < no:
            out.append(po)
        else:
            return False
        return True

    while i < ie:
        c = ((c << 8) | F[i]) & M64
        i += 1
        lc += 8
        while lc >= HUF_DECBITS:
            e = (_s64(c) >> (lc - HUF_DECBITS)) & HUF_DECMASK
            if e in short:
                ln, lit = short[e]
                lc -= ln
                if not getcode(lit):
                    return False
            else:
                lst = longs.get(e)
                if not lst:
                    return False
                for sym in lst:
                    ln = hcode[sym] & 63
                    while lc < ln and i < ie:
                        c = ((c << 8) | F[i]) & M64
                        i += 1
                        lc += 8
                    if lc >= ln and (_s64(hcode[sym]) >> 6) == ((_s64(c) >> (lc - ln)) & ((1 << ln) - 1)):
                        lc -= ln
                        if not getcode(sym):
                            return False
                        break
                else:
                    return False
    k = (8 - ni) & 7
    c = _s64(c) >> k
    lc -= k
    while lc > 0:
        e = ((c << (HUF_DECBITS - lc)) & M64) & HUF_DECMASK
        if e not in short:
            return False
        ln, lit = short[e]
        lc -= ln
        if not getcode(lit):
            return False
    return len(out) == no


def _huf_uncompress(F, p0, n_comp, no):
    """hufUncompress (:2979-3036) -> the ushorts decoded (fewer than `no` on any failure)."""
    out = []
    if n_comp == 0:
        return out
    im, iM, nbits = _s32(F.u32(p0)), _s32(F.u32(p0 + 4)), _s32(F.u32(p0 + 12))
    if im < 0 or im >= HUF_ENCSIZE or iM < 0 or iM >= HUF_ENCSIZE:
        return out
    ok, hcode, p = _huf_unpack(F, p0 + 20, n_comp - 20, im, iM)
    if nbits > 8 * (n_comp - (p - p0)):
        return out
    short, longs = _huf_build_dec(hcode, im, iM)
    _huf_decode(hcode, short, longs, F, p, nbits, iM, no, out)
    return out


def _wdec14(l, h):
    ls = (l.astype(np.int32) ^ 0x8000) - 0x8000
    hs = (h.astype(np.int32) ^ 0x8000) - 0x8000
    ai = ls + (hs & 1) + (hs >> 1)
    return (ai & 0xFFFF).astype(np.uint16), ((ai - hs) & 0xFFFF).astype(np.uint16)


def _wdec16(l, h):
    m, d = l.astype(np.int32), h.astype(np.int32)
    bb = (m - (d >> 1)) & 0xFFFF
    aa = (d + bb - 32768) & 0xFFFF
    return aa.astype(np.uint16), bb.astype(np.uint16)


def wav2_decode(buf, j, nx, ox, ny, oy, mx):
    """wav2Decode (:1995-2109) in place on the uint16 array buf from index j. Within a level the
    2x2 groups, the odd column and the odd line touch disjoint samples, so each is one vector op."""
    wdec = _wdec14 if mx < (1 << 14) else _wdec16
    n = min(nx, ny)
    p = 1
    while p <= n:
        p <<= 1
    p >>= 1
    p2 = p
    p >>= 1
    while p >= 1:
        K, J = nx // p2, ny // p2  # groups per line / lines of groups (the X and Y loops)
        xs = np.arange(K) * (ox * p2)
        ys = np.arange(J) * (oy * p2)
        if K and J:
            b = (j + ys[:, None] + xs[None, :]).ravel()
            p01, p10 = b + ox * p, b + oy * p
            p11 = p10 + ox * p
            i00, i10 = wdec(buf[b], buf[p10])
            i01, i11 = wdec(buf[p01], buf[p11])
            buf[b], buf[p01] = wdec(i00, i01)
            buf[p10], buf[p11] = wdec(i10, i11)
        if nx & p and J:  # odd column (still in the Y loop)
            b = j + ys + K * ox * p2
            i00, buf[b + oy * p] = wdec(buf[b], buf[b + oy * p])
            buf[b] = i00
        if ny & p and K:  # odd line
            b = j + J * oy * p2 + xs
            i00, buf[b + ox * p] = wdec(buf[b], buf[b + ox * p])
            buf[b] = i00
        p2 = p
        p >>= 1


def _piz(src, file, src_off, dst_len, chans, width, num_lines):
    """DecompressPiz (:3228-3375): the pixel bytes (dst_len, line-interleaved like NONE data), or
    None where it returns false. `file`/`src_off`: the chunk's place in the file (past-the-chunk
    reads of damaged data see the following bytes of the file, then zeros)."""
    in_len = len(src)
    if in_len == dst_len:
        return bytes(src)  # stored raw (Issue 40)
    if in_len < 4:
        return None
    F = _Buf(file)
    mn, mxnz = struct.unpack_from("<HH", src, 0)
    if mxnz >= BITMAP_SIZE:
        return None
    bitmap = np.zeros(BITMAP_SIZE, np.uint8)
    rd = 4
    if mn <= mxnz:
        if mxnz - mn + 1 + rd > in_len:
            return None
        bitmap[mn:mxnz + 1] = np.frombuffer(src, np.uint8, mxnz - mn + 1, rd)
        rd += mxnz - mn + 1
    elif not (mn == BITMAP_SIZE - 1 and mxnz == 0):
        return None
    # reverseLutFromBitmap (:3081-3094): value 0 always, then every value whose bit is set
    bits = np.unpackbits(bitmap, bitorder="little").astype(bool)
    bits[0] = True
    vals = np.nonzero(bits)[0].astype(np.uint16)
    lut = np.zeros(1 << 16, np.uint16)
    lut[: len(vals)] = vals
    max_value = (len(vals) - 1) & 0xFFFF
    if rd + 4 > in_len:
        return None
    length = struct.unpack_from("<i", src, rd)[0]
    rd += 4
    if (rd + length) & M64 > in_len:  # size_t((ptr - inPtr) + length)
        return None
    nus = dst_len // 2
    dec = _huf_uncompress(F, src_off + rd, length, nus)
    tmp = np.zeros(nus, np.uint16)
    tmp[: len(dec)] = dec
    # channel planes, one after the other: channel c = width * num_lines * size ushorts
    starts, st = [], 0
    for _, pt in chans:
        sz = 1 if pt == HALF else 2
        starts.append((st, sz))
        st += width * num_lines * sz
    for st, sz in starts:
        for j in range(sz):
            wav2_decode(tmp, st + j, width, sz, num_lines, width * sz, max_value)
    tmp = lut[tmp]
    out = np.empty(nus, np.uint16)  # per line: each channel's width * size ushorts
    o = 0
    for v in range(num_lines):
        for st, sz in starts:
            n = width * sz
            out[o:o + n] = tmp[st + v * n: st + v * n + n]
            o += n
    return out.tobytes()


def _channel_layout(chans):
    offs, pds = [], 0
    for _, pt in chans:
        if pt not in SIZE:
            return None, None
        offs.append(pds)
        pds += SIZE[pt]
    return offs, pds


def _decode_pixels(planes, chans, offs, pds, data, comp, line_order, width, height, x_stride, y, line_no, num_lines,
                   file=b"", src_off=0):
    """DecodePixelData (:3631-4281) into planes (one uint32 bit pattern per sample: HALF as the
    float bits, FLOAT / UINT as stored). False on a decode failure. file / src_off: where `data`
    lies in the file (PIZ's reads of a damaged chunk can run past it)."""
    if comp == PIZ:  # (:3641-3790) line-interleaved pixel data like NONE, rows from line_no
        if width == 0 or num_lines == 0 or pds == 0:
            return False
        buf = _piz(data, file, src_off, width * num_lines * pds, chans, width, num_lines)
        if buf is None:
            return False
        row0 = line_no
    elif comp in (ZIP, ZIPS, RLE):
        dst_len = width * num_lines * pds
        if dst_len == 0:
            return False
        buf = _zip(data, dst_len) if comp != RLE else _rle(data, dst_len)
        if buf is None:
            return False
        row0 = line_no
    elif comp == NONE:
        buf = bytes(data)
        row0 = y
    else:
        return False
    for c, (name, pt) in enumerate(chans):
        s = SIZE[pt]
        for v in range(num_lines):
            base = v * pds * width + offs[c] * width
            if comp == NONE and base + width * s > len(buf):
                return False  # "Insufficient data size" (:4192-4196)
            row = row0 + v if line_order == 0 else height - 1 - (row0 + v)
            if row < 0 or row >= height:
                return False  # (tinyexr writes outside its image: chunkCount > lines, NONE)
            raw = np.frombuffer(buf, np.uint8, width * s, base)
            if pt == HALF:
                vals = raw.view("<f2").astype(np.float32).view(np.uint32)
            else:
                vals = raw.view("<u4")
            planes[c][row * x_stride: row * x_stride + width] = vals
    return True


def _floor_log2(x):  # FloorLog2 (:5582-5592)
    y = 0
    while x > 1:
        y += 1
        x >>= 1
    return y


def _ceil_log2(x):  # CeilLog2 (:5595-5610)
    y = r = 0
    while x > 1:
        if x & 1:
            r = 1
        y += 1
        x >>= 1
    return y + r


def level_size(top, level, rounding):
    """LevelSize (:4967-4979)."""
    b = 1 << level
    ls = top // b
    if rounding == 1 and ls * b < top:
        ls += 1
    return max(ls, 1)


def tile_levels(info):
    """PrecalculateTileInfo + InitTileOffsets (:5616-5802): the offset table's shape as a list of
    levels (lx, ly, tiles across, tiles down) in table order, or None (tinyexr: INVALID_DATA)."""
    x0, y0, x1, y1 = info["dw"]
    w, h = x1 - x0 + 1, y1 - y0 + 1
    mode, rnd = info["tile_mode"], info["tile_round"]
    tx, ty = info["tile"]
    lg = _floor_log2 if rnd == 0 else _ceil_log2
    if mode == 0:
        nxl = nyl = 1
    elif mode == 1:
        nxl = nyl = lg(max(w, h)) + 1
    elif mode == 2:
        nxl, nyl = lg(w) + 1, lg(h) + 1
    else:
        return None

    def ntiles(top, n, size):  # CalculateNumTiles (:5692-5706)
        out = []
        for i in range(n):
            ls = level_size(top, i, rnd)
            if ls > INT_MAX - size + 1:
                return None
            out.append((ls + size - 1) // size)
        return out

    nxt, nyt = ntiles(w, nxl, tx), ntiles(h, nyl, ty)
    if nxt is None or nyt is None:
        return None
    if mode in (0, 1):
        return [(l, l, nxt[l], nyt[l]) for l in range(nxl)]
    return [(lx, ly, nxt[lx], nyt[ly]) for ly in range(nyl) for lx in range(nxl)]


def _level_index(lx, ly, mode, nxl):  # LevelIndex (:4950-4965)
    return {0: 0, 1: lx, 2: lx + ly * nxl}.get(mode, -1)


def _reconstruct_tile_offsets(buf, marker, levels, mode, offs, multipart=False, deep=False):
    """ReconstructTileOffsets (:5867-5974): walk the chunks after the offset table and put each at
    the place its own header names (places no chunk names keep the table's value). The version
    flags reach it from LoadEXRFromMemory (:6101-6103): a multi-part file's chunk starts with a
    4-byte part number that is skipped (the offset recorded is the one before it, :5876-5886);
    a deep one has two int64 sizes after the coordinates, and the walk skips both payloads and
    the unpacked size (:5911-5931). None on failure (a marker moved before the file by a
    negative size also fails: tinyexr reads outside its buffer)."""
    size = len(buf)
    offs = [list(o) for o in offs]
    nxl = max(l[0] for l in levels) + 1
    nyl = max(l[1] for l in levels) + 1
    for _, _, nx, ny in levels:
        for _ in range(nx * ny):
            here = marker
            if multipart:
                if marker < 0 or marker + 4 >= size:
                    return None
                marker += 4
            if marker < 0 or marker + 16 >= size:
                return None
            tx_, ty_, lx, ly = struct.unpack_from("<iiii", buf, marker)
            marker += 16
            if deep:
                if marker + 16 >= size:
                    return None
                pot, ps = struct.unpack_from("<qq", buf, marker)
                marker += 16 + pot + ps + 8
                if marker >= size or marker < 0:
                    return None
            else:
                if marker + 4 >= size:
                    return None
                marker += 4 + _i32(buf, marker)
            # isValidTile (:5814-5865)
            if lx < 0 or ly < 0 or tx_ < 0 or ty_ < 0:
                return None
            if mode == 0 and (lx != 0 or ly != 0):
                return None
            if mode in (1, 2) and (lx >= nxl or ly >= nyl):
                return None
            li = _level_index(lx, ly, mode, nxl)
            if mode == 1 and lx >= len(levels):
                return None
            if li < 0 or li >= len(levels):
                return None
            _, _, nx_, ny_ = levels[li]
            if ty_ >= ny_ or tx_ >= nx_:
                return None
            offs[li][ty_ * nx_ + tx_] = here
    return offs


def decode(buf):
    """LoadEXRFromMemory: (code, width, height, rgba float32 array of shape (h, w, 4) or None)."""
    buf = bytes(buf)
    code, info = parse_header(buf)
    if code != SUCCESS:
        return code, 0, 0, None
    # (LoadEXRFromMemory has no multi-part / deep rejection: only LoadEXR does, :6268-6270; the
    # flags reach only the tile-offset reconstruction below)
    comp = info["compression"]
    size = len(buf)
    if size <= 8:
        return INVALID_ARGUMENT, 0, 0, None
    marker = info["header_len"] + 8
    nsb = {ZIP: 16, PIZ: 32}.get(comp, 1)
    x0, y0, x1, y1 = info["dw"]
    if x1 < x0 or x1 - x0 == INT_MAX:
        return INVALID_DATA, 0, 0, None
    dw = x1 - x0 + 1
    if y1 < y0 or y1 - y0 == INT_MAX:
        return INVALID_DATA, 0, 0, None
    dh = y1 - y0 + 1
    if dw > THRESH or dh > THRESH:
        return INVALID_DATA, 0, 0, None
    chans = info["channels"]
    tiled = info["tiled"]

    def read_offsets(n):
        nonlocal marker
        out = []
        for _ in range(n):
            if marker + 8 >= size:
                return None
            o = struct.unpack_from("<Q", buf, marker)[0]
            if o >= size:
                return None
            marker += 8
            out.append(o)
        return out

    if tiled:
        tx, ty = info["tile"]
        if tx > THRESH or ty > THRESH:
            return INVALID_DATA, 0, 0, None
        if tx == 0 or ty == 0:
            return INVALID_DATA, 0, 0, None  # (tinyexr divides by it)
        mode = info["tile_mode"]
        levels = tile_levels(info)
        if levels is None:
            return INVALID_DATA, 0, 0, None
        nblocks = sum(nx * ny for _, _, nx, ny in levels)
        if info["chunk_count"] > 0 and info["chunk_count"] != nblocks:
            return INVALID_DATA, 0, 0, None
        flat = read_offsets(nblocks)
        if flat is None:
            return INVALID_DATA, 0, 0, None
        offs, k = [], 0
        for _, _, nx, ny in levels:
            offs.append(flat[k:k + nx * ny])
            k += nx * ny
        if any(o == 0 for o in flat):
            offs = _reconstruct_tile_offsets(buf, marker, levels, mode, offs, info["multipart"], info["non_image"])
            if offs is None:
                return INVALID_DATA, 0, 0, None
    else:
        nblocks = info["chunk_count"] if info["chunk_count"] > 0 else (dh + nsb - 1) // nsb
        offsets = read_offsets(nblocks)
        if offsets is None:
            return INVALID_DATA, 0, 0, None
        if any(o == 0 for o in offsets):  # ReconstructLineOffsets (:5544-5580)
            m = marker
            for i in range(nblocks):
                if m + 8 >= size:
                    return INVALID_DATA, 0, 0, None
                dl = struct.unpack_from("<I", buf, m + 4)[0]
                if dl >= size:
                    return INVALID_DATA, 0, 0, None
                offsets[i] = m
                m += dl + 8
    # DecodeChunk (:5163-5542)
    offs_c, pds = _channel_layout(chans)
    if offs_c is None:
        return INVALID_DATA, 0, 0, None
    nch = len(chans)
    if tiled:
        # every level is decoded (DecodeTiledLevel per level: :5282-5354), a failure in any of
        # them fails the read; only level 0 reaches the RGBA output
        tiles0 = None
        for li, (lx, ly, nx, ny) in enumerate(levels):
            lw, lh = level_size(dw, lx, info["tile_round"]), level_size(dh, ly, info["tile_round"])
            invalid = False
            tiles = []
            for idx in range(nx * ny):
                planes = [np.zeros(tx * ty, np.uint32) for _ in range(nch)]
                o = offs[li][idx]
                if o + 20 > size:
                    invalid = True
                    continue
                dsz = size - (o + 20)
                cx, cy, clx, cly = struct.unpack_from("<iiii", buf, o)
                if clx != lx or cly != ly:
                    invalid = True
                    continue
                dlen = _i32(buf, o + 16)
                if dlen < 2 or dlen > dsz:
                    invalid = True
                    continue
                data = buf[o + 20:o + 20 + dlen]
                # DecodeTiledPixelData (:4283-4319), in the level's size
                # (int arithmetic: a damaged tile coordinate's product wraps as it does in the
                # reference build's 32-bit multiplies)
                if _w32(tx * cx) > lw or _w32(ty * cy) > lh:
                    ok = False
                else:
                    w = _w32(lw - _w32(cx * tx)) if _w32(_w32(cx + 1) * tx) >= lw else tx
                    h = _w32(lh - _w32(cy * ty)) if _w32(_w32(cy + 1) * ty) >= lh else ty
                    ok = _decode_pixels(planes, chans, offs_c, pds, data, comp, info["line_order"], w, ty, tx, 0, 0, h,
                                        buf, o + 20)
                if not ok:
                    invalid = True
                tiles.append((cx, cy, planes))
            if invalid:
                return INVALID_DATA, 0, 0, None
            if li == 0:
                tiles0 = tiles
    else:
        invalid = False
        if dw * dh * nch == 0 or dw * dh * nch >= 0x4000000000:
            return INVALID_DATA, 0, 0, None
        planes = [np.zeros(dw * dh, np.uint32) for _ in range(nch)]
        for y in range(nblocks):
            o = offsets[y]
            if o + 8 > size:
                invalid = True
                continue
            dsz = size - (o + 8)
            line_no = _i32(buf, o)
            dlen = _i32(buf, o + 4)
            if dlen > dsz or line_no > (2 << 20) or line_no < -(2 << 20) or dlen == 0:
                invalid = True  # (a negative dlen wraps to a huge size_t: > dsz)
                continue
            if dlen < 0:
                invalid = True
                continue
            end = min(line_no + nsb, y1 + 1)
            nl = end - line_no
            if nl <= 0:
                invalid = True
                continue
            lno = line_no - y0
            if lno > INT_MAX or lno < -INT_MAX or lno < 0:
                invalid = True
                continue
            data = buf[o + 8:o + 8 + dlen]
            if not _decode_pixels(planes, chans, offs_c, pds, data, comp, info["line_order"], dw, dh, dw, y, lno, nl,
                                  buf, o + 8):
                invalid = True
        if invalid:
            return INVALID_DATA, 0, 0, None
    # RGBA (LoadEXRFromMemory :6685-6860)
    names = [c[0] for c in chans]
    idx = {k: (names.index(k) if k in names else -1) for k in "RGBA"}
    # (strcmp runs over every channel and keeps the LAST match: :6690-6703)
    for k in "RGBA":
        for c, nm in enumerate(names):
            if nm == k:
                idx[k] = c
    out = np.zeros((dh, dw, 4), np.uint32)
    one = np.float32(1.0).view(np.uint32)
    if nch != 1 and (idx["R"] < 0 or idx["G"] < 0 or idx["B"] < 0):
        return INVALID_DATA, 0, 0, None
    src = [0, 0, 0, 0] if nch == 1 else [idx["R"], idx["G"], idx["B"], idx["A"]]
    if tiled:
        for cx, cy, pl in tiles0:
            if cx < 0 or cy < 0:
                continue  # (size_t tile origins: past the image, skipped)
            for j in range(ty):
                jj = cy * ty + j
                if jj >= dh or jj < 0:
                    continue
                i0 = cx * tx
                iw = min(tx, dw - i0)
                if iw <= 0:
                    continue
                for k in range(4):
                    if src[k] < 0:
                        out[jj, i0:i0 + iw, k] = one
                    else:
                        out[jj, i0:i0 + iw, k] = pl[src[k]][j * tx:j * tx + iw]
    else:
        for k in range(4):
            out[:, :, k] = one if src[k] < 0 else planes[src[k]].reshape(dh, dw)
    return SUCCESS, dw, dh, out.view(np.float32)
