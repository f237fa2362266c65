"""TEST-ONLY oracle: a Python restatement of tinyexr's LoadEXRFromMemory (/root/reference/tinyexr.h
:6645-6860) for single-part scanline and one-level tiled images, NONE / RLE / ZIPS / ZIP
compression. Only tests/ may import it; libicx never does.

PARITY UNPINNED: tinyexr.h cannot be built here -- it needs miniz (TINYEXR_USE_MINIZ, codecs.cpp:28),
which /root/reference does not ship, or an external zlib -- and the reference holds no .exr file.
This module is pinned only by its own round trips of tools/exrwrite.py files and by following
tinyexr's code line by line; zlib's inflate stands in for miniz's mz_uncompress (both are RFC 1950
/ 1951 decoders that check the Adler-32; a valid stream inflates to the same bytes).

What it returns where tinyexr's result is undefined or out of this build's scope (the GPU path
does the same):
* rows / tile pixels no chunk wrote are 0.0 (tinyexr: uninitialised malloc memory); a NONE
  chunk whose block index lies past the image (chunkCount > lines: tinyexr writes outside its
  buffer) is a decode failure (INVALID_DATA);
* PIZ (4) -> UNSUPPORTED_FORMAT (tinyexr with TINYEXR_USE_PIZ 0), multi-part / deep files and
  mip-/rip-mapped tiles -> UNSUPPORTED_FEATURE; a tile size of 0 -> INVALID_DATA (tinyexr
  divides by it).
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


def _channel_layout(chans):
    offs, pds = [], 0
    for _, pt in chans:
        if pt not in SIZE:
            return None, None
        offs.append(pds)
        pds += SIZE[pt]
    return offs, pds


def _decode_pixels(planes, chans, offs, pds, data, comp, line_order, width, height, x_stride, y, line_no, num_lines):
    """DecodePixelData (:3631-4281) into planes (one uint32 bit pattern per sample: HALF as the
    float bits, FLOAT / UINT as stored). False on a decode failure."""
    if comp in (ZIP, ZIPS, RLE):
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


def decode(buf):
    """LoadEXRFromMemory: (code, width, height, rgba float32 array of shape (h, w, 4) or None)."""
    buf = bytes(buf)
    code, info = parse_header(buf)
    if code != SUCCESS:
        return code, 0, 0, None
    if info["multipart"] or info["non_image"]:
        return UNSUPPORTED_FEATURE, 0, 0, None
    comp = info["compression"]
    if comp == PIZ:
        return UNSUPPORTED_FORMAT, 0, 0, None
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
    if tiled:
        tx, ty = info["tile"]
        if tx > THRESH or ty > THRESH:
            return INVALID_DATA, 0, 0, None
        if info["tile_mode"] != 0:
            return UNSUPPORTED_FEATURE, 0, 0, None
        if tx == 0 or ty == 0:
            return INVALID_DATA, 0, 0, None
        ntx, nty = (dw + tx - 1) // tx, (dh + ty - 1) // ty
        nblocks = ntx * nty
        if info["chunk_count"] > 0 and info["chunk_count"] != nblocks:
            return INVALID_DATA, 0, 0, None
        offsets = []
        for _ in range(nblocks):
            if marker + 8 >= size:
                return INVALID_DATA, 0, 0, None
            o = struct.unpack_from("<Q", buf, marker)[0]
            if o >= size:
                return INVALID_DATA, 0, 0, None
            marker += 8
            offsets.append(o)
        if any(o == 0 for o in offsets):
            return INVALID_DATA, 0, 0, None  # (ReconstructTileOffsets: out of this build's scope)
    else:
        nblocks = info["chunk_count"] if info["chunk_count"] > 0 else (dh + nsb - 1) // nsb
        offsets = []
        for _ in range(nblocks):
            if marker + 8 >= size:
                return INVALID_DATA, 0, 0, None
            o = struct.unpack_from("<Q", buf, marker)[0]
            if o >= size:
                return INVALID_DATA, 0, 0, None
            marker += 8
            offsets.append(o)
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
    if x1 < x0 or y1 < y0 or dw <= 0 or dh <= 0:
        return INVALID_DATA, 0, 0, None
    offs, pds = _channel_layout(chans)
    if offs is None:
        return INVALID_DATA, 0, 0, None
    nch = len(chans)
    invalid = False
    if tiled:
        tiles = []
        for idx in range(nblocks):
            planes = [np.zeros(tx * ty, np.uint32) for _ in range(nch)]
            o = offsets[idx]
            if o + 20 > size:
                invalid = True
                continue
            dsz = size - (o + 20)
            cx, cy, lx, ly = struct.unpack_from("<iiii", buf, o)
            if lx != 0 or ly != 0:
                invalid = True
                continue
            dlen = _i32(buf, o + 16)
            if dlen < 2 or dlen > dsz:
                invalid = True
                continue
            data = buf[o + 20:o + 20 + dlen]
            # DecodeTiledPixelData (:4283-4319)
            if tx * cx > dw or ty * cy > dh:
                ok = False
            else:
                w = dw - cx * tx if (cx + 1) * tx >= dw else tx
                h = dh - cy * ty if (cy + 1) * ty >= dh else ty
                ok = _decode_pixels(planes, chans, offs, pds, data, comp, info["line_order"], w, ty, tx, 0, 0, h)
            if not ok:
                invalid = True
            tiles.append((cx, cy, planes))
        if invalid:
            return INVALID_DATA, 0, 0, None
    else:
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
            if not _decode_pixels(planes, chans, offs, pds, data, comp, info["line_order"], dw, dh, dw, y, lno, nl):
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
        for cx, cy, pl in tiles:
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
