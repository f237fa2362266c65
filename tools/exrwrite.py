"""OpenEXR writer for test fixtures (single part, scanline or one-level tiled; NONE / RLE / ZIPS /
ZIP compression; HALF / FLOAT / UINT channels). TEST INFRASTRUCTURE: it makes the inputs the EXR
tests decode -- no EXR library is importable here, so the files are written from the format as
tinyexr reads it (/root/reference/tinyexr.h: header attributes :4441-4801, offset table :6077-6169,
scanline chunks :5412-5496, tiles :5061-5107, RLE / ZIP byte transforms :1424-1760).

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


def compress(raw: bytes, comp: int) -> bytes:
    if comp == NONE:
        return raw
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


def write_exr(channels, compression=ZIP, tiles=None, line_order=0, origin=(0, 0), sort=True, attrs=None,
              raw_chunks=None, offsets=None, chunk_line=None, version_flags=None, extra_attrs=b"",
              drop=()):
    """channels: list of (name, HxW array) -- dtype float16 / float32 / uint32 picks the pixel type.
    tiles: None (scanline) or (tile_w, tile_h) one-level tiles, round down. origin: dataWindow min.
    raw_chunks(i, bytes) -> bytes may replace chunk i's payload; offsets(list) -> list may edit the
    offset table; chunk_line(i, y) -> y may change a scanline chunk's line number; drop: required
    attribute names to leave out."""
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
        a["tiles"] = attr("tiles", "tiledesc", struct.pack("<IIB", tiles[0], tiles[1], 0))
    for k, v in (attrs or {}).items():
        a[k] = v
    header = b"".join(v for k, v in a.items() if k not in drop) + extra_attrs + b"\0"
    flags = version_flags if version_flags is not None else (0x2 if tiles else 0)
    head = bytes([0x76, 0x2F, 0x31, 0x01, 2, flags, 0, 0]) + header
    chunks = []
    if tiles:
        tw, th = tiles
        nty, ntx = -(-h // th), -(-w // tw)
        for ty in range(nty):
            for tx in range(ntx):
                raw = block_bytes(chans, arrays, ty * th, min(h, ty * th + th), tx * tw, min(w, tx * tw + tw))
                data = compress(raw, compression)
                if raw_chunks:
                    data = raw_chunks(len(chunks), data)
                chunks.append(struct.pack("<iiiii", tx, ty, 0, 0, len(data)) + data)
    else:
        n = LINES[compression]
        for k in range(-(-h // n)):
            raw = block_bytes(chans, arrays, k * n, min(h, k * n + n), 0, w)
            data = compress(raw, compression)
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
