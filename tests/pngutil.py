"""Test helpers for the PNG path: a small PNG reader (zlib + PNG unfiltering, all colour types
at the bit depths lodepng chooses for 8-bit input, non-interlaced) and the synthetic C5 inputs."""
import struct
import zlib

import numpy as np


def chunks(data: bytes):
    assert data[:8] == b"\x89PNG\r\n\x1a\n", "not a PNG"
    p, out = 8, []
    while p < len(data):
        n, t = struct.unpack(">I4s", data[p:p + 8])
        body = data[p + 8:p + 8 + n]
        crc = struct.unpack(">I", data[p + 8 + n:p + 12 + n])[0]
        assert zlib.crc32(t + body) & 0xFFFFFFFF == crc, f"bad CRC in {t}"
        out.append((t.decode(), body))
        p += 12 + n
    return out


def info(data: bytes) -> dict:
    cs = chunks(data)
    w, h, bd, ct, _, _, il = struct.unpack(">IIBBBBB", cs[0][1])
    assert cs[0][0] == "IHDR" and cs[-1][0] == "IEND" and il == 0
    idat = b"".join(b for t, b in cs if t == "IDAT")
    return {"w": w, "h": h, "bitdepth": bd, "colortype": ct, "idat": idat,
            "plte": next((b for t, b in cs if t == "PLTE"), None),
            "trns": next((b for t, b in cs if t == "tRNS"), None), "types": [t for t, _ in cs]}


def unfilter(raw: bytes, h: int, lb: int, bw: int) -> np.ndarray:
    f = np.frombuffer(raw, np.uint8).reshape(h, lb + 1)
    out = np.zeros((h, lb), np.uint8)
    prev = np.zeros(lb, np.int32)
    for y in range(h):
        t, s = f[y, 0], f[y, 1:].astype(np.int32)
        if t == 0:
            cur = s
        elif t == 2:
            cur = (s + prev) & 255
        else:
            cur = np.zeros(lb, np.int32)
            for i in range(lb):  # sequential: left neighbour dependency
                a = cur[i - bw] if i >= bw else 0
                b = prev[i]
                c = prev[i - bw] if i >= bw else 0
                if t == 1:
                    pr = a
                elif t == 3:
                    pr = (a + b) >> 1
                else:
                    pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                    pr = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
                cur[i] = (s[i] + pr) & 255
        out[y] = cur
        prev = cur
    return out


def decode_rgba(data: bytes) -> np.ndarray:
    """PNG -> (h, w, 4) uint8 RGBA (tRNS applied), for round-trip checks on small images."""
    I = info(data)
    w, h, bd, ct = I["w"], I["h"], I["bitdepth"], I["colortype"]
    ch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ct]
    bpp = ch * bd
    lb, bw = (w * bpp + 7) // 8, max(1, bpp // 8)
    rows = unfilter(zlib.decompress(I["idat"]), h, lb, bw)
    if bd < 8:
        bits = np.unpackbits(rows, axis=1)[:, : w * bd].reshape(h, w, bd)
        vals = np.zeros((h, w), np.int32)
        for k in range(bd):
            vals = (vals << 1) | bits[:, :, k]
    else:
        vals = rows[:, : w * ch].reshape(h, w, ch).astype(np.int32)
    out = np.zeros((h, w, 4), np.uint8)
    if ct == 3:
        pal = np.frombuffer(I["plte"], np.uint8).reshape(-1, 3)
        alpha = np.full(len(pal), 255, np.uint8)
        if I["trns"]:
            alpha[: len(I["trns"])] = np.frombuffer(I["trns"], np.uint8)
        idx = vals if bd < 8 else vals[:, :, 0]
        out[..., :3] = pal[idx]
        out[..., 3] = alpha[idx]
        return out
    if bd < 8:
        g = (vals * (255 // ((1 << bd) - 1))).astype(np.uint8)
        out[..., 0] = out[..., 1] = out[..., 2] = g
        out[..., 3] = 255
        if I["trns"]:
            k = struct.unpack(">H", I["trns"])[0]
            out[..., 3][vals == k] = 0
        return out
    if ct in (0, 4):
        out[..., 0] = out[..., 1] = out[..., 2] = vals[..., 0]
        out[..., 3] = vals[..., 1] if ct == 4 else 255
    else:
        out[..., :3] = vals[..., :3]
        out[..., 3] = vals[..., 3] if ct == 6 else 255
    if I["trns"] and ct in (0, 2):
        k = struct.unpack(">HHH", I["trns"]) if ct == 2 else (struct.unpack(">H", I["trns"])[0],) * 3
        m = (vals[..., 0] == k[0]) & (vals[..., min(1, ch - 1)] == k[1]) & (vals[..., min(2, ch - 1)] == k[2])
        out[..., 3][m] = 0
    return out


def to_rgba(px: np.ndarray) -> np.ndarray:
    if px.shape[2] == 4:
        return px
    return np.concatenate([px, np.full(px.shape[:2] + (1,), 255, np.uint8)], axis=2)


def synth_rgba(seed: int, w: int, h: int, opaque: bool = False) -> np.ndarray:
    """C5 input: synthetic RGB + alpha = horizontal gradient (lodepng keeps
    RGBA), or alpha 255 (lodepng drops it: RGB)."""
    from tools import synthpy
    rgb = synthpy.rgb(seed, w, h, 3)
    a = np.full((h, w, 1), 255, np.uint8) if opaque else \
        np.broadcast_to((np.arange(w, dtype=np.int64) * 255 // max(1, w - 1)).astype(np.uint8)[None, :, None], (h, w, 1))
    return np.ascontiguousarray(np.concatenate([rgb, a], axis=2))


def read_fixture_png(path: str) -> np.ndarray:
    return decode_rgba(open(path, "rb").read())
