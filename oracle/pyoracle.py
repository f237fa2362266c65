"""ctypes bindings for the oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module (as the checker). The product (imagecodecs_amd) never does.

  decode(jpeg)            -> (code, w, h, ncomp, bytes)   oracle/liboracle.so  (CPU restatement)
  decode_trace(jpeg)      -> (code, coef[int16 n,64], dc[int32 n])
  tje_encode(q, w, h, c, rgb) -> bytes | None            oracle/liboracle.so
  ref_decode / ref_tje_encode                             oracle/_ref/libref_jpeg.so (the
                                                         reference itself; container only)
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None


def build(ref: bool = False) -> None:
    subprocess.run(["make", "-s", "-C", _HERE, "all"] + (["ref"] if ref else []), check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.or_nj_decode.restype = C.c_int
        L.or_nj_decode.argtypes = [C.c_void_p, C.c_int64, C.POINTER(C.c_void_p), C.POINTER(C.c_int),
                                   C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_void_p]
        L.or_tje_encode.restype = C.c_int
        L.or_tje_encode.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                    C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]
        L.or_jpeg_encode.restype = C.c_int
        L.or_jpeg_encode.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                     C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]
        L.or_png_choose.restype = C.c_int
        L.or_png_choose.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.or_png_filtered_size.restype = C.c_int64
        L.or_png_filtered_size.argtypes = [C.c_int, C.c_int, C.c_void_p]
        L.or_png_filter.restype = C.c_int
        L.or_png_filter.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.or_png_encode.restype = C.c_int
        L.or_png_encode.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p),
                                    C.POINTER(C.c_int64)]
        L.or_hdr_decode.restype = C.c_int
        L.or_hdr_decode.argtypes = [C.c_void_p, C.c_int64, C.POINTER(C.c_void_p), C.POINTER(C.c_int),
                                    C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.or_free.argtypes = [C.c_void_p]
        _LIB = L
    return _LIB


class _Trace(C.Structure):
    _fields_ = [("nblocks", C.c_int32), ("coef", C.c_void_p), ("dc", C.c_void_p), ("cap_blocks", C.c_int32)]


def _decode(data: bytes, trace=None):
    L = lib()
    buf = C.create_string_buffer(bytes(data), len(data))
    out = C.c_void_p()
    w, h, n = C.c_int(), C.c_int(), C.c_int()
    code = L.or_nj_decode(buf, len(data), C.byref(out), C.byref(w), C.byref(h), C.byref(n),
                          C.byref(trace) if trace is not None else None)
    pix = b""
    if out.value:
        pix = C.string_at(out.value, w.value * h.value * n.value)
        L.or_free(out)
    return code, w.value, h.value, n.value, pix


def decode(data: bytes):
    """NanoJPEG-equivalent decode -> (code, w, h, ncomp, pixel bytes)."""
    return _decode(data)


def decode_trace(data: bytes, cap_blocks: int = 1 << 20):
    coef = np.zeros((cap_blocks, 64), np.int16)
    dc = np.zeros(cap_blocks, np.int32)
    t = _Trace(0, coef.ctypes.data, dc.ctypes.data, cap_blocks)
    code = _decode(data, t)[0]
    n = min(t.nblocks, cap_blocks)
    return code, coef[:n].copy(), dc[:n].copy()


def jpeg_encode(quality: int, subsampling: int, w: int, h: int, comps: int, rgb: bytes):
    """C4 extension encoder definition (IJG quality 1..100, 4:4:4 / 4:2:0); None on error."""
    L = lib()
    data = bytes(rgb)
    src = C.create_string_buffer(data, max(1, len(data)))
    out = C.c_void_p()
    n = C.c_int64()
    if not L.or_jpeg_encode(quality, subsampling, w, h, comps, src, C.byref(out), C.byref(n)):
        return None
    res = C.string_at(out.value, n.value)
    L.or_free(out)
    return res


class PngMode(C.Structure):
    _fields_ = [("colortype", C.c_int), ("bitdepth", C.c_int), ("npal", C.c_int), ("pal", C.c_uint8 * 1024),
                ("key_defined", C.c_int), ("key_r", C.c_int), ("key_g", C.c_int), ("key_b", C.c_int)]

    def as_dict(self):
        return {"colortype": self.colortype, "bitdepth": self.bitdepth, "npal": self.npal,
                "palette": bytes(self.pal[: 4 * self.npal]), "key": (self.key_r, self.key_g, self.key_b)
                if self.key_defined else None}


def png_choose(px: bytes, w: int, h: int, d: int) -> PngMode:
    """lodepng auto_convert decision for saveToFile input (d=3 RGB8, d=4 RGBA8)."""
    m = PngMode()
    src = C.create_string_buffer(bytes(px), max(1, len(px)))
    if not lib().or_png_choose(src, w, h, d, C.byref(m)):
        raise ValueError("or_png_choose failed")
    return m


def png_filtered(px: bytes, w: int, h: int, d: int, mode: PngMode = None) -> bytes:
    """The filtered (pre-deflate) IDAT stream lodepng produces for this image."""
    m = mode or png_choose(px, w, h, d)
    n = lib().or_png_filtered_size(w, h, C.byref(m))
    out = C.create_string_buffer(max(1, n))
    src = C.create_string_buffer(bytes(px), max(1, len(px)))
    if not lib().or_png_filter(src, w, h, d, C.byref(m), out):
        raise ValueError("or_png_filter failed")
    return out.raw[:n]


def png_encode_zlib(px: bytes, w: int, h: int, d: int, level: int = 6):
    """Whole PNG: restated colour choice + filters, IDAT by the system zlib (size proxy)."""
    src = C.create_string_buffer(bytes(px), max(1, len(px)))
    out = C.c_void_p()
    n = C.c_int64()
    if not lib().or_png_encode(src, w, h, d, level, C.byref(out), C.byref(n)):
        return None
    res = C.string_at(out.value, n.value)
    lib().or_free(out)
    return res


def tje_encode(quality: int, w: int, h: int, comps: int, rgb: bytes):
    L = lib()
    data = bytes(rgb)
    src = C.create_string_buffer(data, max(1, len(data)))
    out = C.c_void_p()
    n = C.c_int64()
    ok = L.or_tje_encode(quality, w, h, comps, src, C.byref(out), C.byref(n))
    if not ok:
        return None
    res = C.string_at(out.value, n.value)
    L.or_free(out)
    return res


# ---- the reference itself (oracle/_ref, built from /root/reference in place) ----
def ref_available() -> bool:
    return os.path.exists(os.path.join(_HERE, "_ref", "libref_jpeg.so"))


def ref():
    global _REF
    if _REF is None:
        L = C.CDLL(os.path.join(_HERE, "_ref", "libref_jpeg.so"))
        L.ref_nj_decode.restype = C.c_int
        L.ref_nj_decode.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                    C.POINTER(C.c_int), C.c_void_p, C.c_longlong]
        L.ref_tje_encode.restype = C.c_int
        L.ref_tje_encode.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                     C.c_longlong, C.POINTER(C.c_longlong)]
        _REF = L
    return _REF


def ref_decode(data: bytes, cap: int = 1 << 28):
    L = ref()
    src = C.create_string_buffer(bytes(data), max(1, len(data)))
    out = C.create_string_buffer(cap)
    w, h, n = C.c_int(), C.c_int(), C.c_int()
    code = L.ref_nj_decode(src, len(data), C.byref(w), C.byref(h), C.byref(n), out, cap)
    if code != 0:
        return code, 0, 0, 0, b""
    return code, w.value, h.value, n.value, out.raw[: w.value * h.value * n.value]


def ref_tje_encode(quality: int, w: int, h: int, comps: int, rgb: bytes, cap: int = 1 << 28):
    L = ref()
    data = bytes(rgb)
    src = C.create_string_buffer(data, max(1, len(data)))
    out = C.create_string_buffer(cap)
    n = C.c_longlong()
    ok = L.ref_tje_encode(quality, w, h, comps, src, out, cap, C.byref(n))
    if ok != 1:
        return None
    return out.raw[: n.value]


HDR_OK, HDR_NOT_RADIANCE, HDR_BAD_HEADER, HDR_MALFORMED, HDR_TRUNCATED = 0, 1, 2, 3, 4


def hdr_decode(data: bytes):
    """Image::readHdr restatement -> (code, w, h, rows, float32 array (h, w, 4) or None)."""
    L = lib()
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    out = C.c_void_p()
    w, h, rows = C.c_int(), C.c_int(), C.c_int()
    code = L.or_hdr_decode(buf, len(data), C.byref(out), C.byref(w), C.byref(h), C.byref(rows))
    arr = None
    if out.value:
        n = w.value * h.value * 4
        arr = np.frombuffer(C.string_at(out.value, n * 4), dtype=np.float32).reshape(h.value, w.value, 4).copy()
        L.or_free(out)
    return code, w.value, h.value, rows.value, arr
