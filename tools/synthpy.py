"""ctypes bindings for tools/libsynth.so: synthetic RGB images + baseline JPEG encoding.

Used by tests/ and bench.py to generate inputs (SURVEY.md §8(d) recipe). Not product code.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

SAMPLING = {"gray": 0, "444": 0x11, "422": 0x21, "420": 0x22, "440": 0x12, "411": 0x41,
            "y44": 0x44}  # y44: Y 4x4 + Cb + Cr = 18 blocks per MCU (beyond the JPEG limit of 10; NanoJPEG decodes it)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libsynth.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        L = C.CDLL(path)
        L.synth_rgb.restype = C.c_int
        L.synth_rgb.argtypes = [C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.synth_jpeg.restype = C.c_int64
        L.synth_jpeg.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_void_p, C.c_int64]
        L.synth_rgbe.restype = C.c_int
        L.synth_rgbe.argtypes = [C.c_uint64, C.c_int, C.c_int, C.c_void_p]
        L.hdr_encode.restype = C.c_int64
        L.hdr_encode.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int64]
        _LIB = L
    return _LIB


def rgb(seed: int, w: int, h: int, comps: int = 3) -> np.ndarray:
    out = np.empty((h, w, comps), np.uint8)
    if not lib().synth_rgb(seed, w, h, comps, out.ctypes.data):
        raise ValueError("synth_rgb failed")
    return out


def jpeg(pixels: np.ndarray, sampling: str = "420", quality: int = 90, restart: int = 0) -> bytes:
    pixels = np.ascontiguousarray(pixels, dtype=np.uint8)
    if pixels.ndim == 2:
        pixels = pixels[:, :, None]
    h, w, c = pixels.shape
    cap = w * h * c * 2 + 65536
    out = np.empty(cap, np.uint8)
    n = lib().synth_jpeg(pixels.ctypes.data, w, h, c, SAMPLING[sampling], quality, restart,
                         out.ctypes.data, cap)
    if n < 0:
        raise ValueError("synth_jpeg failed")
    return out[:n].tobytes()


def synth_jpeg(seed: int, w: int, h: int, sampling: str = "420", quality: int = 90, restart: int = 0) -> bytes:
    return jpeg(rgb(seed, w, h, 1 if sampling == "gray" else 3), sampling, quality, restart)


HDR_RLE, HDR_FLAT, HDR_OLD_RLE = 0, 1, 2


def rgbe(seed: int, w: int, h: int) -> np.ndarray:
    out = np.empty((h, w, 4), np.uint8)
    if not lib().synth_rgbe(seed, w, h, out.ctypes.data):
        raise ValueError("synth_rgbe failed")
    return out


def hdr(pixels: np.ndarray, mode: int = HDR_RLE) -> bytes:
    """Radiance .hdr file of RGBE pixels (h, w, 4): new RLE, flat, or old-style RLE."""
    pixels = np.ascontiguousarray(pixels, dtype=np.uint8)
    h, w, _ = pixels.shape
    cap = w * h * 5 + 4 * h + 256
    out = np.empty(cap, np.uint8)
    n = lib().hdr_encode(pixels.ctypes.data, w, h, mode, out.ctypes.data, cap)
    if n < 0:
        raise ValueError("hdr_encode overflow")
    return out[:n].tobytes()
