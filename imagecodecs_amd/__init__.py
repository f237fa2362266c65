"""imagecodecs_amd -- MI355X-native JPEG codec behind ImageCodecs' codecs.h API.

The product is the C-ABI library ``imagecodecs_amd/lib/libicx.so`` (include/icx.h): hand-
written gfx950 HIP kernels for the NanoJPEG-exact decode path and the tiny_jpeg-exact
encode path. This module is the host-side mirror of the reference interface for Python
callers (tests, bench): it binds the C ABI with ctypes and offers

  * ``Context``                   -- one device + stream (icx_create)
  * ``Context.nj_decode`` & co.   -- njInit/njDecode/njGet* semantics (jpeg_dec.h:117-171)
  * ``Context.decode``            -- Image::readJpg's one-shot decode (codecs.cpp:821-849)
  * ``Batch``                     -- device-resident batched decode (the throughput path)
  * ``Context.hdr_decode``        -- Image::readHdr's Radiance RGBE -> float decode (codecs.cpp:706-777)
  * ``HdrBatch``                  -- device-resident batched .hdr decode
  * ``Context.exr_decode``        -- Image::readExr's OpenEXR -> RGBA float (tinyexr LoadEXRFromMemory)
  * ``Image``                     -- ImageCodecs::Image (codecs.h:16-103) for .jpg/.jpeg/.png/.hdr

There is deliberately no CPU fallback: if libicx.so is missing or no GPU is visible every
entry point raises ``ICXError``.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

__all__ = ["ICXError", "Context", "Batch", "HdrBatch", "Image", "lib", "build", "LIB_PATH",
           "OK", "NO_JPEG", "UNSUPPORTED", "OUT_OF_MEM", "INTERNAL_ERR", "SYNTAX_ERROR",
           "HDR_OK", "HDR_NOT_RADIANCE", "HDR_BAD_HEADER", "HDR_MALFORMED", "HDR_TRUNCATED",
           "HDR_TOO_LARGE", "HDR_INTERNAL_ERR", "hdr_probe", "exr_probe", "EXR_SUCCESS", "EXR_INVALID_DATA", "Multi", "RECORD_DTYPE", "records_device",
           "checksum64", "multi_shard"]

OK, NO_JPEG, UNSUPPORTED, OUT_OF_MEM, INTERNAL_ERR, SYNTAX_ERROR = range(6)  # nj_result_t
RESULT_NAMES = ["NJ_OK", "NJ_NO_JPEG", "NJ_UNSUPPORTED", "NJ_OUT_OF_MEM", "NJ_INTERNAL_ERR", "NJ_SYNTAX_ERROR"]

_HERE = os.path.dirname(os.path.abspath(__file__))
# ICX_LIB selects another build of the same library (e.g. an instrumented variant); it is
# still the HIP library, there is no other implementation to select.
_DEFAULT_LIB = os.path.join(_HERE, "lib", "libicx.so")
LIB_PATH = os.environ.get("ICX_LIB") or _DEFAULT_LIB
_LIB = None


class ICXError(RuntimeError):
    pass


def build() -> str:
    """Compile libicx.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


_vp, _i32, _i64, _u64, _sz = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_size_t
_SIGS = {
    "icx_version": (C.c_char_p, []),
    "icx_last_error": (C.c_char_p, [_vp]),
    "icx_create": (_vp, [_i32]),
    "icx_destroy": (None, [_vp]),
    "icx_free": (None, [_vp]),
    "icx_jpeg_probe": (_i32, [_vp, _sz, C.POINTER(_i32), C.POINTER(_i32), C.POINTER(_i32)]),
    "icx_nj_init": (None, [_vp]),
    "icx_nj_done": (None, [_vp]),
    "icx_nj_decode": (_i32, [_vp, _vp, _i32]),
    "icx_nj_get_width": (_i32, [_vp]),
    "icx_nj_get_height": (_i32, [_vp]),
    "icx_nj_is_color": (_i32, [_vp]),
    "icx_nj_get_image": (_vp, [_vp]),
    "icx_nj_get_image_size": (_i32, [_vp]),
    "icx_jpeg_decode": (_i32, [_vp, _vp, _sz, C.POINTER(_vp), C.POINTER(_i32), C.POINTER(_i32), C.POINTER(_i32)]),
    "icx_batch_create": (_vp, [_vp, _i32, _i32, _i32, _i32]),
    "icx_batch_destroy": (None, [_vp]),
    "icx_jpeg_batch_decode": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    "icx_jpeg_batch_decode_host": (_i32, [_vp, _i32, _vp, _vp, _vp, _u64, _vp, _vp]),
    "icx_batch_stage_times": (_i32, [_vp, _vp, _vp, _i32]),
    "icx_batch_group": (_i32, [_vp]),
    "icx_batch_groups": (_i32, [_vp, _i32]),
    "icx_batch_path_stats": (_i32, [_vp, C.POINTER(_i32), C.POINTER(_i32), C.POINTER(_i32)]),
    "icx_tje_encode_with_func": (_i32, [_vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp]),
    "icx_tje_encode_to_file_at_quality": (_i32, [_vp, C.c_char_p, _i32, _i32, _i32, _i32, _vp]),
    "icx_tje_encode_to_file": (_i32, [_vp, C.c_char_p, _i32, _i32, _i32, _vp]),
    "icx_jpeg_encode_with_func": (_i32, [_vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp]),
    "icx_encoder_create": (_vp, [_vp]),
    "icx_encoder_destroy": (None, [_vp]),
    "icx_encoder_stage_times": (_i32, [_vp, _vp, _vp, _i32]),
    "icx_png_encode_with_func": (_i32, [_vp, _vp, _vp, _vp, _i32, _i32, _i32]),
    "icx_png_save_to_file": (_i32, [_vp, C.c_char_p, _vp, _i32, _i32, _i32]),
    "icx_png_encoder_create": (_vp, [_vp]),
    "icx_png_encoder_destroy": (None, [_vp]),
    "icx_png_encode_device": (_i32, [_vp, _i32, _i32, _i32, _vp, _vp, _u64, C.POINTER(_u64), _vp]),
    "icx_png_encode_device_batch": (_i32, [_vp, _i32, _i32, _i32, _i32, _vp, _vp, _u64, _vp, _vp, _vp]),
    "icx_png_encoder_stage_times": (_i32, [_vp, C.POINTER(C.c_char_p), C.POINTER(C.c_float), _i32]),
    "icx_jpeg_encode_device": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _u64, C.POINTER(_u64), _vp]),
    "icx_jpeg_encode_device_batch": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _u64, _vp, _vp, _vp]),
    "icx_hdr_probe": (_i32, [_vp, _sz, C.POINTER(_i32), C.POINTER(_i32)]),
    "icx_hdr_decode": (_i32, [_vp, _vp, _sz, C.POINTER(_vp), C.POINTER(_i32), C.POINTER(_i32), C.POINTER(_i32)]),
    "icx_hdr_batch_create": (_vp, [_vp, _i32, _i32, _i32]),
    "icx_hdr_batch_destroy": (None, [_vp]),
    "icx_hdr_batch_decode": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    "icx_hdr_batch_stage_times": (_i32, [_vp, _vp, _vp, _i32]),
    "icx_jpeg_records": (_i32, [_vp, _i32, _vp, _u64, _vp, _vp, _i32, _i32, _vp, _vp]),
    "icx_checksum64": (_u64, [_vp, _sz]),
    "icx_ctx_device": (_i32, [_vp]),
    "icx_ctx_stream": (_vp, [_vp]),
    "icx_multi_create": (_vp, [_vp, _i32, _i32, _i32]),
    "icx_multi_destroy": (None, [_vp]),
    "icx_multi_decode_host": (_i32, [_vp, _i32, _vp, _vp, _vp, _u64, _vp, _vp]),
    "icx_multi_last_error": (C.c_char_p, [_vp]),
    "icx_multi_gather": (C.c_char_p, [_vp]),
    "icx_multi_shard": (_i32, [_vp, _i32, _i32, _vp]),
    "icx_exr_probe": (_i32, [_vp, _sz, C.POINTER(_i32), C.POINTER(_i32)]),
    "icx_exr_decode": (_i32, [_vp, _vp, _sz, C.POINTER(_vp), C.POINTER(_i32), C.POINTER(_i32)]),
    "icx_exr_decode_device": (_i32, [_vp, _vp, _vp, _sz, _vp, _sz, C.POINTER(_i32), C.POINTER(_i32)]),
    "icx_exr_decode_device_batch": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
}

# icx_record (include/icx.h): per-image result record gathered across devices / ranks
RECORD_DTYPE = np.dtype([("status", "<i4"), ("width", "<i4"), ("height", "<i4"), ("ncomp", "<i4"),
                         ("checksum", "<u8")])

# icx_hdr_result (include/icx.h): Image::readHdr outcomes
HDR_OK, HDR_NOT_RADIANCE, HDR_BAD_HEADER, HDR_MALFORMED, HDR_TRUNCATED, HDR_TOO_LARGE = range(6)
HDR_INTERNAL_ERR = -1

# icx_exr_result (include/icx.h): tinyexr's LoadEXRFromMemory codes
EXR_SUCCESS, EXR_INVALID_MAGIC_NUMBER, EXR_INVALID_EXR_VERSION, EXR_INVALID_ARGUMENT, EXR_INVALID_DATA = 0, -1, -2, -3, -4
EXR_UNSUPPORTED_FORMAT, EXR_INVALID_HEADER, EXR_UNSUPPORTED_FEATURE, EXR_INTERNAL_ERR = -8, -9, -10, -100

WRITE_FUNC = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.c_int)


def _share_hip_runtime_with_torch() -> None:
    """PyTorch-ROCm ships its own libamdhip64/libhsa-runtime64 and loads them by file name
    (RPATH $ORIGIN). Preloading exactly those files first makes libicx's DT_NEEDED
    (libamdhip64.so.7 / libhsa-runtime64.so.1, matched by SONAME) bind to the same runtime,
    so device pointers, streams and RCCL are shared whatever the import order."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    tlib = os.path.join(list(spec.submodule_search_locations)[0], "lib")
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        path = os.path.join(tlib, name)
        if os.path.exists(path):
            C.CDLL(path, mode=C.RTLD_GLOBAL)


def lib():
    """Load libicx.so (raises ICXError if it has not been built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ICXError(f"{LIB_PATH} not built: run `make -C imagecodecs_amd` (hipcc, gfx950)")
        _share_hip_runtime_with_torch()
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            try:
                fn = getattr(L, name)
            except AttributeError:
                if LIB_PATH != _DEFAULT_LIB:
                    continue  # (an older build loaded by ICX_LIB for an A/B: that entry is unusable)
                raise
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def _err(ctx_ptr) -> str:
    msg = lib().icx_last_error(ctx_ptr)
    return msg.decode() if msg else ""


class Context:
    """icx_create(device): a device + HIP stream; also holds njDecode-style state."""

    def __init__(self, device: int = 0):
        self._p = lib().icx_create(device)
        if not self._p:
            raise ICXError("icx_create failed: " + _err(None))
        self.device = device

    def close(self):
        if getattr(self, "_p", None):
            lib().icx_destroy(self._p)
            self._p = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def ptr(self):
        return self._p

    # ---- NanoJPEG-compatible state API (jpeg_dec.h:130-171)
    def nj_init(self):
        lib().icx_nj_init(self._p)

    def nj_done(self):
        lib().icx_nj_done(self._p)

    def nj_decode(self, jpeg: bytes) -> int:
        buf = C.create_string_buffer(bytes(jpeg), max(1, len(jpeg)))
        return lib().icx_nj_decode(self._p, buf, len(jpeg))

    def nj_get_width(self) -> int:
        return lib().icx_nj_get_width(self._p)

    def nj_get_height(self) -> int:
        return lib().icx_nj_get_height(self._p)

    def nj_is_color(self) -> int:
        return lib().icx_nj_is_color(self._p)

    def nj_get_image_size(self) -> int:
        return lib().icx_nj_get_image_size(self._p)

    def nj_get_image(self) -> bytes:
        p = lib().icx_nj_get_image(self._p)
        return C.string_at(p, self.nj_get_image_size()) if p else b""

    # ---- one-shot decode (Image::readJpg)
    def decode(self, jpeg: bytes):
        """-> (code, width, height, ncomp, pixel bytes)."""
        buf = C.create_string_buffer(bytes(jpeg), max(1, len(jpeg)))
        out = C.c_void_p()
        w, h, n = C.c_int(), C.c_int(), C.c_int()
        code = lib().icx_jpeg_decode(self._p, buf, len(jpeg), C.byref(out), C.byref(w), C.byref(h), C.byref(n))
        pix = b""
        if out.value:
            pix = C.string_at(out.value, w.value * h.value * n.value)
            lib().icx_free(out)
        if code == INTERNAL_ERR and _err(self._p):
            raise ICXError(_err(self._p))
        return code, w.value, h.value, n.value, pix

    # ---- encode (tiny_jpeg, jpeg_enc.h:114-160)
    def tje_encode(self, quality: int, width: int, height: int, comps: int, src: bytes):
        """tje_encode_with_func into memory -> bytes, or None on error (tje returns 0)."""
        chunks = []

        @WRITE_FUNC
        def sink(_ctx, data, size):
            chunks.append(C.string_at(data, size))

        buf = C.create_string_buffer(bytes(src), max(1, len(src)))
        ok = lib().icx_tje_encode_with_func(self._p, sink, None, quality, width, height, comps, buf)
        return b"".join(chunks) if ok == 1 else None

    def hdr_decode(self, data: bytes):
        """Image::readHdr (codecs.cpp:706-777) on the GPU -> (code, w, h, rows, float32 (h, w, 4) or
        None). Rows past `rows` (a truncated file) are zero; code is an icx_hdr_result."""
        buf = C.create_string_buffer(bytes(data), max(1, len(data)))
        out = C.c_void_p()
        w, h, rows = C.c_int(), C.c_int(), C.c_int()
        code = lib().icx_hdr_decode(self._p, buf, len(data), C.byref(out), C.byref(w), C.byref(h), C.byref(rows))
        if code == HDR_INTERNAL_ERR:
            raise ICXError("icx_hdr_decode: " + _err(self._p))
        arr = None
        if out.value:
            n = w.value * h.value * 4
            arr = np.frombuffer(C.string_at(out.value, n * 4), np.float32).reshape(h.value, w.value, 4).copy()
            lib().icx_free(out)
        return code, w.value, h.value, rows.value, arr

    def exr_decode(self, data: bytes):
        """Image::readExr's LoadEXRFromMemory (tinyexr.h:6645) on the GPU -> (code, w, h, float32
        (h, w, 4) RGBA or None); code is an icx_exr_result (tinyexr's codes)."""
        buf = C.create_string_buffer(bytes(data), max(1, len(data)))
        out = C.c_void_p()
        w, h = C.c_int(), C.c_int()
        code = lib().icx_exr_decode(self._p, buf, len(data), C.byref(out), C.byref(w), C.byref(h))
        if code == EXR_INTERNAL_ERR:
            raise ICXError("icx_exr_decode: " + _err(self._p))
        arr = None
        if out.value:
            n = w.value * h.value * 4
            arr = np.frombuffer(C.string_at(out.value, n * 4), np.float32).reshape(h.value, w.value, 4).copy()
            lib().icx_free(out)
        return code, w.value, h.value, arr

    def exr_decode_device(self, data: bytes, d_data: int, d_out: int, out_floats: int):
        """icx_exr_decode_device: the file resident on the device at ``d_data`` (its ``len(data)``
        bytes + 16 zero bytes; ``data`` is the host copy the header is planned from), RGBA floats to
        device memory ``d_out`` -> (code, w, h)."""
        buf = C.create_string_buffer(bytes(data), max(1, len(data)))
        w, h = C.c_int(), C.c_int()
        code = lib().icx_exr_decode_device(self._p, buf, C.c_void_p(d_data), len(data), C.c_void_p(d_out), out_floats,
                                           C.byref(w), C.byref(h))
        if code == EXR_INTERNAL_ERR:
            raise ICXError("icx_exr_decode_device: " + _err(self._p))
        return code, w.value, h.value

    def exr_decode_device_batch(self, datas, d_ptrs, d_outs, out_floats):
        """icx_exr_decode_device_batch over n files (host copies ``datas``, device copies at
        ``d_ptrs`` each followed by 16 zero bytes, outputs at ``d_outs`` with ``out_floats`` room
        each) -> (codes, widths, heights) as int32 arrays."""
        n = len(datas)
        bufs = [C.create_string_buffer(bytes(d), max(1, len(d))) for d in datas]
        hp = (C.c_void_p * n)(*[C.cast(b, C.c_void_p) for b in bufs])
        dp = (C.c_void_p * n)(*d_ptrs)
        sz = (C.c_size_t * n)(*[len(d) for d in datas])
        op = (C.c_void_p * n)(*d_outs)
        of = (C.c_size_t * n)(*out_floats)
        codes = np.zeros(n, np.int32)
        ws = np.zeros(n, np.int32)
        hs = np.zeros(n, np.int32)
        rc = lib().icx_exr_decode_device_batch(self._p, n, hp, dp, sz, op, of, codes.ctypes.data, ws.ctypes.data,
                                               hs.ctypes.data)
        if rc == EXR_INTERNAL_ERR:
            raise ICXError("icx_exr_decode_device_batch: " + _err(self._p))
        if rc != 0:
            raise ICXError(f"icx_exr_decode_device_batch: code {rc}")
        return codes, ws, hs

    def png_encode(self, width: int, height: int, d: int, src: bytes):
        """PNG bytes of an RGB8 (d=3) / RGBA8 (d=4) image (png_encoder::saveToFile), or None."""
        chunks = []

        @WRITE_FUNC
        def sink(_ctx, data, size):
            chunks.append(C.string_at(data, size))

        buf = C.create_string_buffer(bytes(src), max(1, len(src)))
        ok = lib().icx_png_encode_with_func(self._p, sink, None, buf, width, height, d)
        return b"".join(chunks) if ok == 1 else None

    def jpeg_encode(self, quality: int, subsampling: int, width: int, height: int, comps: int, src: bytes):
        """C4 extension encode (IJG quality 1..100, subsampling 444|420) -> bytes, or None."""
        chunks = []

        @WRITE_FUNC
        def sink(_ctx, data, size):
            chunks.append(C.string_at(data, size))

        buf = C.create_string_buffer(bytes(src), max(1, len(src)))
        ok = lib().icx_jpeg_encode_with_func(self._p, sink, None, quality, subsampling, width, height, comps, buf)
        return b"".join(chunks) if ok == 1 else None


class PngEncoder:
    """Device-resident PNG encode (icx_png_encoder_* / icx_png_encode_device)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self._p = lib().icx_png_encoder_create(ctx.ptr)
        if not self._p:
            raise ICXError("icx_png_encoder_create failed: " + _err(ctx.ptr))

    def close(self):
        if getattr(self, "_p", None):
            lib().icx_png_encoder_destroy(self._p)
            self._p = None

    def __del__(self):
        self.close()

    def encode_device(self, width, height, d, d_src, d_out, out_cap, stream=0):
        """-> (icx_result, file size in bytes)."""
        n = C.c_uint64()
        rc = lib().icx_png_encode_device(self._p, width, height, d, d_src, d_out, out_cap, C.byref(n), stream or None)
        if rc not in (OK, OUT_OF_MEM):
            raise ICXError(f"icx_png_encode_device -> {rc}: {_err(self.ctx.ptr)}")
        return rc, int(n.value)

    def encode_device_batch(self, width, height, d, d_srcs, d_out, out_stride, stream=0):
        """n device images (list of device addresses) -> files at d_out + i*out_stride; returns
        (statuses, sizes) as numpy arrays (icx_png_encode_device_batch)."""
        n = len(d_srcs)
        srcs = (C.c_void_p * max(1, n))(*d_srcs)
        sizes = np.zeros(max(1, n), np.uint64)
        status = np.zeros(max(1, n), np.int32)
        rc = lib().icx_png_encode_device_batch(self._p, n, width, height, d, srcs, d_out, out_stride,
                                               sizes.ctypes.data, status.ctypes.data, stream or None)
        if rc != OK:
            raise ICXError(f"icx_png_encode_device_batch -> {rc}: {_err(self.ctx.ptr)}")
        return status[:n], sizes[:n].astype(np.int64)

    def stage_times(self) -> dict:
        """Summed per-stage ms since the previous call (icx_png_encoder_stage_times)."""
        names = (C.c_char_p * 8)()
        ms = (C.c_float * 8)()
        k = lib().icx_png_encoder_stage_times(self._p, names, ms, 8)
        return {names[i].decode(): float(ms[i]) for i in range(k)}


class Encoder:
    """Device-resident JPEG encode (icx_encoder_* / icx_jpeg_encode_device); pointers are device
    addresses (ints) on the context's device."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self._p = lib().icx_encoder_create(ctx.ptr)
        if not self._p:
            raise ICXError("icx_encoder_create failed: " + _err(ctx.ptr))

    def close(self):
        if getattr(self, "_p", None):
            lib().icx_encoder_destroy(self._p)
            self._p = None

    def __del__(self):
        self.close()

    def encode_device(self, quality, subsampling, width, height, comps, d_src, d_out, out_cap, stream=0):
        """-> (icx_result, file size in bytes)."""
        n = C.c_uint64()
        rc = lib().icx_jpeg_encode_device(self._p, quality, subsampling, width, height, comps, d_src, d_out,
                                          out_cap, C.byref(n), stream or None)
        if rc not in (OK, OUT_OF_MEM):
            raise ICXError(f"icx_jpeg_encode_device -> {rc}: {_err(self.ctx.ptr)}")
        return rc, int(n.value)

    def encode_device_batch(self, quality, subsampling, width, height, comps, d_srcs, d_out, out_stride, stream=0):
        """n device images (list of device addresses) -> files at d_out + i*out_stride;
        returns (statuses, sizes) as numpy arrays (icx_jpeg_encode_device_batch)."""
        n = len(d_srcs)
        srcs = (C.c_void_p * max(1, n))(*d_srcs)
        sizes = np.zeros(max(1, n), np.uint64)
        status = np.zeros(max(1, n), np.int32)
        rc = lib().icx_jpeg_encode_device_batch(self._p, n, quality, subsampling, width, height, comps, srcs, d_out,
                                                out_stride, sizes.ctypes.data, status.ctypes.data, stream or None)
        if rc != OK:
            raise ICXError(f"icx_jpeg_encode_device_batch -> {rc}: {_err(self.ctx.ptr)}")
        return status[:n], sizes[:n].astype(np.int64)

    def stage_times(self) -> dict:
        """Summed per-stage ms since the previous call (icx_encoder_stage_times)."""
        names = (C.c_char_p * 8)()
        ms = (C.c_float * 8)()
        k = lib().icx_encoder_stage_times(self._p, names, ms, 8)
        return {names[i].decode(): float(ms[i]) for i in range(k)}


def probe(jpeg: bytes):
    """Host header walk (njDecode through SOS) -> (code, width, height, ncomp)."""
    w, h, n = C.c_int(), C.c_int(), C.c_int()
    buf = C.create_string_buffer(bytes(jpeg), max(1, len(jpeg)))
    code = lib().icx_jpeg_probe(buf, len(jpeg), C.byref(w), C.byref(h), C.byref(n))
    return code, w.value, h.value, n.value


def records_device(ctx: "Context", n, d_out, out_stride, d_status, d_dims, max_width, max_height, d_records,
                   stream=0):
    """icx_jpeg_records: per-image {status, w, h, ncomp, checksum64} of a batch call's outputs,
    computed on the device into d_records (n x 24 bytes, RECORD_DTYPE)."""
    rc = lib().icx_jpeg_records(ctx.ptr, n, d_out, out_stride, d_status, d_dims, max_width, max_height, d_records,
                                stream or None)
    if rc != OK:
        raise ICXError(f"icx_jpeg_records -> {rc}: {_err(ctx.ptr)}")


def checksum64(data: bytes) -> int:
    """icx_checksum64 on the host (the records' checksum of a decoded image's bytes)."""
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    return int(lib().icx_checksum64(buf, len(data)))


def multi_shard(sizes, ndev: int) -> np.ndarray:
    """icx_multi_shard: the device index each image goes to (greedy longest-first by size)."""
    n = len(sizes)
    sz = (C.c_size_t * max(1, n))(*[int(x) for x in sizes])
    out = np.zeros(max(1, n), np.int32)
    if lib().icx_multi_shard(sz, n, ndev, out.ctypes.data) != OK:
        raise ICXError("icx_multi_shard failed")
    return out[:n]


class Multi:
    """Multi-GPU decode in one process (icx_multi_*): the batch is split over `devices` by
    compressed size, one host thread per device; the records are gathered over RCCL when the
    devices are distinct (`gather` says which), the pixels copied to host memory."""

    def __init__(self, devices, max_width: int, max_height: int):
        devs = (C.c_int * len(devices))(*devices)
        self._p = lib().icx_multi_create(devs, len(devices), max_width, max_height)
        if not self._p:
            raise ICXError("icx_multi_create failed: " + _err(None))
        self.devices = list(devices)
        self.max_width, self.max_height = max_width, max_height

    @property
    def gather(self) -> str:
        return lib().icx_multi_gather(self._p).decode()

    def close(self):
        if getattr(self, "_p", None):
            lib().icx_multi_destroy(self._p)
            self._p = None

    def __del__(self):
        self.close()

    def decode_host(self, jpegs, want_pixels: bool = True):
        """-> (records (RECORD_DTYPE array), shard_of (int32 array), pixels list or None)."""
        n = len(jpegs)
        stride = self.max_width * self.max_height * 3
        bufs = [C.create_string_buffer(bytes(j), max(1, len(j))) for j in jpegs]
        ptrs = (C.c_void_p * max(1, n))(*[C.cast(b, C.c_void_p) for b in bufs])
        sizes = (C.c_size_t * max(1, n))(*[len(j) for j in jpegs])
        outs_np = [np.empty(stride, np.uint8) for _ in range(n)] if want_pixels else None
        outs = (C.c_void_p * max(1, n))(*[o.ctypes.data for o in outs_np]) if want_pixels else None
        rec = np.zeros(max(1, n), RECORD_DTYPE)
        shard_of = np.zeros(max(1, n), np.int32)
        rc = lib().icx_multi_decode_host(self._p, n, ptrs, sizes, outs, stride, rec.ctypes.data, shard_of.ctypes.data)
        if rc != OK:
            msg = lib().icx_multi_last_error(self._p)
            raise ICXError(f"icx_multi_decode_host -> {rc}: {msg.decode() if msg else ''}")
        pix = None
        if want_pixels:
            pix = []
            for i in range(n):
                r = rec[i]
                nb = int(r["width"]) * int(r["height"]) * int(r["ncomp"])
                pix.append(outs_np[i][:nb] if r["status"] == OK else None)
        return rec[:n], shard_of[:n], pix


class Batch:
    """Device-resident batched decode (icx_jpeg_batch_*). Inputs/outputs are device pointers
    (ints) -- e.g. torch CUDA tensors' data_ptr() -- on the context's device."""

    def __init__(self, ctx: Context, max_images: int, max_width: int, max_height: int, group: int = 0):
        self.ctx = ctx
        self._p = lib().icx_batch_create(ctx.ptr, max_images, max_width, max_height, group)
        if not self._p:
            raise ICXError("icx_batch_create failed: " + _err(ctx.ptr))
        self.max_images, self.max_width, self.max_height = max_images, max_width, max_height

    def close(self):
        if getattr(self, "_p", None):
            lib().icx_batch_destroy(self._p)
            self._p = None

    def __del__(self):
        self.close()

    def decode_device(self, n, d_data, d_offsets, d_sizes, d_out, out_stride, d_status, d_dims, stream=0):
        rc = lib().icx_jpeg_batch_decode(self._p, n, d_data, d_offsets, d_sizes, d_out, out_stride,
                                         d_status, d_dims, stream or None)
        if rc != OK:
            raise ICXError(f"icx_jpeg_batch_decode -> {rc}: {_err(self.ctx.ptr)}")

    def decode_host(self, jpegs, out_stride=None):
        """Decode a list of bytes objects -> list of (code, w, h, ncomp, np.ndarray|None)."""
        n = len(jpegs)
        out_stride = out_stride or self.max_width * self.max_height * 3
        bufs = [C.create_string_buffer(bytes(j), max(1, len(j))) for j in jpegs]
        ptrs = (C.c_void_p * n)(*[C.cast(b, C.c_void_p) for b in bufs])
        sizes = (C.c_size_t * n)(*[len(j) for j in jpegs])
        outs_np = [np.empty(out_stride, np.uint8) for _ in range(n)]
        outs = (C.c_void_p * n)(*[o.ctypes.data for o in outs_np])
        status = np.zeros(n, np.int32)
        dims = np.zeros((n, 3), np.int32)
        rc = lib().icx_jpeg_batch_decode_host(self._p, n, ptrs, sizes, outs, out_stride,
                                              status.ctypes.data, dims.ctypes.data)
        if rc != OK:
            raise ICXError(f"icx_jpeg_batch_decode_host -> {rc}: {_err(self.ctx.ptr)}")
        res = []
        for i in range(n):
            w, h, c = (int(x) for x in dims[i])
            pix = outs_np[i][: w * h * c].reshape(h, w, c) if status[i] == OK else None
            res.append((int(status[i]), w, h, c, pix))
        return res

    def path_stats(self) -> dict:
        a, b, c = C.c_int(), C.c_int(), C.c_int()
        lib().icx_batch_path_stats(self._p, C.byref(a), C.byref(b), C.byref(c))
        return {"parallel": a.value, "fallback": b.value, "sequential": c.value}

    @property
    def group(self) -> int:
        """Images per workspace group (icx_batch_group)."""
        return int(lib().icx_batch_group(self._p))

    def groups_per_call(self, n: int) -> int:
        """Groups a call of n images takes (icx_batch_groups): each per-group kernel launches once per group."""
        return int(lib().icx_batch_groups(self._p, n))

    def stage_times(self) -> dict:
        names = (C.c_char_p * 16)()
        ms = (C.c_float * 16)()
        k = lib().icx_batch_stage_times(self._p, names, ms, 16)
        return {names[i].decode(): float(ms[i]) for i in range(k)}


def hdr_probe(data: bytes):
    """Host header walk of readHdr (codecs.cpp:713-750) -> (code, width, height)."""
    w, h = C.c_int(), C.c_int()
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    code = lib().icx_hdr_probe(buf, len(data), C.byref(w), C.byref(h))
    return code, w.value, h.value


def exr_probe(data: bytes):
    """Host header / offset-table / chunk-header walk of LoadEXRFromMemory -> (code, width, height)."""
    w, h = C.c_int(), C.c_int()
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    code = lib().icx_exr_probe(buf, len(data), C.byref(w), C.byref(h))
    return code, w.value, h.value


class HdrBatch:
    """Device-resident batched Radiance .hdr decode (icx_hdr_batch_*): image i is
    d_data[d_offsets[i] .. + d_sizes[i]); 4 floats per pixel at d_out + i*out_stride floats."""

    def __init__(self, ctx: Context, max_images: int, max_width: int, max_height: int):
        self.ctx = ctx
        self._p = lib().icx_hdr_batch_create(ctx.ptr, max_images, max_width, max_height)
        if not self._p:
            raise ICXError("icx_hdr_batch_create failed: " + _err(ctx.ptr))
        self.max_images, self.max_width, self.max_height = max_images, max_width, max_height

    def close(self):
        if getattr(self, "_p", None):
            lib().icx_hdr_batch_destroy(self._p)
            self._p = None

    def __del__(self):
        self.close()

    def decode_device(self, n, d_data, d_offsets, d_sizes, d_out, out_stride, d_status, d_dims, stream=0):
        rc = lib().icx_hdr_batch_decode(self._p, n, d_data, d_offsets, d_sizes, d_out, out_stride,
                                        d_status, d_dims, stream or None)
        if rc != HDR_OK:
            raise ICXError(f"icx_hdr_batch_decode -> {rc}: {_err(self.ctx.ptr)}")

    def stage_times(self) -> dict:
        names = (C.c_char_p * 8)()
        ms = (C.c_float * 8)()
        k = lib().icx_hdr_batch_stage_times(self._p, names, ms, 8)
        return {names[i].decode(): float(ms[i]) for i in range(k)}


class Image:
    """ImageCodecs::Image (codecs.h:16-103) for the JPEG hot path.

    read()/write() dispatch on the lower-cased extension like Image::read/write
    (codecs.cpp:53-122): read .jpg/.jpeg (readJpg) and .hdr (readHdr: d = 4, type FLOAT, the
    floats' bytes in pixels_), write .jpg/.jpeg and .png. Other extensions raise ValueError (the
    reference's std::invalid_argument for unknown types)."""

    UBYTE, USHORT, FLOAT = range(3)  # ImageCodecs::Type (codecs.h:14)
    _ctx = None

    def __init__(self):
        self.h_ = self.w_ = self.d_ = 0
        self.pixels_ = None
        self.type_ = Image.UBYTE

    @classmethod
    def context(cls):
        if cls._ctx is None:
            cls._ctx = Context(0)
        return cls._ctx

    def read(self, filepath: str):
        ext = os.path.splitext(filepath)[1].lower()
        if ext == ".hdr":
            self._read_hdr(filepath)
            return
        if ext == ".exr":
            self._read_exr(filepath)
            return
        if ext not in (".jpg", ".jpeg"):
            raise ValueError("Cannot parse filetype")
        data = open(filepath, "rb").read()
        code, w, h, n, pix = self.context().decode(data)
        if code != OK:
            raise RuntimeError("Error decoding the input file.\n")  # codecs.cpp:836
        self.w_, self.h_, self.d_ = w, h, n
        self.pixels_ = np.frombuffer(pix, np.uint8).copy()
        self.type_ = Image.UBYTE

    def _read_hdr(self, filepath: str):
        """readHdr (codecs.cpp:706-777). A truncated file keeps its decoded rows (the rest are
        zero; the reference leaves them uninitialised); header errors and run-length data the
        reference cannot decode raise RuntimeError("Invalid file format") (:732, :748)."""
        data = open(filepath, "rb").read()
        code, w, h, rows, px = self.context().hdr_decode(data)
        if code not in (HDR_OK, HDR_TRUNCATED):
            raise RuntimeError("Invalid file format")
        self.w_, self.h_, self.d_ = w, h, 4
        self.pixels_ = px.reshape(-1).view(np.uint8).copy()
        self.type_ = Image.FLOAT

    def _read_exr(self, filepath: str):
        """readExr (codecs.cpp:464-493): LoadEXRFromMemory -> d = 4, type FLOAT, the floats' bytes in
        pixels_; a failure raises RuntimeError("Could not load .exr") (:489). (The reference reads
        the file with a loop that appends one extra byte, ifile.get()'s EOF, :468-471; tinyexr
        ignores bytes past the last chunk, so the result is the same.)"""
        data = open(filepath, "rb").read()
        code, w, h, px = self.context().exr_decode(data + b"\xff")
        if code != EXR_SUCCESS:
            raise RuntimeError("Could not load .exr")
        self.w_, self.h_, self.d_ = w, h, 4
        self.pixels_ = px.reshape(-1).view(np.uint8).copy()
        self.type_ = Image.FLOAT

    def write(self, filepath: str):
        ext = os.path.splitext(filepath)[1].lower()
        if ext == ".png":  # writePng -> png_encoder::saveToFile (codecs.cpp:1022-1025)
            out = self.context().png_encode(self.w_, self.h_, self.d_, self.pixels_.tobytes())
        elif ext in (".jpg", ".jpeg"):
            out = self.context().tje_encode(3, self.w_, self.h_, self.d_, self.pixels_.tobytes())  # codecs.cpp:853
        else:
            raise ValueError("Cannot parse filetype")
        with open(filepath, "wb") as f:
            if out is not None:
                f.write(out)

    def load(self, pixels, w: int, h: int, channels: int):
        self.pixels_ = np.ascontiguousarray(pixels, np.uint8).reshape(-1)
        self.w_, self.h_, self.d_ = w, h, channels
        self.type_ = Image.UBYTE

    def rows(self):
        return self.h_

    def cols(self):
        return self.w_

    def channels(self):
        return self.d_

    def empty(self):
        return self.h_ == 0 or self.w_ == 0 or self.d_ == 0 or self.pixels_ is None

    def byteSize(self):
        return 4 if self.type_ == Image.FLOAT else 2 if self.type_ == Image.USHORT else 1

    def type(self):
        return self.type_

    def totalBytes(self):
        return self.w_ * self.h_ * self.d_ * self.byteSize()

    def data(self):
        return self.pixels_
