"""include/imagecodecs/codecs.h: the reference's ImageCodecs::Image read/write usage, compiled
with g++ against libicx.so (tests/cxx/codecs_demo.cpp).

CPU: the header builds and links; unknown extensions throw std::invalid_argument as in
codecs.cpp:80-83; a JPEG read without a GPU throws (no CPU fallback).
GPU: Image::read of data/test.jpg is bit-exact to the NanoJPEG golden; Image::write produces
the byte stream tiny_jpeg's tje_encode_to_file (quality 3) produces for those pixels (oracle).
"""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

LIBDIR = os.path.join(ROOT, "imagecodecs_amd", "lib")


@pytest.fixture(scope="module")
def demo(tmp_path_factory):
    import imagecodecs_amd as icx
    icx.build()
    exe = str(tmp_path_factory.mktemp("cxx") / "codecs_demo")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cxx", "codecs_demo.cpp"), "-L" + LIBDIR, "-licx",
                    "-Wl,-rpath," + LIBDIR, "-o", exe], check=True)
    return exe


def run(exe, *args):
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=300)


def test_dropin_error_behaviour(demo):
    r = run(demo, "errors", os.path.join(GOLDEN, "test.jpg"))
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[:2] == ["invalid_argument ok", "invalid_argument ok"]
    # with a GPU the read succeeds; without one it must fail loudly, never fall back to the CPU
    assert lines[2] == "read ok" or ("runtime_error" in lines[2] and "no HIP device" in lines[2])


@pytest.mark.gpu
def test_dropin_read_bit_exact(demo, tmp_path):
    out = str(tmp_path / "t.rgb")
    r = run(demo, "read", os.path.join(GOLDEN, "test.jpg"), out)
    assert r.returncode == 0, r.stderr
    raw = open(out, "rb").read()
    w, h, d = np.frombuffer(raw[:12], np.int32)
    assert (w, h, d) == (499, 289, 3)
    assert hashlib.sha256(raw[12:]).hexdigest() == "dc95c1dd9716f324b0eeaffc3e739f832e925112d2f80b37d5ca13549f89fff9"


@pytest.mark.gpu
def test_dropin_write_matches_tiny_jpeg(demo, tmp_path):
    from oracle import pyoracle
    dst = str(tmp_path / "rt.jpg")
    r = run(demo, "roundtrip", os.path.join(GOLDEN, "test.jpg"), dst)
    assert r.returncode == 0, r.stdout + r.stderr
    code, w, h, n, pix = pyoracle.decode(open(os.path.join(GOLDEN, "test.jpg"), "rb").read())
    assert code == 0
    assert open(dst, "rb").read() == pyoracle.tje_encode(3, w, h, 3, pix)


@pytest.mark.gpu
def test_dropin_read_hdr(demo, tmp_path):
    """Image::read(".hdr") (readHdr, codecs.cpp:706-777): d = 4 floats per pixel, bit-identical
    to the oracle on the reference's data/test.hdr."""
    from oracle import pyoracle
    src = os.path.join(GOLDEN, "test.hdr")
    out = str(tmp_path / "t.f32")
    r = run(demo, "read", src, out)
    assert r.returncode == 0, r.stderr
    raw = open(out, "rb").read()
    w, h, d = np.frombuffer(raw[:12], np.int32)
    assert (w, h, d) == (499, 289, 4)
    code, _, _, rows, arr = pyoracle.hdr_decode(open(src, "rb").read())
    assert code == 0 and rows == 289
    assert raw[12:] == arr.tobytes()


def _utils_expect(px: np.ndarray):
    """numpy restatement of the reference's flip (codecs.cpp:162-196), then swapBR (:198-251),
    then idx at (0,0,0), (h-1,w-1,d-1), (h/2,1,1) on the swapped image."""
    f = px[::-1].copy()
    s = f.copy()
    if s.shape[2] >= 3:
        s[..., [0, 2]] = s[..., [2, 0]]
    h, w, d = s.shape
    pts = [s[0, 0, 0], s[h - 1, w - 1, d - 1], s[h // 2, 1, 1]]
    return f, s, pts


def _utils_read(path, dtype):
    raw = open(path, "rb").read()
    w, h, d, bs = np.frombuffer(raw[:16], np.int32)
    n = w * h * d * bs
    f = np.frombuffer(raw[16:16 + n], dtype).reshape(h, w, d)
    s = np.frombuffer(raw[16 + n:16 + 2 * n], dtype).reshape(h, w, d)
    pts = np.frombuffer(raw[16 + 2 * n:], dtype)
    return f, s, list(pts)


def test_dropin_utils_on_loaded_buffer(demo, tmp_path):
    """flip / swapBR / idx<T> (codecs.h:80, 82-88, 98) on an adopted UBYTE buffer (no GPU)."""
    out = str(tmp_path / "u.bin")
    r = run(demo, "loadutils", out)
    assert r.returncode == 0, r.stderr
    px = ((np.arange(60) * 7 + 3) & 255).astype(np.uint8).reshape(3, 5, 4)
    f, s, pts = _utils_read(out, np.uint8)
    ef, es, epts = _utils_expect(px)
    np.testing.assert_array_equal(f, ef)
    np.testing.assert_array_equal(s, es)
    assert pts == epts


@pytest.mark.gpu
@pytest.mark.parametrize("src", ["test.jpg", "test.hdr"])
def test_dropin_utils_after_gpu_read(demo, tmp_path, src):
    """The pixel utilities after a GPU read(): UBYTE (JPEG) and FLOAT (HDR) images."""
    from oracle import pyoracle
    out = str(tmp_path / "u.bin")
    r = run(demo, "utils", os.path.join(GOLDEN, src), out)
    assert r.returncode == 0, r.stderr
    data = open(os.path.join(GOLDEN, src), "rb").read()
    if src.endswith(".jpg"):
        code, w, h, n, pix = pyoracle.decode(data)
        px, dt = np.frombuffer(pix, np.uint8).reshape(h, w, n), np.uint8
    else:
        code, w, h, rows, arr = pyoracle.hdr_decode(data)
        px, dt = np.asarray(arr, np.float32).reshape(h, w, 4), np.float32
    f, s, pts = _utils_read(out, dt)
    ef, es, epts = _utils_expect(px)
    np.testing.assert_array_equal(f, ef)
    np.testing.assert_array_equal(s, es)
    assert [float(a) for a in pts] == [float(b) for b in epts]
