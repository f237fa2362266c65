"""CPU tests of the OpenEXR read (Image::readExr -> tinyexr LoadEXRFromMemory, tinyexr.h:6645):
the oracle (oracle/exr_oracle.py) against the reference's own tinyexr compiled in place
(oracle/_ref/libref_exr.so: tinyexr's zlib route, TINYEXR_USE_MINIZ 0, tinyexr.h:109-112, 664-671)
on every fixture and on seeded damage; the fixtures against the manifest; and the GPU path's own
host plan, decompressors and per-pixel gather (icx_exr_plan.h / icx_exr_core.h, run on the CPU by
tests/emu/exr_emu.cpp) against the oracle, bit for bit. Parity: pinned to the reference build for
NONE / RLE / PIZ chunks and all header and offset logic; ZIP / ZIPS inflate through the system
zlib in place of the reference's un-vendored miniz (both check the Adler-32, so a valid stream
inflates to the same bytes). PIZ is in scope: the reference builds tinyexr with TINYEXR_USE_PIZ 1
(tinyexr.h:126-128, codecs.cpp:27-29)."""
import ctypes as C
import hashlib
import json
import os
import subprocess
import sys
import zlib

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from oracle import exr_oracle as O
from tools import exrwrite as W

MAN = json.load(open(os.path.join(GOLDEN, "exr_manifest.json")))
EXR = os.path.join(GOLDEN, "exr")
_L = None


def emu():
    global _L
    if _L is None:
        d = os.path.join(ROOT, "tests", "emu")
        subprocess.run(["make", "-s", "-C", d, "libexremu.so"], check=True)
        import imagecodecs_amd
        imagecodecs_amd._share_hip_runtime_with_torch()
        L = C.CDLL(os.path.join(d, "libexremu.so"))
        L.emu_exr_decode.restype = C.c_int
        L.emu_exr_decode.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.emu_exr_inflate.restype = C.c_int
        L.emu_exr_inflate.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
        L.emu_exr_inflate_ring.restype = C.c_int
        L.emu_exr_inflate_ring.argtypes = L.emu_exr_inflate.argtypes
        _L = L
    return _L


def emu_decode(data: bytes, cap=1 << 22):
    out = np.zeros(cap * 4, np.uint32)
    w, h = C.c_int(), C.c_int()
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    code = emu().emu_exr_decode(buf, len(data), out.ctypes.data, cap, C.byref(w), C.byref(h))
    img = out[: w.value * h.value * 4].reshape(h.value, w.value, 4) if code == 0 else None
    return code, w.value, h.value, img


def emu_inflate(src: bytes, cap: int, ring: bool = False):
    """ring: the GPU's form (16 KiB LDS ring, farther matches read back from the output)."""
    dst = np.zeros(max(1, cap), np.uint8)
    n = C.c_int64()
    buf = C.create_string_buffer(bytes(src), max(1, len(src)))
    f = emu().emu_exr_inflate_ring if ring else emu().emu_exr_inflate
    ok = f(buf, len(src), dst.ctypes.data, cap, C.byref(n))
    return dst[: n.value].tobytes() if ok else None


def sha(img):
    return hashlib.sha256(np.ascontiguousarray(img).view(np.uint32).tobytes()).hexdigest()


@pytest.mark.parametrize("name", sorted(MAN))
def test_fixture_oracle_manifest(name):
    """The committed fixtures decode to the manifest's result with the oracle (pins the files)."""
    code, w, h, img = O.decode(open(os.path.join(EXR, name), "rb").read())
    e = MAN[name]
    assert (code, w, h) == (e["code"], e["w"], e["h"])
    assert (sha(img) if img is not None else None) == e["sha256"]


@pytest.mark.parametrize("name", sorted(MAN))
def test_gpu_path_logic_matches_oracle(name):
    """The GPU path's plan / decompressors / gather, run on the CPU, give the oracle's code and
    bits on every fixture."""
    data = open(os.path.join(EXR, name), "rb").read()
    code, w, h, img = emu_decode(data)
    e = MAN[name]
    assert (code, w, h) == (e["code"], e["w"], e["h"]), name
    if code == 0:
        assert sha(img) == e["sha256"], name


def _zstreams():
    rng = np.random.default_rng(3)
    out = []
    for n in (0, 1, 7, 300, 5000, 70000, 200000):
        for kind in ("rand", "text", "runs"):
            if kind == "rand":
                raw = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            elif kind == "text":
                raw = (b"the quick brown fox jumps over the lazy dog %d " % n) * (n // 40 + 1)
                raw = raw[:n]
            else:
                raw = np.repeat(rng.integers(0, 4, n // 50 + 1, dtype=np.uint8), 50)[:n].tobytes()
            for level in (0, 1, 6, 9):
                out.append((raw, zlib.compress(raw, level)))
            co = zlib.compressobj(6, zlib.DEFLATED, 15, 9, zlib.Z_FIXED)
            out.append((raw, co.compress(raw) + co.flush()))
    return out


@pytest.mark.parametrize("ring", [False, True])
def test_inflate_matches_zlib(ring):
    """exr_inflate == zlib on stored, fixed and dynamic blocks, windows past 32 KiB, and an output
    capacity of exactly / one short of / more than the data; with the full window and in the
    GPU's form (16 KiB ring, matches from farther back read from the output)."""
    for raw, z in _zstreams():
        assert emu_inflate(z, len(raw), ring) == raw
        assert emu_inflate(z, len(raw) + 100, ring) == raw
        if raw:
            assert emu_inflate(z, len(raw) - 1, ring) is None  # (mz_uncompress: MZ_BUF_ERROR)


def test_inflate_far_matches_ring():
    """Streams whose matches reach 16-32 KiB back (a 24 KiB random block repeated, odd lengths): the
    GPU's ring form reads them from the output, bit-exact to zlib."""
    rng = np.random.default_rng(11)
    for size, tail in ((24 << 10, 7), ((20 << 10) + 3, 1), (30 << 10, 5)):
        block = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        raw = block + block + block[: size // 3 + tail]
        z = zlib.compress(raw, 9)
        assert emu_inflate(z, len(raw), True) == raw
        assert emu_inflate(z, len(raw), False) == raw


@pytest.mark.parametrize("ring", [False, True])
def test_inflate_corrupt_streams(ring):
    """Truncated streams, bad check bits, a preset dictionary, a wrong Adler-32 and random byte
    damage: fail whenever zlib fails, else produce zlib's bytes (both window forms)."""
    rng = np.random.default_rng(4)
    agree = total = 0
    for raw, z in _zstreams()[::3]:
        assert emu_inflate(z[:-1], len(raw) + 10, ring) is None
        assert emu_inflate(z[: len(z) // 2], len(raw) + 10, ring) is None or len(raw) == 0
        assert emu_inflate(bytes([z[0], z[1] ^ 1]) + z[2:], len(raw), ring) is None
        assert emu_inflate(bytes([z[0], z[1] | 0x20]) + z[2:], len(raw), ring) is None
        assert emu_inflate(z[:-1] + bytes([z[-1] ^ 0x40]), len(raw), ring) is None
        for _ in range(20):
            b = bytearray(z)
            b[int(rng.integers(2, len(b)))] ^= int(rng.integers(1, 256))
            d = zlib.decompressobj()
            try:
                ref = d.decompress(bytes(b), len(raw) + 64)
                ref = ref if d.eof and not d.unconsumed_tail else None
            except zlib.error:
                ref = None
            got = emu_inflate(bytes(b), len(raw) + 64, ring)
            total += 1
            agree += got == ref
    # (the two decoders differ only on streams zlib and miniz themselves disagree about: an
    # incomplete one-symbol code, a window size field above 32 KiB)
    assert agree >= total - 2, (agree, total)


@pytest.mark.parametrize("seed", range(4))
def test_random_damage_same_result(seed):
    """Random byte damage to header, offset table and chunks of small files: the GPU path's
    logic returns the oracle's code and, when it decodes, the oracle's bits."""
    rng = np.random.default_rng(100 + seed)
    names = [n for n in sorted(MAN) if MAN[n]["code"] == 0 and "wide" not in n]
    for k in range(60):
        data = bytearray(open(os.path.join(EXR, names[int(rng.integers(0, len(names)))]), "rb").read())
        for _ in range(1 + k % 3):
            data[int(rng.integers(0, len(data)))] ^= int(rng.integers(1, 256))
        data = bytes(data)
        oc, ow, oh, oimg = O.decode(data)
        ec, ew, eh, eimg = emu_decode(data)
        assert (ec, ew, eh) == (oc, ow, oh), (seed, k)
        if oc == 0:
            assert np.array_equal(eimg, oimg.view(np.uint32)), (seed, k)


@pytest.mark.parametrize("seed", range(3))
def test_piz_and_levels_damage_same_result(seed):
    """Random damage to PIZ chunks (range header, Huffman table and codes -- tinyexr ignores the
    Huffman decoder's failures and keeps what it decoded) and to mip- / rip-mapped files: the GPU
    path's logic returns the oracle's code and bits."""
    rng = np.random.default_rng(200 + seed)
    names = [n for n in sorted(MAN) if MAN[n]["code"] == 0 and ("piz" in n or n.startswith(("mip", "rip")))
             and "w16" not in n and "longcodes" not in n]
    for k in range(40):
        data = bytearray(open(os.path.join(EXR, names[int(rng.integers(0, len(names)))]), "rb").read())
        lo = len(data) // 3 if k % 2 else 0  # (half of the draws hit the chunk data only)
        for _ in range(1 + k % 4):
            data[int(rng.integers(lo, len(data)))] ^= int(rng.integers(1, 256))
        data = bytes(data)
        oc, ow, oh, oimg = O.decode(data)
        ec, ew, eh, eimg = emu_decode(data)
        assert (ec, ew, eh) == (oc, ow, oh), (seed, k)
        if oc == 0:
            assert np.array_equal(eimg, oimg.view(np.uint32)), (seed, k)


def test_piz_wavelet_inverse():
    """wav2Decode (oracle) inverts wav2Encode (writer) for 14- and 16-bit data, odd sizes and
    strides 1 and 2 (the two halves of a FLOAT / UINT sample)."""
    rng = np.random.default_rng(9)
    for nx, ny in ((1, 1), (7, 3), (32, 32), (33, 17), (64, 5), (5, 64)):
        for sz in (1, 2):
            for top in (1 << 14, 1 << 16):
                a = rng.integers(0, top, nx * ny * sz, dtype=np.int64).astype(np.uint16)
                b = a.copy()
                for j in range(sz):
                    W.wav2_encode(b, j, nx, sz, ny, nx * sz, top - 1)
                for j in range(sz):
                    O.wav2_decode(b, j, nx, sz, ny, nx * sz, top - 1)
                assert np.array_equal(a, b), (nx, ny, sz, top)


def test_writer_roundtrip_every_layout():
    """tools/exrwrite.py -> oracle returns the written samples (HALF via float32, UINT bits,
    DECREASING_Y scanlines flipped as tinyexr places them)."""
    rng = np.random.default_rng(7)
    h, w = 19, 23
    R, G = (rng.standard_normal((h, w)).astype(np.float16) for _ in range(2))
    B = rng.standard_normal((h, w)).astype(np.float32)
    A = rng.integers(0, 2**32, (h, w), dtype=np.uint32)
    exp = np.stack([R.astype(np.float32), G.astype(np.float32), B, A.view(np.float32)], -1).view(np.uint32)
    for comp in (W.NONE, W.RLE, W.ZIPS, W.ZIP, W.PIZ):
        for tiles, levels in ((None, 0), ((8, 4), 0), ((32, 32), 0), ((8, 4), 1), ((16, 8), 2)):
            data = W.write_exr([("R", R), ("G", G), ("B", B), ("A", A)], compression=comp, tiles=tiles, origin=(2, -7),
                               levels=levels, rounding=levels == 2)
            code, ww, hh, img = O.decode(data)
            assert code == 0 and (ww, hh) == (w, h)
            assert np.array_equal(img.view(np.uint32), exp)
            lo = W.write_exr([("R", R), ("G", G), ("B", B), ("A", A)], compression=comp, line_order=1)
            assert np.array_equal(O.decode(lo)[3].view(np.uint32), exp[::-1])


REFERENCE = "/root/reference/tinyexr.h"


def _exrref(*args):
    """tests/exrref.py in its own process (the allocator settings it needs act at start-up)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    env = dict(os.environ, GLIBC_TUNABLES="glibc.malloc.tcache_count=0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "exrref.py"), *args], env=env, check=True,
                       capture_output=True, text=True, timeout=600)
    return json.loads(r.stdout)


@pytest.mark.skipif(not os.path.exists(REFERENCE), reason="the reference (container only)")
def test_oracle_vs_live_tinyexr_fixtures():
    """Every fixture: the reference build's code and every float it defines equal the oracle's;
    the rows it leaves uninitialised are exactly the manifest's (the oracle writes 0.0 there)."""
    rep = _exrref("fixtures")
    assert rep["checked"] == len(MAN)
    assert rep["failures"] == {}
    for name, e in MAN.items():
        assert rep["undefined_rows"].get(name, []) == e["ref_undefined_rows"], name


@pytest.mark.skipif(not os.path.exists(REFERENCE), reason="the reference (container only)")
@pytest.mark.parametrize("seed", [1, 2])
def test_oracle_vs_live_tinyexr_damage(seed):
    """Seeded variants of every fixture (version flags: tiled / deep / multi-part bits flipped;
    1-3 bytes replaced; truncation) give the reference's code and floats."""
    rep = _exrref("fuzz", str(seed), "4")
    assert rep["checked"] > 8 * len(MAN)
    assert rep["failures"] == {}


def test_multipart_and_deep_flags_reach_only_tile_offsets():
    """LoadEXRFromMemory (tinyexr.h:6645-6683) has no multi-part / deep rejection (LoadEXR's is at
    :6268-6270): a single-part file with either version bit decodes; the bits change only how
    ReconstructTileOffsets walks the chunks (:5876-5931)."""
    for name in ("multipart_flag.exr", "multipart_tiled.exr", "deep_flag_scan.exr"):
        assert MAN[name]["code"] == 0, name
    for name in ("multipart_tiles_zero.exr", "deep_tiles_zero.exr"):
        assert MAN[name]["code"] == O.INVALID_DATA, name
