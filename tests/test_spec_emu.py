"""CPU tests of the parallel entropy-decode ALGORITHM (icx_spec.hip) without a GPU.

tests/emu/spec_emu.cpp runs the kernels' per-lane code (imagecodecs_amd/csrc/icx_spec_core.h,
compiled __host__ __device__) lane by lane on the CPU: unstuff, speculative guess, count/verify,
scan, whole-block write. Its quantized coefficients and DC values must equal the oracle's
NanoJPEG trace block for block, for every subsequence size tried."""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from oracle import pyoracle as O
from tools import synthpy as S
from driutil import dri_corruptions, elsewhere_case

EMU_DIR = os.path.join(ROOT, "tests", "emu")
MANIFEST = json.load(open(os.path.join(GOLDEN, "decode_manifest.json")))
_L = None


def emu_lib():
    global _L
    if _L is None:
        subprocess.run(["make", "-s", "-C", EMU_DIR], check=True)
        import imagecodecs_amd
        imagecodecs_amd._share_hip_runtime_with_torch()
        L = C.CDLL(os.path.join(EMU_DIR, "libspecemu.so"))
        L.emu_spec_decode.restype = C.c_int
        L.emu_spec_decode.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_void_p, C.c_int64,
                                      C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.c_void_p]
        _L = L
    return _L


def emu(data: bytes, sub_bytes: int = 256, cap: int = 1 << 17):
    coef = np.zeros((cap, 64), np.int16)
    dc = np.zeros(cap, np.int32)
    nb, st = C.c_int64(), C.c_int32()
    stats = np.zeros(4, np.int64)
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    mode = emu_lib().emu_spec_decode(buf, len(data), sub_bytes, coef.ctypes.data, dc.ctypes.data, cap,
                                     C.byref(nb), C.byref(st), stats.ctypes.data)
    return mode, st.value, coef[: nb.value], dc[: nb.value]


def check(data, sub_bytes, allow_fallback=False):
    mode, st, coef, dc = emu(data, sub_bytes)
    if mode == 2:
        return mode
    if mode == 1:
        assert allow_fallback, "parallel chain failed to verify"
        return mode
    oc, ocoef, odc = O.decode_trace(data)
    assert st == (0 if oc == 0 else 5), (st, oc)
    if oc == 0:
        assert np.array_equal(coef, ocoef) and np.array_equal(dc, odc)
    return mode


@pytest.mark.parametrize("sub_bytes", [64, 256, 512, 2048])
def test_emulated_parallel_decode_goldens(sub_bytes):
    """Every non-DRI golden finishes on the parallel path (repair walks included)."""
    modes = [check(open(os.path.join(GOLDEN, n), "rb").read(), sub_bytes, allow_fallback=False) for n in sorted(MANIFEST)]
    assert modes.count(0) >= 40 and modes.count(1) == 0


@pytest.mark.parametrize("sampling", ["420", "444", "422", "gray", "440", "411"])
def test_emulated_parallel_decode_synthetic(sampling):
    rng = np.random.default_rng(hash(sampling) % 1000)
    for k in range(3):
        w, h = int(rng.integers(40, 400)), int(rng.integers(40, 400))
        data = S.synth_jpeg(4000 + k, w, h, sampling, int(rng.integers(20, 100)))
        for sub in (32, 256, 2048):  # tiny lanes may exceed the 64-lane repair walk -> fallback
            assert check(data, sub, allow_fallback=sub < 256) in ((0, 1) if sub < 256 else (0,))


def test_emulated_parallel_decode_corrupt_streams_status():
    rng = np.random.default_rng(11)
    base = bytearray(S.synth_jpeg(77, 200, 150, "420", 85))
    sos = base.index(b"\xff\xda")
    start = sos + 2 + ((base[sos + 2] << 8) | base[sos + 3])
    for t in range(40):
        d = bytearray(base)
        for _ in range(1 + t % 4):
            d[int(rng.integers(start, len(d) - 2))] = int(rng.integers(0, 256))
        check(bytes(d), [32, 256, 2048][t % 3], allow_fallback=True)


def test_emulated_resync_statistics_4k():
    """At the production lane size (2 KiB) a 4:2:0 q90 4096x1024 image resyncs inside almost
    every lane; the repair walk covers the rest (bit-exact either way)."""
    data = S.synth_jpeg(4242, 4096, 1024, "420", 90)
    coef = np.zeros((1 << 17, 64), np.int16)
    dc = np.zeros(1 << 17, np.int32)
    nb, st = C.c_int64(), C.c_int32()
    stats = np.zeros(4, np.int64)
    buf = C.create_string_buffer(data, len(data))
    mode = emu_lib().emu_spec_decode(buf, len(data), 2048, coef.ctypes.data, dc.ctypes.data, 1 << 17, C.byref(nb),
                                     C.byref(st), stats.ctypes.data)
    assert mode == 0 and st.value == 0
    oc, ocoef, odc = O.decode_trace(data)
    assert np.array_equal(coef[: nb.value], ocoef) and np.array_equal(dc[: nb.value], odc)
    lanes = (len(data) + 2047) // 2048
    assert stats[3] >= 0.97 * (lanes - 1), stats  # lanes spliced at a recorded state


# Annex K (JPEG spec) luminance/chrominance AC code-length counts; symbols are placeholders.
_K3 = [0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7D]
_K5 = [0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77]
_K1 = [0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0]
_K2 = [0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0]


def _huff_selftest(counts):
    L = emu_lib()
    L.emu_huff_selftest.restype = C.c_int
    L.emu_huff_selftest.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.POINTER(C.c_int)]
    n = sum(counts)
    syms = bytes((i * 37 + 11) & 0xFF for i in range(n))
    nsub = C.c_int()
    bad = L.emu_huff_selftest(bytes([0] + counts), syms, n, C.byref(nsub))
    return bad, nsub.value


@pytest.mark.parametrize("counts", [_K1, _K2, _K3, _K5], ids=["dc_luma", "dc_chroma", "ac_luma", "ac_chroma"])
def test_two_level_huffman_annex_k(counts):
    bad, nsub = _huff_selftest(counts)
    assert bad == 0
    assert 0 <= nsub <= 8  # the standard tables fit the subtable budget


def test_two_level_huffman_random_tables():
    rng = np.random.default_rng(7)
    over_budget = 0
    for _ in range(300):
        # random Kraft-valid length counts (possibly incomplete code space), up to 256 symbols
        counts, space, total = [0] * 16, 1 << 16, 0
        for L in range(1, 17):
            cap = min(space >> (16 - L), 256 - total)
            c = int(rng.integers(0, cap + 1)) if cap > 0 and rng.random() < 0.7 else 0
            if L == 16 and rng.random() < 0.5:
                c = cap
            counts[L - 1] = c
            space -= c << (16 - L)
            total += c
        bad, nsub = _huff_selftest(counts)
        assert bad == 0, counts
        over_budget += nsub > 8
    assert over_budget > 0  # the exact-search fallback was exercised too


def _step_selftest(dc_counts, dc_syms, ac_counts, ac_syms, seed, nblocks=3000):
    L = emu_lib()
    L.emu_step_selftest.restype = C.c_int
    L.emu_step_selftest.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_char_p, C.c_char_p, C.c_int, C.c_uint64,
                                    C.c_int, C.c_void_p]
    stats = np.zeros(4, np.int64)
    bad = L.emu_step_selftest(bytes([0] + dc_counts), bytes(dc_syms), len(dc_syms), bytes([0] + ac_counts),
                              bytes(ac_syms), len(ac_syms), seed, nblocks, stats.ctypes.data)
    return bad, stats


def _ac_symbols(rng, n, invalid_rate=0.0):
    valid = [0x00, 0xF0] + [(r << 4) | s for r in range(16) for s in range(1, 11)]
    out = []
    for _ in range(n):
        if rng.random() < invalid_rate:
            out.append(int(rng.integers(1, 16)) << 4)  # size 0, not ZRL: a syntax error (:669)
        else:
            out.append(valid[int(rng.integers(0, len(valid)))])
    return out


@pytest.mark.parametrize("seed", range(4))
def test_step_tables_annex_k(seed):
    """Step tables (icx_step.h: multi-symbol scan runs, write pairs, long-code pool) decode
    random streams exactly like the symbol-by-symbol canonical walk with NanoJPEG's block rules."""
    rng = np.random.default_rng(seed)
    dc_counts = _K1 if seed % 2 == 0 else _K2
    ac_counts = _K3 if seed % 2 == 0 else _K5
    dc_syms = list(range(sum(dc_counts)))
    ac_syms = _ac_symbols(rng, sum(ac_counts), invalid_rate=0.02 * seed)
    bad, stats = _step_selftest(dc_counts, dc_syms, ac_counts, ac_syms, 1000 + seed)
    assert bad == 0, stats
    assert stats[2] < stats[1] and stats[3] < stats[1]  # runs / pairs took several symbols per lookup


def test_step_tables_random_tables():
    rng = np.random.default_rng(21)
    for t in range(120):
        tabs = []
        for _ in range(2):
            counts, space, total = [0] * 16, 1 << 16, 0
            for L in range(1, 17):
                cap = min(space >> (16 - L), 256 - total)
                c = int(rng.integers(0, cap + 1)) if cap > 0 and rng.random() < 0.6 else 0
                counts[L - 1] = c
                space -= c << (16 - L)
                total += c
            tabs.append((counts, total))
        (dcc, ndc), (acc, nac) = tabs
        dc_syms = [int(x) for x in rng.integers(0, 256, ndc)]
        ac_syms = _ac_symbols(rng, nac, invalid_rate=0.05)
        bad, stats = _step_selftest(dcc, dc_syms, acc, ac_syms, 7 + t, nblocks=400)
        assert bad == 0, (t, dcc, acc)


def ref_unstuff(R: bytes):
    """NanoJPEG's byte rules (jpeg_dec.h:447-482) read sequentially: FF00 / FFFF -> FF, FFD0-7
    kept (both bytes, position recorded), FFD9 ends the data, any other FFxx or FF at the end of
    the file ends it with a syntax error (errpos = unstuffed length)."""
    out, rst, p, err = bytearray(), [], 0, None
    while p < len(R):
        c = R[p]
        if c != 0xFF:
            out.append(c)
            p += 1
            continue
        if p + 1 >= len(R):
            err = len(out)
            break
        m = R[p + 1]
        if m in (0x00, 0xFF):
            out.append(0xFF)
        elif m & 0xF8 == 0xD0:
            rst.append((len(out) << 3) | (m & 7))
            out += bytes([0xFF, m])
        else:
            err = len(out) if m != 0xD9 else None
            break
        p += 2
    return bytes(out), err, rst


def emu_unstuff(data: bytes, sh: int):
    L = emu_lib()
    L.emu_unstuff_sh.restype = C.c_int64
    cap = len(data) + 64
    out = C.create_string_buffer(cap)
    rst = np.zeros(1 << 16, np.int64)
    errpos, giveup, nrst, so = C.c_int64(), C.c_int32(), C.c_int64(), C.c_int64()
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    n = L.emu_unstuff_sh(buf, C.c_int64(len(data)), sh, out, C.c_int64(cap), C.byref(errpos), C.byref(giveup),
                         rst.ctypes.data_as(C.c_void_p), C.c_int64(len(rst)), C.byref(nrst), C.byref(so))
    if n < 0:
        return None
    e = None if errpos.value == (1 << 63) - 1 else errpos.value
    return out.raw[:n], e, list(rst[: nrst.value]), so.value


def _stuffing_corpus():
    files = [open(os.path.join(GOLDEN, n), "rb").read() for n in sorted(MANIFEST)]
    # adversarial scans: FF runs of every length, stuffing / restart / end markers at every offset
    # of a 16-byte chunk and across 1 KiB round and 4 KiB tile boundaries
    rng = np.random.default_rng(77)
    base = S.synth_jpeg(11, 64, 64, "420", 90)
    sos = base.index(b"\xff\xda")
    head = base[: sos + 2 + int.from_bytes(base[sos + 2: sos + 4], "big")]
    pieces = [b"\xff\x00", b"\xff\xff", b"\xff\xd0", b"\xff\xd3", b"\xff\xd7", b"\xff" * 3 + b"\x00", b"\xff" * 5 + b"\xd1"]
    for k in range(24):
        body = bytearray()
        while len(body) < 9000:
            body += bytes(rng.integers(0, 255, int(rng.integers(0, 40)), dtype=np.uint8))
            body += pieces[int(rng.integers(0, len(pieces)))]
        tail = [b"\xff\xd9", b"\xff\xc4", b"\xff", b""][k % 4]
        files.append(head + bytes(body) + tail)
    # dense stuffing (several FF 00 pairs per 16-byte chunk, FFs at every chunk offset including
    # the last, whose 00 is the next chunk's first byte): ustf16's stuffing-only tier
    for k in range(8):
        body = bytearray()
        while len(body) < 9000:
            body += bytes(rng.integers(0, 255, int(rng.integers(0, 7)), dtype=np.uint8))
            body += b"\xff\x00" if rng.random() < 0.97 else pieces[int(rng.integers(1, len(pieces)))]
        files.append(head + bytes(body) + [b"\xff\xd9", b""][k % 2])
    return files


def test_emulated_unstuff_every_alignment():
    """k_ustf_count / k_ustf_write's aligned-tile unstuff (icx_spec_core.h ustf16) gives the same
    stream, error position and restart records as NanoJPEG's sequential byte rules, for all 16
    alignments of the scan start (the GPU takes the alignment from the data's address)."""
    checked = 0
    for data in _stuffing_corpus():
        r0 = emu_unstuff(data, 0)
        if r0 is None:
            continue
        so = r0[3]
        ref = ref_unstuff(data[so:])
        for sh in range(16):
            u, e, rst, _ = emu_unstuff(data, sh)
            assert (u, e, rst) == ref, sh
        checked += 1
    assert checked >= 148


FOREIGN = json.load(open(os.path.join(GOLDEN, "foreign_manifest.json")))


@pytest.mark.parametrize("sub_bytes", [256, 2048])
def test_emulated_parallel_decode_foreign(sub_bytes):
    """Foreign-encoder tables (libjpeg-turbo optimised Huffman, other quant scalings) and the
    crafted corner streams (long codes on common symbols, tables beyond the pool): the lane code
    verifies its chains and writes the oracle's coefficients block for block."""
    modes = []
    for n in sorted(FOREIGN):
        if FOREIGN[n]["code"] != 0:
            continue
        modes.append(check(open(os.path.join(GOLDEN, n), "rb").read(), sub_bytes, allow_fallback=False))
    assert modes.count(1) == 0 and modes.count(0) >= 40, modes


# ---- guess-write path (icx_spec.hip k_gw_*): the emulator's emu_gw_decode runs the same lane
# functions (icx_spec_core.h gc_find / gc_write / gw_lane_total / gw_lane_err / GwSlots) ----
def gw_lib():
    L = emu_lib()
    if not hasattr(L, "_gw"):
        L.emu_gw_decode.restype = C.c_int
        L.emu_gw_decode.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int64, C.c_double, C.c_void_p, C.c_void_p,
                                    C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.c_void_p]
        L._gw = True
    return L


def gw_check(data, sub=256, lead=2048, frac=1.1, cap=1 << 18):
    coef = np.zeros((cap, 64), np.int16)
    dc = np.zeros(cap, np.int32)
    nb, st = C.c_int64(), C.c_int32()
    stats = np.zeros(8, np.int64)
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    mode = gw_lib().emu_gw_decode(buf, len(data), sub, lead, frac, coef.ctypes.data, dc.ctypes.data, cap, C.byref(nb),
                                  C.byref(st), stats.ctypes.data)
    if mode != 0:
        return mode, stats
    oc, ocoef, odc = O.decode_trace(data)
    assert st.value == (0 if oc == 0 else 5), (st.value, oc)
    if oc == 0:
        n = nb.value
        assert np.array_equal(dc[:n], odc) and np.array_equal(coef[:n], ocoef)
    return mode, stats


@pytest.mark.parametrize("sub,lead", [(64, 0), (256, 512), (2048, 2048)])
def test_gw_goldens(sub, lead):
    """Every non-DRI golden decodes bit-exact on the guess-write path; only streams whose data
    ends before the last block without an error (NanoJPEG reads on into the 0xFF padding) go
    sequential."""
    modes = {}
    for n in sorted(MANIFEST):
        m, _ = gw_check(open(os.path.join(GOLDEN, n), "rb").read(), sub, lead)
        modes.setdefault(m, []).append(n)
    assert len(modes.get(0, [])) >= 40
    assert all("truncated" in n for n in modes.get(1, [])), modes.get(1)


@pytest.mark.parametrize("sub,frac", [(256, 1.1), (2048, 1.1), (512, 0.05)])
def test_gw_foreign_and_overflow_chunks(sub, frac):
    """Foreign-encoder and crafted streams, with the static slots per lane cut to 5% so most
    blocks go through chained overflow chunks (GwSlots)."""
    tot = np.zeros(8, np.int64)
    for n in sorted(FOREIGN):
        if FOREIGN[n]["code"] != 0:
            continue
        m, st = gw_check(open(os.path.join(GOLDEN, n), "rb").read(), sub, 2048, frac)
        assert m == 0 or (m == 2 and "rst" in n), n  # (restart-marker streams take the DRI lanes)
        tot += st
    assert tot[2] > 0 and tot[3] > 0  # some lanes were count-decoded and spliced
    if frac < 1:
        assert tot[5] > 100  # overflow chunks in use


@pytest.mark.parametrize("sampling", ["420", "444", "422", "gray", "440", "411"])
def test_gw_synthetic_random_leads(sampling):
    rng = np.random.default_rng(abs(hash("gw" + sampling)) % 1000)
    for k in range(2):
        w, h = int(rng.integers(40, 500)), int(rng.integers(40, 500))
        data = S.synth_jpeg(5000 + k, w, h, sampling, int(rng.integers(10, 100)))
        for sub in (64, 512):
            m, _ = gw_check(data, sub, int(rng.integers(0, 3000)), float(rng.choice([0.02, 1.1])))
            assert m == 0


# ---- restart intervals (k_spec_write mode 3 + k_spec_finish) ----
def dri_emu(data, cap=1 << 17):
    L = emu_lib()
    L.emu_dri_decode.restype = C.c_int
    L.emu_dri_decode.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64),
                                 C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    coef = np.zeros((cap, 64), np.int16)
    dc = np.zeros(cap, np.int32)
    nb, st, first = C.c_int64(), C.c_int32(), C.c_int32()
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    mode = L.emu_dri_decode(buf, len(data), coef.ctypes.data, dc.ctypes.data, cap, C.byref(nb), C.byref(st),
                            C.byref(first))
    return mode, st.value, first.value, coef[: nb.value], dc[: nb.value]


def dri_check(data):
    """Emulated DRI decode vs the oracle: a parallel result must carry NanoJPEG's status, and its
    coefficients when that is OK. Returns the mode (0 parallel, 1 sequential, 2 not eligible)."""
    mode, st, first, coef, dc = dri_emu(data)
    if mode != 0:
        return mode
    oc, ocoef, odc = O.decode_trace(data)
    assert st == (0 if oc == 0 else 5), (st, oc, first)
    if oc == 0:
        assert np.array_equal(coef, ocoef) and np.array_equal(dc, odc)
    return mode


@pytest.mark.parametrize("restart,sampling", [(1, "420"), (3, "gray"), (5, "444"), (16, "422")])
def test_emulated_dri_clean(restart, sampling):
    """Clean DRI streams: every interval ends at its marker; coefficients equal the trace."""
    for k in range(3):
        data = S.synth_jpeg(8100 + k, 120 + 56 * k, 96 + 40 * k, sampling, 70 + 10 * k, restart)
        mode, st, first, _, _ = dri_emu(data)
        assert mode == 0 and st == 0 and first == 2**31 - 1
        assert dri_check(data) == 0


@pytest.mark.parametrize("restart,sampling", [(1, "420"), (2, "gray"), (7, "444"), (40, "420")])
def test_emulated_dri_corrupt_status(restart, sampling):
    """Corrupt DRI streams: the parallel status equals NanoJPEG's for every variant the lanes can
    decide (the first interval not ending at its marker); only FF D0+(j&7) read somewhere other
    than marker j sends an image to the sequential kernel."""
    rng = np.random.default_rng(restart * 100 + len(sampling))
    base = S.synth_jpeg(8200 + restart, 200, 152, sampling, 85, restart)
    modes = [dri_check(v) for v in dri_corruptions(base, rng, 64)]
    assert modes.count(2) == 0
    assert modes.count(1) <= 2, modes  # (these seeds: none)


def test_emulated_dri_elsewhere_goes_sequential():
    v, j = elsewhere_case()
    mode, st, first, _, _ = dri_emu(v)
    assert mode == 1 and first == 2 * j + 1, (mode, first, j)
