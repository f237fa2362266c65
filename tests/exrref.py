"""TEST INFRASTRUCTURE: the reference's tinyexr (oracle/_ref/libref_exr.so, compiled in place from
/root/reference/tinyexr.h by `make -C oracle ref`) against the EXR oracle.

Run as a script in its own process (tests/test_exr_oracle.py does), because telling tinyexr's
defined output from the floats it never writes needs the allocator set up at process start:
GLIBC_TUNABLES=glibc.malloc.tcache_count=0 (every allocation goes through malloc's perturb path)
and mallopt(M_PERTURB) inside the library. Each input is loaded twice with different perturb
bytes; floats that differ between the two loads are uninitialised memory in the reference
(tinyexr mallocs the RGBA buffer, :6785-6787, and rows or tiles no chunk writes keep whatever was
there). The oracle writes 0.0 there (oracle/exr_oracle.py header); everywhere else the two must
agree bit for bit, and the result codes always.

    python3 tests/exrref.py fixtures            -> JSON report over tests/golden/exr
    python3 tests/exrref.py fuzz SEED N         -> flags / byte damage / truncation variants
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import exr_oracle as O  # noqa: E402

LIB = os.path.join(ROOT, "oracle", "_ref", "libref_exr.so")
EXR = os.path.join(ROOT, "tests", "golden", "exr")
ENV = {"GLIBC_TUNABLES": "glibc.malloc.tcache_count=0"}
_L = None
_OUT = None


def lib():
    global _L
    if _L is None:
        L = C.CDLL(LIB)
        L.ref_exr_load.restype = C.c_int
        L.ref_exr_load.argtypes = [C.c_char_p, C.c_longlong, C.c_void_p, C.c_longlong, C.POINTER(C.c_int),
                                   C.POINTER(C.c_int)]
        L.ref_exr_perturb.argtypes = [C.c_int]
        _L = L
    return _L


def ref_load(data: bytes, perturb: int):
    """Image::readExr's call (codecs.cpp:464-476): the file's bytes plus the EOF byte (0xFF) its
    ifstream loop appends (:468-471), into LoadEXRFromMemory."""
    global _OUT
    L = lib()
    L.ref_exr_perturb(perturb)
    if _OUT is None:
        _OUT = np.zeros(1 << 22, np.uint32)  # (reused: the fixtures are at most 1M pixels)
    out, cap = _OUT, _OUT.size
    w, h = C.c_int(), C.c_int()
    d = bytes(data) + b"\xff"
    code = L.ref_exr_load(d, len(d), out.ctypes.data, cap, C.byref(w), C.byref(h))
    img = out[: w.value * h.value * 4].reshape(h.value, w.value, 4).copy() if code == 0 else None
    return code, w.value, h.value, img


def compare(data: bytes):
    """(ok, detail): the oracle against the reference on one input; detail also lists the rows
    the reference leaves undefined."""
    a = ref_load(data, 0x55)
    b = ref_load(data, 0xAA)
    oc, ow, oh, oimg = O.decode(data)
    if a[:3] != b[:3]:
        return False, {"nondeterministic": [a[:3], b[:3]]}
    if a[:3] != (oc, ow, oh):
        return False, {"ref": list(a[:3]), "oracle": [oc, ow, oh]}
    det = {"code": oc}
    if oc == 0:
        o32 = np.ascontiguousarray(oimg).view(np.uint32)
        undef = a[3] != b[3]
        bad = (a[3] != o32) & ~undef
        det["undefined_rows"] = sorted(set(np.nonzero(undef.any(axis=(1, 2)))[0].tolist()))
        if bad.any():
            return False, dict(det, mismatched_floats=int(bad.sum()))
        if undef.any() and not (o32[undef] == 0).all():
            return False, dict(det, undefined_not_zero=True)
    return True, det


def variants(seed: int, per_file: int):
    """Seeded variants of every fixture: the version-flag bits flipped (tiled, deep, multi-part),
    1-3 random bytes replaced, and a truncation."""
    rng = np.random.default_rng(seed)
    for name in sorted(os.listdir(EXR)):
        base = open(os.path.join(EXR, name), "rb").read()
        for f in (0x02, 0x08, 0x10, 0x18):
            b = bytearray(base)
            if len(b) > 5:
                b[5] ^= f
            yield f"{name}:flag{f:#x}", bytes(b)
        for k in range(per_file):
            b = bytearray(base)
            for _ in range(int(rng.integers(1, 4))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            yield f"{name}:dmg{k}", bytes(b)
        if len(base) > 9:
            yield f"{name}:trunc", base[: int(rng.integers(8, len(base)))]


def main():
    mode = sys.argv[1]
    rep = {"checked": 0, "failures": {}, "undefined_rows": {}}
    if mode == "fixtures":
        items = [(n, open(os.path.join(EXR, n), "rb").read()) for n in sorted(os.listdir(EXR))]
    else:
        items = variants(int(sys.argv[2]), int(sys.argv[3]))
    for tag, data in items:
        ok, det = compare(data)
        rep["checked"] += 1
        if not ok:
            rep["failures"][tag] = det
        elif det.get("undefined_rows"):
            rep["undefined_rows"][tag] = det["undefined_rows"]
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
