#!/usr/bin/env python3
"""CPU-baseline calibration (container only): the bench's CPU leg times the
oracle restatement (oracle/liboracle.so), because the reference cannot travel to the GPU box.
Here both the restatement and the reference NanoJPEG compiled in place (oracle/_ref) decode the
same synthetic images on one core; the ratio restatement / reference is written to
profiles/cpu_calibration.json, which bench.py reports beside its CPU number.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pyoracle as O  # noqa: E402
from tools import synthpy as S  # noqa: E402


def ref_decode_fast(data, _cache={}):
    """oracle/_ref decode into a reused output buffer (pyoracle.ref_decode allocates 256 MB per
    call, which would dominate a 1024^2 timing)."""
    import ctypes as C
    L = O.ref()
    key = len(data)
    if "out" not in _cache:
        _cache["out"] = C.create_string_buffer(4096 * 4096 * 3)
    src = C.create_string_buffer(bytes(data), max(1, len(data)))
    w, h, n = C.c_int(), C.c_int(), C.c_int()
    code = L.ref_nj_decode(src, len(data), C.byref(w), C.byref(h), C.byref(n), _cache["out"], 4096 * 4096 * 3)
    return code, key


def rate(fn, data, w, h, reps):
    fn(data)  # warm
    t = time.perf_counter()
    for _ in range(reps):
        code = fn(data)[0]
        assert code == 0
    return reps * w * h / 1e6 / (time.perf_counter() - t)


def main():
    if not O.ref_available():
        O.build(ref=True)
    out = {"host": os.uname().nodename, "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": "),
           "cases": {}}
    for (w, h, reps) in ((1024, 1024, 12), (4096, 4096, 3)):
        data = S.synth_jpeg(1234, w, h, "420", 90)
        port = rate(O.decode, data, w, h, reps)
        ref = rate(ref_decode_fast, data, w, h, reps)
        assert O.decode(data)[4] == O.ref_decode(data)[4]
        out["cases"][f"{w}x{h}_420_q90"] = {"port_mpx_s": round(port, 2), "reference_mpx_s": round(ref, 2),
                                           "ratio": round(port / ref, 3), "reps": reps}
        print(w, h, port, ref)
    out["ratio_1024"] = out["cases"]["1024x1024_420_q90"]["ratio"]
    out["ratio_4096"] = out["cases"]["4096x4096_420_q90"]["ratio"]
    json.dump(out, open(os.path.join(ROOT, "profiles", "cpu_calibration.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
