#!/usr/bin/env python3
"""Generate tests/golden/ from the REFERENCE ITSELF (oracle/_ref, compiled in place from
/root/reference). Container-only: the GPU box has no /root/reference and only reads the
committed fixtures.

Writes:
  tests/golden/test.jpg                 the reference's own fixture (data/test.jpg), copied as data
  tests/golden/jpeg/*.jpg               small synthetic + hand-corrupted JPEG streams
  tests/golden/decode_manifest.json     per file: NanoJPEG code, w, h, ncomp, sha256(pixels)
                                        (+ raw pixel hex for the tiniest images)
  tests/golden/tje/*.rgb                small RGB/RGBA inputs for the encoder
  tests/golden/tje_manifest.json        per input x quality: sha256 + length of tiny_jpeg output
  tests/golden/synth_manifest.json      generator parameters -> sha256(jpeg), sha256(NanoJPEG pixels)
                                        for larger images regenerated on the fly by tests/bench
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pyoracle as O  # noqa: E402
from tools import synthpy as S  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def ref_entry(data: bytes, raw_limit: int = 0) -> dict:
    code, w, h, n, pix = O.ref_decode(data)
    e = {"code": code, "w": w, "h": h, "ncomp": n, "sha256": sha(pix) if code == 0 else None}
    if code == 0 and len(pix) <= raw_limit:
        e["pixels_hex"] = pix.hex()
    return e


def corruptions(base: bytes) -> dict[str, bytes]:
    """Hand-made negative cases mapping to nj_result_t codes (jpeg_dec.h:117-125)."""
    out = {}
    b = bytearray(base)
    sof = b.index(b"\xff\xc0")
    sos = b.index(b"\xff\xda")
    scan_start = sos + 2 + ((b[sos + 2] << 8) | b[sos + 3])
    p = bytearray(b); p[sof + 1] = 0xC2; out["progressive_sof2"] = bytes(p)        # -> UNSUPPORTED
    p = bytearray(b); p[sof + 4] = 12; out["precision12"] = bytes(p)               # -> UNSUPPORTED
    p = bytearray(b); p[sof + 9] = 4; out["ncomp4"] = bytes(p)                     # -> UNSUPPORTED
    p = bytearray(b); p[sof + 11] = 0x31; out["sampling3"] = bytes(p)              # -> UNSUPPORTED (non pow2)
    p = bytearray(b); p[sof + 11] = 0x01; out["sampling0"] = bytes(p)              # -> SYNTAX
    out["not_jpeg"] = b"\x89PNG" + bytes(b[4:])                                    # -> NO_JPEG
    out["one_byte"] = b"\xff"                                                      # -> NO_JPEG
    out["truncated_header"] = bytes(b[: sof + 6])                                  # -> SYNTAX
    out["truncated_scan_mid"] = bytes(b[: scan_start + (len(b) - scan_start) // 2])
    out["truncated_scan_end"] = bytes(b[:-2])                                      # no EOI
    p = bytearray(b); q = scan_start + (len(b) - scan_start) // 3
    p[q] = 0xFF; p[q + 1] = 0xC4; out["bad_marker_in_scan"] = bytes(p)
    p = bytearray(b); p[-2] = 0xFF; p[-1] = 0xFF; out["ff_at_eof"] = bytes(p)      # FF FF then EOF
    out["garbage_after_eoi"] = bytes(b) + b"\x12\x34\xff\x00\xffGARBAGE"
    out["sos_without_frame"] = b"\xff\xd8\xff\xda\x00\x06\x00\x00\x3f\x00"         # NJ: OK, 0x0 image
    out["unknown_marker"] = bytes(b[:2]) + b"\xff\xc8\x00\x02" + bytes(b[2:])      # -> UNSUPPORTED
    out["com_zero_len"] = bytes(b[:2]) + b"\xff\xfe\x00\x00" + bytes(b[2:])        # -> SYNTAX
    p = bytearray(b); p[scan_start + 5] ^= 0x5A; p[scan_start + 40] ^= 0xA5; out["bitflips"] = bytes(p)
    # DHT with class/id bits the reference rejects
    dht = b.index(b"\xff\xc4")
    p = bytearray(b); p[dht + 4] = 0x02; out["dht_id2"] = bytes(p)                 # -> UNSUPPORTED
    p = bytearray(b); p[dht + 4] = 0x20; out["dht_class2"] = bytes(p)              # -> SYNTAX
    return out


def main() -> None:
    if not O.ref_available():
        O.build(ref=True)
    os.makedirs(os.path.join(G, "jpeg"), exist_ok=True)
    os.makedirs(os.path.join(G, "tje"), exist_ok=True)
    shutil.copyfile("/root/reference/data/test.jpg", os.path.join(G, "test.jpg"))

    manifest: dict[str, dict] = {}
    manifest["test.jpg"] = ref_entry(open(os.path.join(G, "test.jpg"), "rb").read())
    rng = np.random.default_rng(2024)
    cases = []
    for samp in ["gray", "444", "422", "420", "440", "411"]:
        for (w, h) in [(8, 8), (16, 16), (3, 3), (13, 7), (37, 29), (64, 48), (101, 67)]:
            if samp != "gray" and samp != "444" and min(w, h) < 6:
                continue  # the reference rejects subsampled comps < 3 px
            for ri in (0, 1, 5):
                q = int(rng.integers(10, 100))
                cases.append((samp, w, h, q, ri))
    for i, (samp, w, h, q, ri) in enumerate(cases):
        data = S.synth_jpeg(1000 + i, w, h, samp, q, ri)
        name = f"s{i:03d}_{samp}_{w}x{h}_q{q}_r{ri}.jpg"
        open(os.path.join(G, "jpeg", name), "wb").write(data)
        manifest["jpeg/" + name] = ref_entry(data, raw_limit=16 * 16 * 3)
    base = S.synth_jpeg(7, 48, 40, "420", 80, 0)
    base_r = S.synth_jpeg(8, 48, 40, "420", 80, 2)
    for tag, src in (("", base), ("dri_", base_r)):
        for k, data in corruptions(src).items():
            name = f"bad_{tag}{k}.jpg"
            open(os.path.join(G, "jpeg", name), "wb").write(data)
            manifest["jpeg/" + name] = ref_entry(data)
    json.dump(manifest, open(os.path.join(G, "decode_manifest.json"), "w"), indent=1, sort_keys=True)

    tje: dict[str, dict] = {}
    for (w, h, c) in [(8, 8, 3), (17, 9, 3), (33, 31, 4), (64, 48, 3), (9, 70, 4)]:
        px = S.rgb(w * 131 + h, w, h, c).tobytes()
        name = f"rgb_{w}x{h}x{c}.rgb"
        open(os.path.join(G, "tje", name), "wb").write(px)
        for q in (1, 2, 3):
            out = O.ref_tje_encode(q, w, h, c, px)
            tje[f"{name}:q{q}"] = {"w": w, "h": h, "comps": c, "quality": q, "len": len(out), "sha256": sha(out)}
    tp = open("/root/reference/data/test.jpg", "rb").read()
    code, w, h, n, pix = O.ref_decode(tp)
    out = O.ref_tje_encode(3, w, h, 3, pix)
    tje["test.jpg-decoded:q3"] = {"w": w, "h": h, "comps": 3, "quality": 3, "len": len(out), "sha256": sha(out),
                                  "source": "NanoJPEG decode of tests/golden/test.jpg"}
    for q in (1, 2, 3):
        out = O.ref_tje_encode(q, 1, 1, 3, b"\x10\x80\xf0")
        tje[f"1x1:q{q}"] = {"w": 1, "h": 1, "comps": 3, "quality": q, "len": len(out), "sha256": sha(out),
                            "rgb_hex": "1080f0"}
    json.dump(tje, open(os.path.join(G, "tje_manifest.json"), "w"), indent=1, sort_keys=True)

    synth: dict[str, dict] = {}
    for (seed, w, h, samp, q, ri) in [(1234, 1024, 1024, "420", 90, 0), (1235, 1024, 1024, "420", 90, 64),
                                      (1236, 999, 777, "422", 85, 0), (1237, 640, 480, "444", 95, 0),
                                      (1238, 1000, 1000, "gray", 90, 0), (1239, 2048, 2048, "420", 90, 0),
                                      (1240, 4096, 4096, "420", 90, 0)]:
        data = S.synth_jpeg(seed, w, h, samp, q, ri)
        code, ow, oh, n, pix = O.ref_decode(data)
        synth[f"{seed}_{w}x{h}_{samp}_q{q}_r{ri}"] = {
            "seed": seed, "w": w, "h": h, "sampling": samp, "quality": q, "restart": ri,
            "jpeg_len": len(data), "jpeg_sha256": sha(data), "code": code, "sha256": sha(pix)}
    json.dump(synth, open(os.path.join(G, "synth_manifest.json"), "w"), indent=1, sort_keys=True)
    print("goldens written:", len(manifest), "decode,", len(tje), "tje,", len(synth), "synth")


if __name__ == "__main__":
    main()
