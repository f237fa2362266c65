#!/usr/bin/env python3
"""Writes tests/golden/exr/*.exr and tests/golden/exr_manifest.json: OpenEXR files (tools/exrwrite.py)
covering every compression / pixel type / layout the GPU read takes, and files tinyexr rejects at
each check, with the oracle's result (oracle/exr_oracle.py: code, size, sha256 of the RGBA float
bits). TEST INFRASTRUCTURE (container-only; the GPU box only reads the committed files).

Parity is unpinned (oracle/exr_oracle.py header): no EXR library is importable here and
tinyexr.h does not build without miniz."""
import hashlib
import json
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import exr_oracle as O  # noqa: E402
from tools import exrwrite as W  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "exr")


def image(seed, h, w):
    """Smooth HDR-ish planes with specials (negative, tiny, large, inf, nan, denormal halves)."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    base = [np.sin(x * (0.05 + 0.01 * k) + k) * np.cos(y * 0.07) * (4.0 + k) + rng.normal(0, 0.3, (h, w)) for k in range(4)]
    planes = [b.astype(np.float32) for b in base]
    flat = planes[0].reshape(-1)
    sp = np.array([0.0, -0.0, 1e-7, 6e-8, -3e-5, 65504.0, np.inf, -np.inf, np.nan, 1e30], np.float32)
    flat[: min(len(sp), flat.size)] = sp[: flat.size]
    return planes


def rgba(seed, h, w, kind):
    p = image(seed, h, w)
    if kind == "half":
        return [(n, a.astype(np.float16)) for n, a in zip("RGBA", p)]
    if kind == "float":
        return [(n, a) for n, a in zip("RGBA", p)]
    if kind == "uint":
        return [(n, (a.view(np.uint32) ^ np.uint32(0x5A5A5A5A))) for n, a in zip("RGBA", p)]
    if kind == "mixed":
        return [("R", p[0].astype(np.float16)), ("G", p[1]), ("B", p[2].astype(np.float16)),
                ("A", (p[3].view(np.uint32) & np.uint32(0xFFFF)))]
    raise ValueError(kind)


def cases():
    c = {}
    for comp, cn in ((W.NONE, "none"), (W.RLE, "rle"), (W.ZIPS, "zips"), (W.ZIP, "zip")):
        for kind in ("half", "float", "uint", "mixed"):
            c[f"scan_{cn}_{kind}.exr"] = W.write_exr(rgba(len(c), 37, 61, kind), compression=comp, origin=(-3, 5))
        c[f"tile_{cn}_half.exr"] = W.write_exr(rgba(len(c), 45, 70, "half"), compression=comp, tiles=(16, 12))
        c[f"scan_{cn}_desc.exr"] = W.write_exr(rgba(len(c), 33, 40, "half"), compression=comp, line_order=1)
    # channel sets (LoadEXRFromMemory :6685-6860)
    p = image(90, 20, 30)
    c["gray_y_half.exr"] = W.write_exr([("Y", p[0].astype(np.float16))], compression=W.ZIP)
    c["rgb_no_alpha.exr"] = W.write_exr([(n, a.astype(np.float16)) for n, a in zip("RGB", p)], compression=W.ZIPS)
    c["rgba_extra_channels.exr"] = W.write_exr([(n, a.astype(np.float16)) for n, a in zip("RGBA", p)] +
                                               [("Z", p[0]), ("N.x", p[1].astype(np.float16))], compression=W.ZIP)
    c["missing_g.exr"] = W.write_exr([("R", p[0]), ("B", p[1])], compression=W.NONE)
    c["unsorted_channels.exr"] = W.write_exr([("B", p[2]), ("A", p[3]), ("R", p[0]), ("G", p[1])], compression=W.RLE,
                                             sort=False)
    c["tile_big_tiles.exr"] = W.write_exr(rgba(91, 20, 30, "float"), compression=W.ZIP, tiles=(64, 64))
    c["tile_desc_edge.exr"] = W.write_exr(rgba(92, 21, 30, "half"), compression=W.NONE, tiles=(8, 8), line_order=1)
    c["scan_1x1.exr"] = W.write_exr(rgba(93, 1, 1, "half"), compression=W.ZIP)
    c["scan_wide.exr"] = W.write_exr(rgba(94, 3, 700, "half"), compression=W.ZIP)
    # offset-table reconstruction (:6146-6168): zeros in the table
    c["offsets_zero.exr"] = W.write_exr(rgba(95, 40, 20, "half"), compression=W.ZIP, offsets=lambda o: [0] * len(o))
    # rejected by header / table / chunk checks
    good = W.write_exr(rgba(96, 16, 16, "half"), compression=W.ZIP)
    c["bad_magic.exr"] = b"\x76\x2f\x31\x02" + good[4:]
    c["bad_version.exr"] = good[:4] + b"\x03" + good[5:]
    c["too_short.exr"] = good[:6]
    c["missing_lineorder.exr"] = W.write_exr(rgba(96, 16, 16, "half"), compression=W.ZIP, drop=("lineOrder",))
    c["pxr24.exr"] = W.write_exr(rgba(96, 16, 16, "half"), compression=W.ZIP,
                                 attrs={"compression": W.attr("compression", "compression", bytes([5]))})
    c["piz.exr"] = W.write_exr(rgba(96, 16, 16, "half"), compression=W.ZIP,
                               attrs={"compression": W.attr("compression", "compression", bytes([4]))})
    c["type_mismatch.exr"] = W.write_exr(rgba(96, 16, 16, "half"), compression=W.ZIP,
                                         extra_attrs=W.attr("type", "string", b"tiledimage"))
    c["multipart_flag.exr"] = W.write_exr(rgba(96, 16, 16, "half"), compression=W.ZIP, version_flags=0x10,
                                          extra_attrs=W.attr("name", "string", b"a") + W.attr("type", "string", b"scanlineimage"))
    c["mipmap_tiles.exr"] = W.write_exr(rgba(97, 16, 16, "half"), compression=W.NONE, tiles=(8, 8),
                                        attrs={"tiles": W.attr("tiles", "tiledesc", struct.pack("<IIB", 8, 8, 1))})
    c["inverted_window.exr"] = W.write_exr(rgba(96, 16, 16, "half"), compression=W.ZIP,
                                           attrs={"dataWindow": W.attr("dataWindow", "box2i", struct.pack("<iiii", 5, 0, 4, 15))})
    c["offset_past_end.exr"] = W.write_exr(rgba(96, 16, 16, "half"), compression=W.ZIP, offsets=lambda o: [o[0] + 10**6])
    c["zip_bad_adler.exr"] = W.write_exr(rgba(96, 16, 16, "half"), compression=W.ZIP,
                                         raw_chunks=lambda i, d: d[:-1] + bytes([d[-1] ^ 1]))
    c["zip_truncated.exr"] = W.write_exr(rgba(96, 16, 16, "half"), compression=W.ZIP, raw_chunks=lambda i, d: d[: len(d) // 2])
    c["rle_truncated.exr"] = W.write_exr(rgba(98, 16, 16, "half"), compression=W.RLE,
                                         raw_chunks=lambda i, d: d[: max(3, len(d) - 5)] if i == 3 else d)
    c["none_short_chunk.exr"] = W.write_exr(rgba(99, 16, 16, "half"), compression=W.NONE,
                                            raw_chunks=lambda i, d: d[:-2] if i == 7 else d)
    c["line_out_of_range.exr"] = W.write_exr(rgba(99, 16, 16, "half"), compression=W.ZIP, chunk_line=lambda i, y: y - 100)
    c["zip_zero_len.exr"] = W.write_exr(rgba(99, 16, 16, "half"), compression=W.ZIPS, raw_chunks=lambda i, d: b"" if i == 2 else d)
    return c


def main():
    os.makedirs(OUT, exist_ok=True)
    man = {}
    with np.errstate(over="ignore"):  # (values past 65504 become half infinities, on purpose)
        all_cases = cases()
    for name, data in all_cases.items():
        open(os.path.join(OUT, name), "wb").write(data)
        code, w, h, img = O.decode(data)
        man[name] = {"code": code, "w": w, "h": h,
                     "sha256": hashlib.sha256(img.tobytes()).hexdigest() if img is not None else None}
    json.dump(man, open(os.path.join(ROOT, "tests", "golden", "exr_manifest.json"), "w"), indent=1, sort_keys=True)
    ok = sum(1 for v in man.values() if v["code"] == 0)
    print(f"{len(man)} files ({ok} decode, {len(man) - ok} rejected)")


if __name__ == "__main__":
    main()
