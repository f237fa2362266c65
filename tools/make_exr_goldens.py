#!/usr/bin/env python3
"""Writes tests/golden/exr/*.exr and tests/golden/exr_manifest.json: OpenEXR files (tools/exrwrite.py)
covering every compression / pixel type / layout the GPU read takes, and files tinyexr rejects at
each check, with the oracle's result (oracle/exr_oracle.py: code, size, sha256 of the RGBA float
bits). TEST INFRASTRUCTURE (container-only; the GPU box only reads the committed files).

Pinned: every file is also loaded by the reference's own tinyexr, compiled in place with its
zlib route (oracle/Makefile `ref`), and the oracle must agree with it on every code and every
float the reference defines (ref_check); the rows it leaves uninitialised are listed per file
("ref_undefined_rows", where the oracle and the GPU write 0.0)."""
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
    # a ZIP payload labelled PIZ: DecompressPiz reads it as a range header (INVALID_DATA or garbage)
    c["piz.exr"] = W.write_exr(rgba(96, 16, 16, "half"), compression=W.ZIP,
                               attrs={"compression": W.attr("compression", "compression", bytes([4]))})
    c["type_mismatch.exr"] = W.write_exr(rgba(96, 16, 16, "half"), compression=W.ZIP,
                                         extra_attrs=W.attr("type", "string", b"tiledimage"))
    c["multipart_flag.exr"] = W.write_exr(rgba(96, 16, 16, "half"), compression=W.ZIP, version_flags=0x10,
                                          extra_attrs=W.attr("name", "string", b"a") + W.attr("type", "string", b"scanlineimage"))
    # LoadEXRFromMemory accepts the multi-part and deep version bits (only LoadEXR rejects them,
    # tinyexr.h:6268-6270); they reach ReconstructTileOffsets (:5876-5931): a zeroed table walks
    # the chunks skipping a part number (multi-part) or two deep sizes and their payloads
    nt = W.attr("name", "string", b"a") + W.attr("type", "string", b"tiledimage")
    c["multipart_tiled.exr"] = W.write_exr(smooth(24, 40, "half", 31), compression=W.ZIP, tiles=(16, 16),
                                           version_flags=0x12, extra_attrs=nt)
    c["multipart_tiles_zero.exr"] = W.write_exr(smooth(24, 40, "half", 32), compression=W.ZIP, tiles=(16, 16),
                                                version_flags=0x12, extra_attrs=nt, offsets=lambda o: [0] * len(o))
    c["deep_flag_scan.exr"] = W.write_exr(rgba(98, 16, 16, "half"), compression=W.RLE, version_flags=0x08,
                                          extra_attrs=W.attr("name", "string", b"d") + W.attr("type", "string", b"scanlineimage"))
    c["deep_tiles_zero.exr"] = W.write_exr(smooth(24, 40, "half", 33), compression=W.NONE, tiles=(16, 16),
                                           version_flags=0x0A, extra_attrs=nt, offsets=lambda o: [0] * len(o))
    # the mipmap flag on a one-level file: the offset table is shorter than the levels need
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
    c.update(piz_and_level_cases())
    return c


def smooth(h, w, kind, seed=0):
    """Smooth planes quantised to 1/64 (the PIZ wavelet + Huffman compress them; noise would be
    stored raw, Issue 40)."""
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    p = [np.round((np.sin(x * (0.05 + 0.01 * k) + k + seed) * np.cos(y * 0.07) * (4 + k)) * 64) / 64 for k in range(4)]
    if kind == "half":
        return [(n, a.astype(np.float16)) for n, a in zip("RGBA", p)]
    if kind == "float":
        return [(n, a.astype(np.float32)) for n, a in zip("RGBA", p)]
    if kind == "uint":
        return [(n, (np.abs(a) * 1000).astype(np.uint32)) for n, a in zip("RGBA", p)]
    return [("R", p[0].astype(np.float16)), ("G", p[1].astype(np.float32)), ("B", p[2].astype(np.float16)),
            ("A", (np.abs(p[3]) * 100).astype(np.uint32))]


def piz_and_level_cases():
    """PIZ (TINYEXR_USE_PIZ is on in the reference build, tinyexr.h:126-128) and mip- / rip-mapped
    tiles (DecodeChunk decodes every level, :5282-5354; the output is level 0)."""
    c = {}
    for kind in ("half", "float", "uint", "mixed"):
        c[f"scan_piz_{kind}.exr"] = W.write_exr(smooth(70, 90, kind, len(c)), compression=W.PIZ, origin=(4, -9))
    c["scan_piz_desc.exr"] = W.write_exr(smooth(45, 61, "half", 1), compression=W.PIZ, line_order=1)
    c["tile_piz_half.exr"] = W.write_exr(smooth(70, 90, "half", 2), compression=W.PIZ, tiles=(64, 32))
    y, x = np.mgrid[0:40, 0:600]
    h = (np.sin(x * 0.05) * np.cos(y * 0.1) * 8).astype(np.float16)
    # > 16384 distinct values in a chunk: wdec16 (maxValue >= 1 << 14, :2003)
    c["scan_piz_w16.exr"] = W.write_exr([("R", h), ("G", h), ("B", h), ("A", (x * 3 + y * 1801).astype(np.uint32))],
                                        compression=W.PIZ)
    h2 = h.copy()  # rare outliers: codes longer than the 14-bit direct table (:2574-2606, :2849-2887)
    h2[::7, ::13] = np.float16(1234.5) + x[::7, ::13].astype(np.float16)
    c["scan_piz_longcodes.exr"] = W.write_exr([("R", h2), ("G", h), ("B", h)], compression=W.PIZ)
    z = np.zeros((33, 50), np.float16)  # bitmap empty: minNonZero 8191, maxNonZero 0 (Issue 194)
    c["scan_piz_zero.exr"] = W.write_exr([("R", z), ("G", z), ("B", z)], compression=W.PIZ)
    rng = np.random.default_rng(5)
    c["scan_piz_raw.exr"] = W.write_exr([(n, rng.standard_normal((40, 30)).astype(np.float32)) for n in "RGB"],
                                        compression=W.PIZ)  # (stored raw: not smaller, Issue 40)
    # range header / length rejected by DecompressPiz (:3249-3314)
    c["piz_bad_bitmap.exr"] = W.write_exr(smooth(40, 50, "half", 3), compression=W.PIZ,
                                          raw_chunks=lambda i, d: d[:2] + b"\x00\x20" + d[4:] if i == 0 else d)
    c["piz_bad_length.exr"] = W.write_exr(smooth(40, 50, "half", 4), compression=W.PIZ,
                                          raw_chunks=lambda i, d: _piz_set_length(d, 10**6) if i == 0 else d)
    # damaged Huffman data: tinyexr ignores hufUncompress's failure and keeps what was decoded
    c["piz_damaged_codes.exr"] = W.write_exr(smooth(40, 50, "half", 5), compression=W.PIZ,
                                             raw_chunks=lambda i, d: d[: len(d) * 2 // 3] + bytes(len(d) - len(d) * 2 // 3))
    c["piz_short_length.exr"] = W.write_exr(smooth(40, 50, "half", 6), compression=W.PIZ,
                                            raw_chunks=lambda i, d: _piz_set_length(d, 7) if i == 0 else d)
    # levels
    c["mip_none_half.exr"] = W.write_exr(smooth(45, 70, "half", 7), compression=W.NONE, tiles=(16, 16), levels=1)
    c["mip_zip_mixed.exr"] = W.write_exr(smooth(45, 70, "mixed", 8), compression=W.ZIP, tiles=(16, 8), levels=1)
    c["mip_piz_half.exr"] = W.write_exr(smooth(90, 70, "half", 9), compression=W.PIZ, tiles=(64, 32), levels=1)
    c["mip_round_up.exr"] = W.write_exr(smooth(45, 70, "half", 10), compression=W.RLE, tiles=(16, 16), levels=1,
                                        rounding=1)
    c["rip_zips_half.exr"] = W.write_exr(smooth(45, 70, "half", 11), compression=W.ZIPS, tiles=(16, 16), levels=2)
    c["rip_piz_round_up.exr"] = W.write_exr(smooth(45, 70, "float", 12), compression=W.PIZ, tiles=(64, 32), levels=2,
                                            rounding=1)
    c["mip_desc.exr"] = W.write_exr(smooth(21, 30, "half", 13), compression=W.NONE, tiles=(8, 8), levels=1, line_order=1)
    # a level-1 tile naming the wrong level / damaged data in the last level: the read fails
    # although level 0 is intact (:5085-5094, :5124-5127)
    c["mip_wrong_level.exr"] = W.write_exr(smooth(45, 70, "half", 14), compression=W.ZIP, tiles=(16, 16), levels=1,
                                           raw_chunks=None, offsets=None)
    c["mip_wrong_level.exr"] = _patch_tile_level(c["mip_wrong_level.exr"], 1)
    c["mip_damaged_last.exr"] = W.write_exr(smooth(45, 70, "half", 15), compression=W.ZIP, tiles=(16, 16), levels=1,
                                            raw_chunks=lambda i, d: d[:-1] + bytes([d[-1] ^ 1]) if i == 19 else d)
    c["tile_mode3.exr"] = W.write_exr(smooth(16, 16, "half", 16), compression=W.NONE, tiles=(8, 8),
                                      attrs={"tiles": W.attr("tiles", "tiledesc", struct.pack("<IIB", 8, 8, 3))})
    # tile offsets to reconstruct (:6100-6108, :5867-5974)
    c["tile_offsets_zero.exr"] = W.write_exr(smooth(45, 70, "half", 17), compression=W.ZIP, tiles=(16, 16),
                                             offsets=lambda o: [0] * len(o))
    c["mip_offsets_zero.exr"] = W.write_exr(smooth(45, 70, "half", 18), compression=W.RLE, tiles=(16, 16), levels=1,
                                            offsets=lambda o: [0 if k % 3 == 0 else v for k, v in enumerate(o)])
    return c


def _piz_set_length(d, n):
    """The Huffman length field of a PIZ chunk payload (after the range header)."""
    mn, mx = struct.unpack_from("<HH", d, 0)
    at = 4 + (mx - mn + 1 if mn <= mx else 0)
    return d[:at] + struct.pack("<i", n) + d[at + 4:]


def _patch_tile_level(data, k):
    """Tile chunk k's level field (lx) + 1: the table still names it at its level."""
    code, info = O.parse_header(data)
    marker = info["header_len"] + 8
    o = struct.unpack_from("<Q", data, marker + 8 * k)[0]
    lx = struct.unpack_from("<i", data, o + 8)[0]
    return data[: o + 8] + struct.pack("<i", lx + 1) + data[o + 12:]


def ref_check():
    """The reference's tinyexr (oracle/_ref, built in place) over the written files, in its own
    process (tests/exrref.py): every code and every defined float must equal the oracle's, and
    the rows the reference leaves uninitialised are recorded in the manifest."""
    import subprocess
    if not os.path.exists("/root/reference/tinyexr.h"):
        raise SystemExit("the reference is needed to pin the EXR manifest (container only)")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    env = dict(os.environ, GLIBC_TUNABLES="glibc.malloc.tcache_count=0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "exrref.py"), "fixtures"], env=env, check=True,
                       capture_output=True, text=True)
    rep = json.loads(r.stdout)
    if rep["failures"]:
        raise SystemExit(f"oracle differs from the reference build: {rep['failures']}")
    return rep["undefined_rows"]


def main():
    os.makedirs(OUT, exist_ok=True)
    man = {}
    with np.errstate(over="ignore"):  # (values past 65504 become half infinities, on purpose)
        all_cases = cases()
    for name, data in all_cases.items():
        open(os.path.join(OUT, name), "wb").write(data)
    undef = ref_check()
    for name, data in all_cases.items():
        code, w, h, img = O.decode(data)
        man[name] = {"code": code, "w": w, "h": h,
                     "sha256": hashlib.sha256(img.tobytes()).hexdigest() if img is not None else None,
                     "ref_undefined_rows": undef.get(name, [])}
    json.dump(man, open(os.path.join(ROOT, "tests", "golden", "exr_manifest.json"), "w"), indent=1, sort_keys=True)
    ok = sum(1 for v in man.values() if v["code"] == 0)
    print(f"{len(man)} files ({ok} decode, {len(man) - ok} rejected)")


if __name__ == "__main__":
    main()
