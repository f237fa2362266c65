"""Radiance .hdr test corpus shared by the oracle tests (CPU) and the GPU parity tests.

Inputs come from tools/synth.c (synth_rgbe pixels, hdr_encode in three pixel-data layouts) and
from byte-level edits of those files; everything is seeded, so the CPU and GPU runs see the same
bytes. `expected_floats` is an independent statement of workOnRGBE/convertComponent
(codecs.cpp:617-628, 610-615) for well-formed files: v * 2^(E-136) per channel, E as float.
"""
import numpy as np

from tools import synthpy as S

RLE, FLAT, OLD = S.HDR_RLE, S.HDR_FLAT, S.HDR_OLD_RLE


def header(w: int, h: int) -> bytes:
    return b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y %d +X %d\n" % (h, w)


def row_bytes(px_row: np.ndarray, mode: int) -> bytes:
    """Pixel data of one scanline (1, w, 4) coded as `mode`, without the header."""
    w = px_row.shape[1]
    f = S.hdr(px_row.reshape(1, w, 4), mode)
    return f[len(header(w, 1)):]


def expected_floats(rgbe: np.ndarray) -> np.ndarray:
    rgbe = np.asarray(rgbe, np.uint8)
    e = rgbe[..., 3].astype(np.int32) - 136
    out = np.empty(rgbe.shape, np.float32)
    for c in range(3):
        out[..., c] = np.ldexp(rgbe[..., c].astype(np.float32), e)
    out[..., 3] = rgbe[..., 3].astype(np.float32)
    return out


def mixed_file(seed: int, w: int, h: int):
    """Rows cycle through new-style RLE, flat, old-style RLE and flat rows whose first pixel
    starts with 2 (decrunchHDR's (2, G, B, E) fallback, codecs.cpp:679-683)."""
    px = S.rgbe(seed, w, h)
    parts = [header(w, h)]
    for y in range(h):
        k = y % 4
        if k == 3:
            px[y, 0] = (2, 5 + y % 7, 77, 130)
        mode = (RLE, FLAT, OLD, FLAT)[k]
        parts.append(row_bytes(px[y:y + 1], mode))
    return b"".join(parts), px


def valid_cases():
    """(name, file bytes, rgbe pixels) for well-formed files."""
    out = []
    for mode, mname in ((RLE, "rle"), (FLAT, "flat"), (OLD, "old")):
        for i, (w, h) in enumerate([(1, 3), (5, 4), (7, 9), (8, 8), (9, 5), (64, 33), (258, 20), (1000, 7)]):
            px = S.rgbe(100 + 10 * mode + i, w, h)
            out.append((f"{mname}_{w}x{h}", S.hdr(px, mode), px))
    for i, (w, h) in enumerate([(8, 12), (33, 17), (300, 9)]):
        f, px = mixed_file(7 + i, w, h)
        out.append((f"mixed_{w}x{h}", f, px))
    # literals that contain the new-style scanline start pattern 2 2 w>>8 w&255 (false candidates)
    w, h = 258, 6
    px = S.rgbe(55, w, h)
    for y in range(h):
        px[y, 10:14, 0] = (2, 2, w >> 8, w & 255)
        px[y, 40:44, 1] = (2, 2, w >> 8, w & 255)
    out.append(("rle_false_candidates", S.hdr(px, RLE), px))
    # old-style chained run counts (rshift 8): 1 1 1 2, then 1 1 1 1 -> 2 + (1 << 8) = 258 repeats
    w, h = 300, 2
    px = S.rgbe(56, w, h)
    body = []
    for y in range(h):
        px[y, 1:259] = px[y, 0]
        body.append(bytes(px[y, 0]) + bytes((1, 1, 1, 2)) + bytes((1, 1, 1, 1)) + px[y, 259:].tobytes())
    out.append(("old_chained_runs", header(w, h) + b"".join(body), px))
    return out


def edge_cases():
    """(name, file bytes) for header errors, truncation, undefined run-length data and fuzz."""
    out = []
    px = S.rgbe(9, 40, 6)
    rle, flat, old = S.hdr(px, RLE), S.hdr(px, FLAT), S.hdr(px, OLD)
    hl = len(header(40, 6))
    out += [
        ("empty", b""),
        ("not_radiance", b"#?RGBE\n\n-Y 2 +X 2\n" + bytes(16)),
        ("short_magic", b"#?RADIAN"),
        ("no_blank_line", b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n-Y 2 +X 2"),
        ("no_reso_newline", b"#?RADIANCE\nA\n\n-Y 2 +X 2"),
        ("reso_x_first", b"#?RADIANCE\n\n\n+X 2 -Y 2\n" + bytes(16)),
        ("reso_only_y", b"#?RADIANCE\nA\n\n-Y 2\n" + bytes(16)),
        ("reso_zero", b"#?RADIANCE\nA\n\n-Y 0 +X 4\n"),
        ("reso_negative", b"#?RADIANCE\nA\n\n-Y 2 +X -4\n" + bytes(64)),
        ("reso_spaces", b"#?RADIANCE\nA\n\n-Y   2   +X\t3\n" + bytes(range(24))),
        ("reso_huge", b"#?RADIANCE\nA\n\n-Y 100000 +X 100000\n" + bytes(64)),
        ("header_only", header(40, 6)),
    ]
    for frac in (0.1, 0.5, 0.97):
        for name, f in (("rle", rle), ("flat", flat), ("old", old)):
            cut = hl + int((len(f) - hl) * frac)
            out.append((f"trunc_{name}_{frac}", f[:cut]))
    out.append(("trunc_flat_minus1", flat[:-1]))
    out.append(("trunc_rle_minus1", rle[:-1]))
    out.append(("trunc_in_row_header", rle[:hl + 2]))
    # new-style run that overflows the scanline (undefined in the reference)
    bad = bytearray(header(10, 1) + bytes((2, 2, 0, 10)) + bytes((128 + 11, 7)))
    out.append(("rle_run_overflow", bytes(bad) + bytes(64)))
    out.append(("rle_literal_overflow", header(10, 1) + bytes((2, 2, 0, 10, 12)) + bytes(80)))
    # old-style run on the first pixel of a scanline: count > 0 reads scanline[-1]; count 0 is fine
    out.append(("old_run_first_px", header(4, 1) + bytes((1, 1, 1, 3)) + bytes(16)))
    out.append(("old_run_zero_first_px", header(4, 1) + bytes((1, 1, 1, 0)) + bytes((9, 9, 9, 129)) * 4))
    # four chained markers: rshift reaches 24 with a zero count, then 32 (over-wide)
    chain = bytes((5, 6, 7, 130)) + bytes((1, 1, 1, 0)) * 3 + bytes((1, 1, 1, 0)) + bytes((1, 1, 1, 1))
    out.append(("old_rshift_24_zero", header(4, 1) + bytes((5, 6, 7, 130)) + bytes((1, 1, 1, 0)) * 3
                + bytes((8, 8, 8, 128)) * 3))
    out.append(("old_rshift_32", header(4, 1) + chain + bytes(16)))
    out.append(("old_run_past_end", header(4, 1) + bytes((5, 6, 7, 130)) + bytes((1, 1, 1, 9)) + bytes(16)))
    # width bytes of a new-style row header disagree with the image width (still new-style)
    f = bytearray(rle)
    f[hl + 2], f[hl + 3] = 0, 99
    out.append(("rle_width_mismatch", bytes(f)))
    # width outside 8..0x7fff: every row is old-style even if it starts 2 2
    out.append(("narrow_2_2", header(4, 2) + bytes((2, 2, 0, 4)) * 2 + bytes(range(24))))
    # trailing bytes after the last scanline are ignored
    out.append(("rle_trailing", rle + bytes(100)))
    out.append(("flat_trailing", flat + bytes((1, 1, 1, 1)) * 8))
    # seeded fuzz: byte flips in the pixel data of each layout
    rng = np.random.default_rng(1234)
    for name, f in (("rle", rle), ("flat", flat), ("old", old)):
        for k in range(12):
            g = bytearray(f)
            for _ in range(1 + k % 4):
                p = int(rng.integers(hl, len(g)))
                g[p] = int(rng.choice([0, 1, 2, 128, 129, 200, 255, int(rng.integers(0, 256))]))
            out.append((f"fuzz_{name}_{k}", bytes(g)))
    return out
