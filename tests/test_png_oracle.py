"""PNG oracle (oracle/png_oracle.c): lodepng's colour choice + filter bytes, restated.

png_encoder.cpp includes libpng's png.h (absent here), so the reference is unbuildable; the
restatement is pinned by (1) the reference's own data/test.png, whose lodepng encode SURVEY.md
§8(c) records as palette, 8-bit, filter 0 for every row (container-only: /root/reference is
read in place, never copied), and (2) rule checks on synthetic images for every branch of
auto_choose_color (png_encoder.cpp:3552-3616).
"""
import os
import zlib

import numpy as np
import pytest

from oracle import pyoracle as O
import pngutil as P

REF_PNG = "/root/reference/data/test.png"


@pytest.mark.skipif(not os.path.exists(REF_PNG), reason="reference data only in the build container")
def test_oracle_png_reference_fixture():
    px = P.read_fixture_png(REF_PNG)  # opaque RGBA, 499 x 289
    h, w = px.shape[:2]
    assert (w, h) == (499, 289) and px[..., 3].min() == 255
    m = O.png_choose(px.tobytes(), w, h, 4)
    assert (m.colortype, m.bitdepth) == (3, 8)  # palette, 8-bit
    f = O.png_filtered(px.tobytes(), w, h, 4, m)
    assert len(f) == h * (w + 1) and set(f[:: w + 1]) == {0}  # filter 0 on every row
    png = O.png_encode_zlib(px.tobytes(), w, h, 4)
    np.testing.assert_array_equal(P.decode_rgba(png), px)


def _mode(px):
    h, w, d = px.shape
    m = O.png_choose(px.tobytes(), w, h, d)
    return m.colortype, m.bitdepth, m.npal, m.key_defined


def test_oracle_png_choices():
    rng = np.random.default_rng(7)
    g = rng.integers(0, 256, (40, 50, 1), dtype=np.uint8)
    grey = np.repeat(g, 3, axis=2)
    assert _mode(grey)[:2] == (0, 8)                                      # grey 8
    assert _mode(np.repeat((g // 128) * 255, 3, axis=2))[:2] == (0, 1)    # 2 grey levels -> 1-bit
    assert _mode(np.repeat((g // 64) * 85, 3, axis=2))[:2] == (0, 2)      # multiples of 85 -> 2-bit
    col = rng.integers(0, 256, (40, 50, 3), dtype=np.uint8)
    assert _mode(col)[:2] == (2, 8)                                       # RGB
    rgba = np.concatenate([col, rng.integers(1, 255, (40, 50, 1), dtype=np.uint8)], axis=2)
    assert _mode(rgba)[:2] == (6, 8)                                      # RGBA
    opaque = np.concatenate([col, np.full((40, 50, 1), 255, np.uint8)], axis=2)
    assert _mode(opaque)[:2] == (2, 8)                                    # opaque RGBA -> RGB
    pal = rng.integers(0, 256, (12, 3), dtype=np.uint8)[rng.integers(0, 12, (40, 50))]
    ct, bd, n, _ = _mode(pal)
    assert (ct, bd, n) == (3, 4, 12)                                      # 12 colours -> 4-bit palette
    keyed = opaque.copy()
    keyed[5, 7] = (1, 2, 3, 0)
    keyed[9, 9] = (1, 2, 3, 0)
    keyed[..., :3][(keyed[..., :3] == (1, 2, 3)).all(axis=2) & (keyed[..., 3] == 255)] = 0
    assert _mode(keyed)[0] == 2 and _mode(keyed)[3] == 1                  # RGB + tRNS key
    keyed[0, 0] = (1, 2, 3, 255)                                          # opaque key colour -> alpha
    assert _mode(keyed)[:2] == (6, 8)
    gray_alpha = np.concatenate([grey, rng.integers(0, 255, (40, 50, 1), dtype=np.uint8)], axis=2)
    assert _mode(gray_alpha)[:2] == (4, 8)


@pytest.mark.parametrize("kind", ["rgba", "opaque", "grey4", "pal16", "pal200"])
def test_oracle_png_roundtrip(kind):
    rng = np.random.default_rng(11)
    w, h = 37, 23
    if kind in ("rgba", "opaque"):
        px = P.synth_rgba(3, w, h, opaque=kind == "opaque")
    elif kind == "grey4":
        px = np.repeat((rng.integers(0, 16, (h, w, 1)) * 17).astype(np.uint8), 3, axis=2)
    else:
        n = 16 if kind == "pal16" else 200
        pal = rng.integers(0, 256, (n, 4), dtype=np.uint8)
        px = pal[rng.integers(0, n, (h, w))]
    d = px.shape[2]
    png = O.png_encode_zlib(px.tobytes(), w, h, d)
    np.testing.assert_array_equal(P.decode_rgba(png), P.to_rgba(px))
    I = P.info(png)
    assert zlib.decompress(I["idat"]) == O.png_filtered(px.tobytes(), w, h, d)
