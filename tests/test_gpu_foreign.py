"""GPU parity on streams from a foreign encoder and on crafted corner streams.

Every stream in tests/golden/foreign_manifest.json (PIL/libjpeg-turbo: optimised Huffman tables,
q 50..100, 4:4:4 / 4:2:2 / 4:2:0, restart markers, gray, RGB colour space, custom quant tables,
progressive; tools/coefjpeg.py: large dequantized AC values, long codes on common symbols,
tables beyond the pool, DC beyond int16) decodes through the C ABI to NanoJPEG's status and
pixels, bit for bit (expected values from oracle/_ref, the reference compiled in place). Every
valid stream must stay on the parallel entropy path: no sequential fallback."""
import hashlib
import json
import os

import pytest

from conftest import GOLDEN
import imagecodecs_amd as icx
from tools import foreign as F

pytestmark = pytest.mark.gpu

MANIFEST = json.load(open(os.path.join(GOLDEN, "foreign_manifest.json")))
LARGE = json.load(open(os.path.join(GOLDEN, "foreign_large.json")))


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def ctx():
    c = icx.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_foreign_single(ctx, name):
    exp = MANIFEST[name]
    code, w, h, n, pix = ctx.decode(open(os.path.join(GOLDEN, name), "rb").read())
    assert code == exp["code"], (code, exp["code"])
    if code == icx.OK:
        assert (w, h, n) == (exp["w"], exp["h"], exp["ncomp"])
        assert sha(pix) == exp["sha256"]


def _batch_check(ctx, names, max_w, max_h):
    jpegs = [open(os.path.join(GOLDEN, n), "rb").read() for n in names]
    b = icx.Batch(ctx, len(jpegs), max_w, max_h)
    res = b.decode_host(jpegs)
    stats = b.path_stats()
    nvalid = sum(1 for n in names if MANIFEST[n]["code"] == 0)
    assert stats["parallel"] == nvalid and stats["fallback"] == 0, stats
    for n, (code, w, h, c, pix) in zip(names, res):
        exp = MANIFEST[n]
        assert code == exp["code"], n
        if code == icx.OK:
            assert sha(pix.tobytes()) == exp["sha256"], n
    b.close()


@pytest.mark.parametrize("gw", ["1", "0", None])
@pytest.mark.parametrize("mode", ["0", "1", "2", "3", "4", "5"])
def test_foreign_batch_all_plane_modes(ctx, monkeypatch, mode, gw):
    """All foreign + crafted streams in one batch, under each 4:2:0 plane mode (the lane-pair IDCT
    of modes 1 and 2 meets the large-coefficient streams) and each entropy path (ICX_GW 1:
    guess-write, 0: three passes, unset: the workspace-size choice): parallel path for every
    valid one."""
    monkeypatch.setenv("ICX_FUSE420", mode)
    if gw is None:
        monkeypatch.delenv("ICX_GW", raising=False)
    else:
        monkeypatch.setenv("ICX_GW", gw)
    names = sorted(MANIFEST)
    mw = max(MANIFEST[n]["w"] for n in names)
    mh = max(MANIFEST[n]["h"] for n in names)
    _batch_check(ctx, names, mw, mh)


def test_crafted_big_coefficients_each_mode(ctx, monkeypatch):
    """a dequantized AC of 2500 at natural (0,1) passes the lane-pair IDCT's
    2^14 gate; its 181 products need 32 bits."""
    name = "crafted/bigac_420_zz1_q250.jpg"
    data = open(os.path.join(GOLDEN, name), "rb").read()
    for mode in ("5", "4", "3", "2", "1", "0"):
        monkeypatch.setenv("ICX_FUSE420", mode)
        b = icx.Batch(ctx, 1, 64, 64)
        code, w, h, c, pix = b.decode_host([data])[0]
        assert code == 0 and sha(pix.tobytes()) == MANIFEST[name]["sha256"], mode
        b.close()


@pytest.mark.parametrize("mode", [None, "2", "3", "4", "5"])
def test_foreign_large_regenerated(ctx, monkeypatch, mode):
    """The large regenerated inputs (tools/foreign.LARGE): a 4096^2 q90 4:2:0 optimised-table
    photo-like image, 4:4:4 q100 at 1.3 B/px (more than one workspace slot of U: the pool),
    restart markers per MCU row, odd sizes. One batch, parallel path, bit-exact."""
    if mode is not None:
        monkeypatch.setenv("ICX_FUSE420", mode)
    names = sorted(LARGE)
    jpegs = []
    for n in names:
        data = F.large(n)
        assert sha(data) == LARGE[n]["jpeg_sha256"], f"{n}: PIL wrote other bytes than the manifest pins"
        jpegs.append(data)
    b = icx.Batch(ctx, len(jpegs), 4096, 4096)
    res = b.decode_host(jpegs)
    stats = b.path_stats()
    assert stats == {"parallel": len(jpegs), "fallback": 0, "sequential": 0}, stats
    for n, (code, w, h, c, pix) in zip(names, res):
        e = LARGE[n]
        assert (code, w, h, c) == (e["code"], e["w"], e["h"], e["ncomp"]), n
        assert sha(pix.tobytes()) == e["sha256"], n
    b.close()


def test_foreign_large_single_q100_444(ctx):
    """One-image decode (a one-slot workspace) of the 1.3 B/px 4:4:4 q100 stream: the U pool
    holds it, so the image takes the parallel path."""
    n = "photo4096_q100_444_opt"
    data = F.large(n)
    b = icx.Batch(ctx, 1, 4096, 2048)
    code, w, h, c, pix = b.decode_host([data])[0]
    assert b.path_stats() == {"parallel": 1, "fallback": 0, "sequential": 0}
    assert code == 0 and sha(pix.tobytes()) == LARGE[n]["sha256"]
    b.close()
