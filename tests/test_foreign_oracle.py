"""Pin the oracle on foreign-encoder and crafted streams (tier 1).

tests/golden/foreign_manifest.json holds NanoJPEG's results (oracle/_ref, the reference compiled
in place) for PIL/libjpeg-turbo files with optimised Huffman tables, other quant scalings,
restart markers, gray / RGB colour space and progressive streams, and for coefficient-level
streams (tools/coefjpeg.py) that reach the decoder's corners: large dequantized AC values,
15-16-bit codes for common symbols, tables beyond the second-level pool, DC beyond int16.
The same files drive the GPU tests (tests/test_gpu_foreign.py) and the lane emulator here."""
import hashlib
import json
import os

import pytest

from conftest import GOLDEN
from oracle import pyoracle as O
from tools import foreign as F

MANIFEST = json.load(open(os.path.join(GOLDEN, "foreign_manifest.json")))
LARGE = json.load(open(os.path.join(GOLDEN, "foreign_large.json")))


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_oracle_foreign_golden(name):
    exp = MANIFEST[name]
    data = open(os.path.join(GOLDEN, name), "rb").read()
    assert len(data) == exp["bytes"]
    code, w, h, n, pix = O.decode(data)
    assert code == exp["code"]
    if code == 0:
        assert (w, h, n) == (exp["w"], exp["h"], exp["ncomp"])
        assert sha(pix) == exp["sha256"]


def test_foreign_set_covers_the_verdict_grid():
    names = " ".join(MANIFEST)
    for tag in ("_opt", "_std", "q50", "q75", "q95", "q100", "_444", "_422", "_420", "rst", "gray",
                "progressive", "keep_rgb", "bigac_", "longcodes_", "search_", "dcwrap_"):
        assert tag in names, tag
    assert sum(1 for e in MANIFEST.values() if e["code"] == 2) >= 2  # progressive -> NJ_UNSUPPORTED
    assert "photo4096_q90_420_opt" in LARGE


@pytest.mark.parametrize("name", ["photo1024_q50_420_std", "photo2048_q75_422_opt_rst"])
def test_oracle_foreign_large_regenerated(name):
    """The regenerated large inputs: PIL writes the pinned bytes, the oracle the pinned pixels
    (the 4096^2 cases are decoded by the GPU tests only, to keep this suite fast)."""
    exp = LARGE[name]
    data = F.large(name)
    assert sha(data) == exp["jpeg_sha256"], "PIL wrote other bytes than the manifest pins"
    code, w, h, n, pix = O.decode(data)
    assert (code, w, h, n) == (exp["code"], exp["w"], exp["h"], exp["ncomp"])
    assert sha(pix) == exp["sha256"]


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref is built only where /root/reference exists")
@pytest.mark.parametrize("name", sorted(MANIFEST)[::5])
def test_foreign_manifest_matches_live_reference(name):
    data = open(os.path.join(GOLDEN, name), "rb").read()
    code, w, h, n, pix = O.ref_decode(data)
    e = MANIFEST[name]
    assert code == e["code"] and (code != 0 or sha(pix) == e["sha256"])
