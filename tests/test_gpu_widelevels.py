"""Hard-edged content at high quality on every decode path: one-pixel stripes and checkers of
0 / 255 give AC levels in the hundreds (the synthetic noise images never pass |AC| 83, even at
q100; the oracle's coefficient trace proves the wide levels per case). Every entropy path (three
passes, guess-write, DRI lanes, count lanes, the sequential kernel) and every 4:2:0 back-half mode
must stay bit-exact on them (jpeg_dec.h:658-676). Round 4 kept these as the regression set of an
int8 coefficient-cell pool with int16 copies of such blocks (measured slower, reverted: DESIGN.md
§4, profiles/r04j_int8_cells_ab.txt)."""
import numpy as np
import pytest

import imagecodecs_amd as icx
from oracle import pyoracle as O
from tools import synthpy as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = icx.Context(0)
    yield c
    c.close()


def hard_jpeg(seed, w, h, sampling, quality, restart=0):
    """Noise with a quarter of the 8x8 cells each holding vertical stripes, horizontal stripes or a
    checker of 0 / 255 (the rest noise around mid-grey): at q100 a quarter to two thirds of the
    blocks have an AC level outside [-127, 127]."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    px = (rng.integers(0, 256, (h, w, 3)) // 4 + 96).astype(np.uint8)
    kind = rng.integers(0, 4, (h // 8 + 1, w // 8 + 1))[y // 8, x // 8]
    pat = np.select([kind == 0, kind == 1, kind == 2], [(x & 1) * 255, (y & 1) * 255, ((x ^ y) & 1) * 255], -1)
    m = pat >= 0
    px[m] = pat[m][:, None].astype(np.uint8)
    if sampling == "gray":
        px = px[:, :, :1]
    return S.jpeg(px, sampling, quality, restart)


def _wide_levels(jpeg):
    code, coef, dc = O.decode_trace(jpeg, cap_blocks=1 << 19)
    assert code == 0
    return int((np.abs(coef[:, 1:].astype(np.int32)) > 127).any(axis=1).sum())


def _check(res, jpegs):
    for j, (code, w, h, n, pix) in zip(jpegs, res):
        ocode, ow, oh, on, opix = O.decode(j)
        assert (code, w, h, n) == (ocode, ow, oh, on)
        assert pix.tobytes() == opix


@pytest.mark.parametrize("sampling,w,h,cap,restart", [
    ("444", 700, 500, 1024, 0),     # three-pass path
    ("420", 1024, 768, 1024, 0),
    ("422", 640, 480, 1024, 0),     # generic IDCT (k_idct)
    ("420", 2048, 2048, 2048, 0),   # guess-write path (k_gw_lane / k_gw_count)
    ("444", 2048, 1536, 2048, 0),
    ("420", 1000, 1000, 1024, 7),   # DRI lanes
])
def test_wide_levels_bit_exact(ctx, sampling, w, h, cap, restart):
    jpegs = [hard_jpeg(7300 + k, w, h, sampling, q, restart) for k, q in enumerate((100, 90))]
    assert _wide_levels(jpegs[0]) > 0
    b = icx.Batch(ctx, len(jpegs), cap, cap)
    res = b.decode_host(jpegs)
    assert b.path_stats()["sequential"] == 0
    _check(res, jpegs)
    b.close()


@pytest.mark.parametrize("mode", ["0", "1", "2", "3", "4", "5"])
def test_wide_levels_420_modes(ctx, monkeypatch, mode):
    """4:2:0 back halves: generic (0), fused luma (1), lane-pair IDCT + stream convert (2),
    k_back420 (3)."""
    monkeypatch.setenv("ICX_FUSE420", mode)
    jpegs = [hard_jpeg(7400 + k, 1536, 1024, "420", q) for k, q in enumerate((100, 95))]
    assert _wide_levels(jpegs[0]) > 0
    b = icx.Batch(ctx, 2, 2048, 2048)
    _check(b.decode_host(jpegs), jpegs)
    b.close()


def test_wide_levels_sequential_kernel(ctx):
    """18 blocks per MCU (non-conforming, NanoJPEG decodes it): the sequential kernel."""
    j = hard_jpeg(7500, 512, 512, "y44", 100)
    b = icx.Batch(ctx, 1, 512, 512)
    res = b.decode_host([j])
    assert _wide_levels(j) > 0 and b.path_stats()["parallel"] == 0
    _check(res, [j])
    b.close()
