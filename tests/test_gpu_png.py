"""GPU PNG encoder parity: through the C ABI, lodepng's colour
type / palette / tRNS and its filter bytes must equal the oracle exactly, and the IDAT must
inflate (Python zlib) to the oracle's filtered stream; the whole file must decode back to the
input pixels. Compressed size is reported against the system zlib (level 6) on the identical
filtered stream -- lodepng's own deflate is unbuildable here (png.h absent), see DESIGN.md."""
import zlib

import numpy as np
import pytest

import imagecodecs_amd as icx
from oracle import pyoracle as O
import pngutil as P

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = icx.Context(0)
    yield c
    c.close()


def check(ctx, px, decode=True):
    h, w, d = px.shape
    png = ctx.png_encode(w, h, d, px.tobytes())
    assert png is not None
    I = P.info(png)  # also verifies every chunk CRC
    m = O.png_choose(px.tobytes(), w, h, d)
    assert (I["colortype"], I["bitdepth"]) == (m.colortype, m.bitdepth)
    if m.colortype == 3:
        pal = np.frombuffer(bytes(m.pal[: 4 * m.npal]), np.uint8).reshape(-1, 4)
        assert I["plte"] == pal[:, :3].tobytes()
        a = pal[:, 3]
        nz = np.nonzero(a != 255)[0]
        assert I["trns"] == (a[: nz[-1] + 1].tobytes() if len(nz) else None)
    elif m.key_defined:
        k = [m.key_r, m.key_g, m.key_b] if m.colortype == 2 else [m.key_r]
        assert I["trns"] == b"".join(int(v).to_bytes(2, "big") for v in k)
    else:
        assert I["trns"] is None
    assert zlib.decompress(I["idat"]) == O.png_filtered(px.tobytes(), w, h, d, m)
    if decode:
        np.testing.assert_array_equal(P.decode_rgba(png), P.to_rgba(px))
    return png


@pytest.mark.parametrize("w,h", [(1, 1), (3, 2), (37, 23), (257, 5), (64, 64)])
@pytest.mark.parametrize("kind", ["rgba", "opaque", "rgb3"])
def test_png_synthetic(ctx, w, h, kind):
    px = P.synth_rgba(w * 7 + h, w, h, opaque=kind != "rgba")
    if kind == "rgb3":
        px = np.ascontiguousarray(px[..., :3])
    check(ctx, px)


def _palette_img(rng, n, w, h, alpha=False):
    pal = rng.integers(0, 256, (n, 4), dtype=np.uint8)
    if not alpha:
        pal[:, 3] = 255
    return pal[rng.integers(0, n, (h, w))]


@pytest.mark.parametrize("case", ["grey8", "grey1", "grey2", "grey4", "pal2", "pal4", "pal16", "pal60", "pal256",
                                  "pal_alpha", "key_rgb", "key_grey", "grey_alpha", "white_only"])
def test_png_colour_modes(ctx, case):
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    w, h = 45, 31
    if case.startswith("grey") and case != "grey_alpha":
        levels = {"grey8": 256, "grey1": 2, "grey2": 4, "grey4": 16}[case]
        g = (rng.integers(0, levels, (h, w, 1)) * (255 // (levels - 1))).astype(np.uint8)
        px = np.repeat(g, 3, axis=2)
    elif case.startswith("pal") and case != "pal_alpha":
        px = _palette_img(rng, int(case[3:]), w, h)
    elif case == "pal_alpha":
        px = _palette_img(rng, 40, w, h, alpha=True)
    elif case == "key_rgb":
        px = P.synth_rgba(5, w, h, opaque=True)
        px[..., :3][(px[..., :3] == (9, 9, 9)).all(axis=2)] = 10
        px[3:6, 4:9] = (9, 9, 9, 0)
    elif case == "key_grey":
        g = rng.integers(0, 256, (h, w, 1)).astype(np.uint8)
        g[g == 77] = 78
        px = np.concatenate([np.repeat(g, 3, axis=2), np.full((h, w, 1), 255, np.uint8)], axis=2)
        px[2:4, 2:4] = (77, 77, 77, 0)
    elif case == "grey_alpha":
        g = rng.integers(0, 256, (h, w, 1)).astype(np.uint8)
        px = np.concatenate([np.repeat(g, 3, axis=2), rng.integers(0, 256, (h, w, 1)).astype(np.uint8)], axis=2)
    else:
        px = np.full((h, w, 4), 255, np.uint8)
    check(ctx, px)


def test_png_large_rgba_and_size(ctx):
    """A 2048^2 alpha-gradient image: exact filtered stream, size within 5% of zlib -6."""
    w = h = 2048
    px = P.synth_rgba(99, w, h)
    png = check(ctx, px, decode=False)
    ref = O.png_encode_zlib(px.tobytes(), w, h, 4, 6)
    assert len(png) <= 1.05 * len(ref), (len(png), len(ref))


def test_png_block_plan_without_lds(ctx, monkeypatch):
    """the deflate block grouping reads its counts from global memory when they do
    not fit its LDS (more than 4 GiB of filtered bytes) instead of failing; forced here with
    ICX_PNG_PLAN_LDS=0 on an image of several base blocks: the same file bytes."""
    w = h = 1024
    px = P.synth_rgba(7, w, h)
    want = ctx.png_encode(w, h, 4, px.tobytes())
    monkeypatch.setenv("ICX_PNG_PLAN_LDS", "0")
    assert ctx.png_encode(w, h, 4, px.tobytes()) == want


def test_png_device_api(ctx):
    import torch
    w, h = 640, 480
    px = P.synth_rgba(1, w, h)
    enc = icx.PngEncoder(ctx)
    d_src = torch.from_numpy(px).cuda()
    d_out = torch.empty(w * h * 4 * 2, dtype=torch.uint8, device="cuda")
    rc, n = enc.encode_device(w, h, 4, d_src.data_ptr(), d_out.data_ptr(), 100)
    assert rc == icx.OUT_OF_MEM and n > 100
    rc, n2 = enc.encode_device(w, h, 4, d_src.data_ptr(), d_out.data_ptr(), d_out.numel())
    assert rc == icx.OK and n2 == n
    png = d_out[:n].cpu().numpy().tobytes()
    assert png == ctx.png_encode(w, h, 4, px.tobytes())  # deterministic
    np.testing.assert_array_equal(P.decode_rgba(png), px)
    enc.close()


@pytest.mark.parametrize("inflight", ["1", "2", "3", "8"])
def test_png_device_batch(ctx, monkeypatch, inflight):
    """icx_png_encode_device_batch (ICX_PNG_INFLIGHT images in flight, each on its own workspace
    and stream; 8 is more than the 7 images): every
    file equals the one-image entry's bytes, including a palette image (the colour-mode read-back
    path), a grey image and an odd size; a slot too small reports ICX_OUT_OF_MEM and the bytes
    needed without disturbing the other images."""
    import torch
    w, h = 333, 211
    pxs = [P.synth_rgba(10 + k, w, h) for k in range(5)]
    pxs.append(np.repeat(np.arange(w * h, dtype=np.uint32).reshape(h, w, 1) % 7 * 30, 4, axis=2).astype(np.uint8))
    pxs.append(np.repeat((np.arange(w * h) % 251).reshape(h, w, 1), 4, axis=2).astype(np.uint8))
    pxs[-1][..., 3] = 255
    monkeypatch.setenv("ICX_PNG_INFLIGHT", inflight)
    want = [ctx.png_encode(w, h, 4, p.tobytes()) for p in pxs]
    stride = max(len(x) for x in want) + 4096
    enc = icx.PngEncoder(ctx)
    d_src = [torch.from_numpy(np.ascontiguousarray(p)).cuda() for p in pxs]
    d_out = torch.zeros(len(pxs) * stride, dtype=torch.uint8, device="cuda")
    st, sz = enc.encode_device_batch(w, h, 4, [t.data_ptr() for t in d_src], d_out.data_ptr(), stride)
    assert (st == icx.OK).all(), st
    out = d_out.cpu().numpy()
    for i, wb in enumerate(want):
        assert int(sz[i]) == len(wb)
        assert out[i * stride: i * stride + sz[i]].tobytes() == wb, i
    # a slot smaller than the files: every image reports ICX_OUT_OF_MEM with its size
    small = 1000
    d_small = torch.zeros(len(pxs) * small, dtype=torch.uint8, device="cuda")
    st2, sz2 = enc.encode_device_batch(w, h, 4, [t.data_ptr() for t in d_src], d_small.data_ptr(), small)
    assert (st2 == icx.OUT_OF_MEM).all() and list(sz2) == [len(x) for x in want]
    enc.close()


def test_png_rejects(ctx):
    assert ctx.png_encode(4, 4, 2, bytes(32)) is None
    assert ctx.png_encode(0, 4, 4, b"") is None


def test_png_c5_8192_rgba(ctx):
    """C5 at full size: one 8192^2 RGBA alpha-gradient image (tests/pngutil.synth_rgba, the
    bench's input): exact colour type and filtered stream (the oracle's MINSUM filters), IDAT
    inflating to it, and a size within 5% of zlib -6 on the same filtered stream."""
    w = h = 8192
    px = P.synth_rgba(8192, w, h)
    png = check(ctx, px, decode=False)
    ref = O.png_encode_zlib(px.tobytes(), w, h, 4, 6)
    assert len(png) <= 1.05 * len(ref), (len(png), len(ref))


PNG_FIX = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "png")


def _bmp(name):
    """The reference's data/*.bmp (committed as data fixtures under tests/golden/png) as RGB."""
    from PIL import Image
    return np.asarray(Image.open(__import__("os").path.join(PNG_FIX, name)).convert("RGB"))


def test_png_reference_anchor(ctx):
    """the reference's one PNG anchor on the GPU path -- data/test.png's pixels
    (opaque RGBA 499 x 289) encode as lodepng encodes them: palette colour type,
    8-bit, the palette in first-seen order, filter 0 on every row; and decode back exactly."""
    px = P.read_fixture_png(__import__("os").path.join(PNG_FIX, "test.png"))
    h, w = px.shape[:2]
    assert (w, h) == (499, 289) and px[..., 3].min() == 255
    png = check(ctx, px)
    I = P.info(png)
    assert (I["colortype"], I["bitdepth"]) == (3, 8)
    raw = zlib.decompress(I["idat"])
    assert set(raw[:: w + 1]) == {0}
    # first-seen order: palette entry k is the k-th distinct colour in raster order
    flat = px.reshape(-1, 4)
    _, first = np.unique(flat.view(np.uint32), return_index=True)
    order = flat[np.sort(first)][:, :3]
    assert I["plte"] == order.tobytes()


def _size_vs_zlib(ctx, px, decode=True):
    h, w, d = px.shape
    png = check(ctx, px, decode)
    I = P.info(png)
    m = O.png_choose(px.tobytes(), w, h, d)
    z6 = len(zlib.compress(O.png_filtered(px.tobytes(), w, h, d, m), 6))
    return len(I["idat"]) / z6


@pytest.mark.parametrize("name", ["test.bmp", "cat.bmp"])
@pytest.mark.parametrize("alpha", [False, True])
def test_png_size_real_content(ctx, name, alpha, capsys):
    """IDAT size on the reference's own photographs (data/test.bmp, cat.bmp)
    as RGB (opaque RGBA: lodepng drops alpha) and with a gradient alpha (RGBA kept), against
    system zlib -6 on the identical filtered stream (the contract: within 5% of lodepng's size;
    lodepng itself is unbuildable here, zlib -6 stands in)."""
    rgb = _bmp(name)
    h, w = rgb.shape[:2]
    a = np.full((h, w, 1), 255, np.uint8) if not alpha else \
        np.broadcast_to((np.arange(w) * 255 // max(1, w - 1)).astype(np.uint8)[None, :, None], (h, w, 1))
    px = np.ascontiguousarray(np.concatenate([rgb, a], axis=2))
    r = _size_vs_zlib(ctx, px)
    with capsys.disabled():
        print(f"\n  {name} {'RGBA' if alpha else 'RGB'} {w}x{h}: GPU IDAT / zlib-6 = {r:.3f}")
    assert r <= 1.05, r


def test_png_size_photo_4096(ctx, capsys):
    """A 4096^2 photo-like image (tools/foreign.py photo: flat sky, noise band, hard edges,
    stripes) with gradient alpha: IDAT size against zlib -6."""
    from tools import foreign
    rgb = foreign.photo(7101, 4096, 4096)
    a = np.broadcast_to((np.arange(4096) * 255 // 4095).astype(np.uint8)[None, :, None], (4096, 4096, 1))
    px = np.ascontiguousarray(np.concatenate([rgb, a], axis=2))
    r = _size_vs_zlib(ctx, px, decode=False)
    with capsys.disabled():
        print(f"\n  photo 4096^2 RGBA: GPU IDAT / zlib-6 = {r:.3f}")
    assert r <= 1.05, r
