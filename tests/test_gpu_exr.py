"""GPU tests of the OpenEXR read (Image::readExr -> tinyexr LoadEXRFromMemory, tinyexr.h:6645) through
the C ABI (icx_exr_decode): every fixture's code and RGBA float bits equal the manifest (the
oracle's result), larger images and random damage equal the oracle live. The oracle is pinned to
the reference's tinyexr compiled in place (tests/test_exr_oracle.py, oracle/exr_oracle.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
import imagecodecs_amd as icx
from oracle import exr_oracle as O
from tools import exrwrite as W

pytestmark = pytest.mark.gpu

MAN = json.load(open(os.path.join(GOLDEN, "exr_manifest.json")))
EXR = os.path.join(GOLDEN, "exr")


@pytest.fixture(scope="module")
def ctx():
    c = icx.Context(0)
    yield c
    c.close()


def sha(img):
    return hashlib.sha256(np.ascontiguousarray(img).view(np.uint32).tobytes()).hexdigest()


@pytest.mark.parametrize("name", sorted(MAN))
def test_exr_fixture(ctx, name):
    data = open(os.path.join(EXR, name), "rb").read()
    code, w, h, img = ctx.exr_decode(data)
    e = MAN[name]
    assert (code, w, h) == (e["code"], e["w"], e["h"])
    assert icx.exr_probe(data)[0] == code or code == icx.EXR_INVALID_DATA  # (pixel-data failures: device)
    if code == 0:
        assert sha(img) == e["sha256"]


@pytest.mark.parametrize("comp,tiles,levels", [(W.ZIP, None, 0), (W.ZIPS, None, 0), (W.RLE, None, 0), (W.NONE, None, 0),
                                               (W.ZIP, (64, 64), 0), (W.RLE, (128, 32), 0), (W.PIZ, None, 0),
                                               (W.PIZ, (128, 64), 1), (W.ZIP, (64, 32), 2)])
def test_exr_large_vs_oracle(ctx, comp, tiles, levels):
    """A 1000x700 half RGBA image (ZIP chunks of 16 lines = 22 KB of samples each, windows
    reaching back past 32 KiB of output; PIZ chunks of 32 lines = 256 KB of samples) decodes to
    the oracle's bits; mip- / rip-mapped files decode every level and output level 0."""
    rng = np.random.default_rng(comp * 10 + (tiles is not None))
    h, w = (700, 1000) if comp != W.PIZ else (350, 500)  # (the PIZ oracle is pure Python)
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    chans = [(n, (np.sin(x * (0.01 + 0.003 * k)) * np.cos(y * 0.013) * 50 + rng.normal(0, 0.05, (h, w))).astype(np.float16))
             for k, n in enumerate("RGBA")]
    data = W.write_exr(chans, compression=comp, tiles=tiles, levels=levels)
    oc, ow, oh, oimg = O.decode(data)
    code, ww, hh, img = ctx.exr_decode(data)
    assert (code, ww, hh) == (oc, ow, oh) == (0, w, h)
    assert np.array_equal(img.view(np.uint32), oimg.view(np.uint32))


@pytest.mark.parametrize("mode", ["stored", "fixed", "best", "flat"])
def test_exr_zip_block_types_vs_oracle(ctx, monkeypatch, mode):
    """Every deflate block type through the wave inflate (icx_exr.hip exr_inflate_wave): stored
    blocks (zlib level 0), fixed-Huffman blocks (Z_FIXED), level 9, and a flat image whose chunks
    are long repeats (distance < length, and matches reaching past the 16 KiB ring) -- each equal
    to the oracle bit for bit."""
    import zlib

    class Z:  # (tools/exrwrite.py's compressor, replaced for this file)
        @staticmethod
        def compress(data, level=6):
            if mode == "stored":
                return zlib.compress(data, 0)
            if mode == "fixed":
                c = zlib.compressobj(6, zlib.DEFLATED, 15, 9, zlib.Z_FIXED)
                return c.compress(data) + c.flush()
            return zlib.compress(data, 9)

    monkeypatch.setattr(W, "zlib", Z)
    rng = np.random.default_rng(77)
    h, w = 160, 1500
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    if mode == "flat":
        chans = [(n, np.full((h, w), 0.25 * (k + 1), np.float16)) for k, n in enumerate("RGBA")]
        chans[0] = ("R", (np.floor(x / 700) * 0.5).astype(np.float16))  # (a step every 700 columns)
    else:
        chans = [(n, (np.sin(x * (0.01 + 0.003 * k)) * np.cos(y * 0.013) * 50 + rng.normal(0, 0.05, (h, w))).astype(np.float16))
                 for k, n in enumerate("RGBA")]
    data = W.write_exr(chans, compression=W.ZIP)
    oc, ow, oh, oimg = O.decode(data)
    code, ww, hh, img = ctx.exr_decode(data)
    assert (code, ww, hh) == (oc, ow, oh) == (0, w, h)
    assert np.array_equal(img.view(np.uint32), oimg.view(np.uint32))


def test_exr_random_damage(ctx):
    """Random byte damage to fixtures: the GPU's code equals the oracle's, and so do the bits of
    the files that still decode."""
    rng = np.random.default_rng(11)
    names = [n for n in sorted(MAN) if MAN[n]["code"] == 0 and "wide" not in n]
    for k in range(80):
        data = bytearray(open(os.path.join(EXR, names[int(rng.integers(0, len(names)))]), "rb").read())
        for _ in range(1 + k % 3):
            data[int(rng.integers(0, len(data)))] ^= int(rng.integers(1, 256))
        data = bytes(data)
        oc, ow, oh, oimg = O.decode(data)
        code, w, h, img = ctx.exr_decode(data)
        assert (code, w, h) == (oc, ow, oh), k
        if oc == 0:
            assert np.array_equal(img.view(np.uint32), oimg.view(np.uint32)), k


def test_exr_piz_damage(ctx):
    """Random damage to PIZ and level fixtures: the GPU's code and bits equal the oracle's
    (damaged Huffman data decodes to what tinyexr keeps: it ignores hufUncompress's failure)."""
    rng = np.random.default_rng(12)
    names = [n for n in sorted(MAN) if MAN[n]["code"] == 0 and ("piz" in n or n.startswith(("mip", "rip")))
             and "w16" not in n and "longcodes" not in n]
    for k in range(60):
        data = bytearray(open(os.path.join(EXR, names[int(rng.integers(0, len(names)))]), "rb").read())
        lo = len(data) // 3 if k % 2 else 0
        for _ in range(1 + k % 4):
            data[int(rng.integers(lo, len(data)))] ^= int(rng.integers(1, 256))
        data = bytes(data)
        oc, ow, oh, oimg = O.decode(data)
        code, w, h, img = ctx.exr_decode(data)
        assert (code, w, h) == (oc, ow, oh), k
        if oc == 0:
            assert np.array_equal(img.view(np.uint32), oimg.view(np.uint32)), k


def test_image_read_exr(tmp_path):
    """Image.read('.exr') = readExr: d = 4, FLOAT, the decoded floats' bytes; a broken file raises."""
    name = "scan_zip_half.exr"
    p = tmp_path / "a.exr"
    p.write_bytes(open(os.path.join(EXR, name), "rb").read())
    im = icx.Image()
    im.read(str(p))
    assert (im.cols(), im.rows(), im.d_, im.type_) == (MAN[name]["w"], MAN[name]["h"], 4, icx.Image.FLOAT)
    assert hashlib.sha256(im.pixels_.tobytes()).hexdigest() == MAN[name]["sha256"]
    q = tmp_path / "b.exr"
    q.write_bytes(open(os.path.join(EXR, "zip_bad_adler.exr"), "rb").read())
    with pytest.raises(RuntimeError):
        icx.Image().read(str(q))


def test_exr_decode_device_matches_host_entry(ctx):
    """icx_exr_decode_device (file resident on the device, floats to device memory) returns the
    host entry's code and the same float bits on every fixture that decodes (scanline, tiled,
    PIZ, mip / rip levels) and on those whose pixel data fails; an output buffer one float short is
    a call-level error."""
    import torch
    dev = torch.device("cuda", 0)
    for name in sorted(MAN):
        data = open(os.path.join(EXR, name), "rb").read()
        code, w, h, img = ctx.exr_decode(data)
        if code not in (0, icx.EXR_INVALID_DATA):
            continue
        d_file = torch.zeros(len(data) + 16, dtype=torch.uint8, device=dev)
        d_file[:len(data)] = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).to(dev)
        pw, ph = icx.exr_probe(data)[1:3] if code != 0 else (w, h)
        n = max(1, pw * ph * 4)
        d_out = torch.full((n,), -1.0, dtype=torch.float32, device=dev)
        c2, w2, h2 = ctx.exr_decode_device(data, d_file.data_ptr(), d_out.data_ptr(), n)
        assert c2 == code, name
        if code == 0:
            assert (w2, h2) == (w, h), name
            got = d_out.cpu().numpy().reshape(h, w, 4)
            assert sha(got) == sha(img), name
    data = open(os.path.join(EXR, "scan_zip_half.exr"), "rb").read()
    code, w, h, _ = ctx.exr_decode(data)
    assert code == 0
    d_file = torch.zeros(len(data) + 16, dtype=torch.uint8, device=dev)
    d_file[:len(data)] = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).to(dev)
    d_out = torch.zeros(w * h * 4, dtype=torch.float32, device=dev)
    with pytest.raises(icx.ICXError):
        ctx.exr_decode_device(data, d_file.data_ptr(), d_out.data_ptr(), w * h * 4 - 1)
    # the chunk readers load 16-byte words, so a misaligned device copy is refused
    d_odd = torch.zeros(len(data) + 17, dtype=torch.uint8, device=dev)
    d_odd[1:1 + len(data)] = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).to(dev)
    assert ctx.exr_decode_device(data, d_odd.data_ptr() + 1, d_out.data_ptr(), w * h * 4)[0] == icx.EXR_INVALID_ARGUMENT


def test_exr_decode_device_batch_matches_single(ctx):
    """icx_exr_decode_device_batch over every fixture at once (planning failures, pixel-data
    failures, scanline / tiled / PIZ / level files mixed in one call): per-file codes, sizes and
    float bits equal the single-file host entry's."""
    import torch
    dev = torch.device("cuda", 0)
    names = sorted(MAN)
    datas = [open(os.path.join(EXR, nm), "rb").read() for nm in names]
    ref = [ctx.exr_decode(d) for d in datas]
    files, outs, room = [], [], []
    for d, nm in zip(datas, names):
        f = torch.zeros(len(d) + 16, dtype=torch.uint8, device=dev)
        if len(d):
            f[:len(d)] = torch.from_numpy(np.frombuffer(d, np.uint8).copy()).to(dev)
        files.append(f)
        pw, ph = icx.exr_probe(d)[1:3]
        n = max(1, pw * ph * 4)
        outs.append(torch.full((n,), -1.0, dtype=torch.float32, device=dev))
        room.append(n)
    codes, ws, hs = ctx.exr_decode_device_batch(datas, [f.data_ptr() for f in files], [o.data_ptr() for o in outs], room)
    for k, (nm, (code, w, h, img)) in enumerate(zip(names, ref)):
        assert codes[k] == code, nm
        if code == 0:
            assert (ws[k], hs[k]) == (w, h), nm
            assert sha(outs[k].cpu().numpy()[: w * h * 4].reshape(h, w, 4)) == sha(img), nm


def test_exr_piz_many_small_tiles(ctx):
    """PIZ files of many small tiles (4x4 tiles, mipmapped: 341 chunks per 64x64 file, more than
    k_exr_piz's 256 pool slots, so workgroups walk several chunks with one reused long-code
    slot), alone and three in one batch call: the oracle's bits (the per-chunk
    PizWork used to grow the scratch with the chunk count)."""
    import torch
    dev = torch.device("cuda", 0)
    datas, refs = [], []
    for k in range(2):
        rng = np.random.default_rng(50 + k)
        y, x = np.mgrid[0:64, 0:64].astype(np.float32)
        chans = [(n, (np.sin(x * (0.02 + 0.01 * j)) * np.cos(y * 0.03) * 9 + rng.normal(0, 0.1, x.shape)).astype(np.float16))
                 for j, n in enumerate("RGBA")]
        d = W.write_exr(chans, compression=W.PIZ, tiles=(4, 4), levels=1)
        oc, ow, oh, oimg = O.decode(d)
        assert (oc, ow, oh) == (0, 64, 64)
        code, w, h, img = ctx.exr_decode(d)
        assert (code, w, h) == (0, 64, 64)
        assert sha(img) == sha(oimg)
        datas.append(d)
        refs.append(oimg)
    datas.append(datas[0])  # (three files in the call, two of them the same bytes)
    refs.append(refs[0])
    files = []
    for d in datas:
        f = torch.zeros(len(d) + 16, dtype=torch.uint8, device=dev)
        f[:len(d)] = torch.from_numpy(np.frombuffer(d, np.uint8).copy()).to(dev)
        files.append(f)
    outs = [torch.zeros(64 * 64 * 4, dtype=torch.float32, device=dev) for _ in datas]
    codes, ws, hs = ctx.exr_decode_device_batch(datas, [f.data_ptr() for f in files], [o.data_ptr() for o in outs],
                                                [64 * 64 * 4] * 3)
    assert list(codes) == [0, 0, 0]
    for o, r in zip(outs, refs):
        assert sha(o.cpu().numpy().reshape(64, 64, 4)) == sha(r)
