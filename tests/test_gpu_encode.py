"""GPU encoder parity: the HIP tiny_jpeg path must produce the reference's exact bytes
(jpeg_enc.h; goldens from the reference build) and round-trip through the decoder."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
import imagecodecs_amd as icx
from oracle import pyoracle as O
from tools import synthpy as S

pytestmark = pytest.mark.gpu
TJE = json.load(open(os.path.join(GOLDEN, "tje_manifest.json")))


@pytest.fixture(scope="module")
def ctx():
    c = icx.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("key", sorted(TJE))
def test_tje_golden(ctx, key):
    e = TJE[key]
    if "rgb_hex" in e:
        px = bytes.fromhex(e["rgb_hex"])
    elif "source" in e:
        px = O.decode(open(os.path.join(GOLDEN, "test.jpg"), "rb").read())[4]
    else:
        px = open(os.path.join(GOLDEN, "tje", key.split(":")[0]), "rb").read()
    out = ctx.tje_encode(e["quality"], e["w"], e["h"], e["comps"], px)
    assert out is not None and len(out) == e["len"] and hashlib.sha256(out).hexdigest() == e["sha256"]


@pytest.mark.parametrize("q", [1, 2, 3])
def test_tje_large_matches_oracle_and_roundtrips(ctx, q):
    px = S.rgb(77 + q, 1024, 768, 3)
    out = ctx.tje_encode(q, 1024, 768, 3, px.tobytes())
    assert out == O.tje_encode(q, 1024, 768, 3, px.tobytes())
    code, w, h, n, dec = ctx.decode(out)
    assert code == 0 and (w, h, n) == (1024, 768, 3)
    assert dec == O.decode(out)[4]
    err = np.abs(np.frombuffer(dec, np.uint8).astype(int) - px.reshape(-1).astype(int)).max()
    assert err <= {1: 80, 2: 30, 3: 8}[q]


def test_tje_rejects_like_reference(ctx):
    assert ctx.tje_encode(0, 8, 8, 3, bytes(192)) is None
    assert ctx.tje_encode(3, 8, 8, 2, bytes(128)) is None


# ---- C4 encode extension: byte-exact to oracle/tje_oracle.c or_jpeg_encode -----------------
EXT = json.load(open(os.path.join(GOLDEN, "ext_manifest.json")))


@pytest.mark.parametrize("key", sorted(EXT))
def test_ext_manifest(ctx, key):
    e = EXT[key]
    px = S.rgb(e["seed"], e["w"], e["h"], e["comps"]).tobytes()
    out = ctx.jpeg_encode(e["quality"], e["subsampling"], e["w"], e["h"], e["comps"], px)
    assert out is not None and len(out) == e["len"] and hashlib.sha256(out).hexdigest() == e["sha256"]


@pytest.mark.parametrize("w,h,c", [(1, 1, 3), (16, 16, 3), (15, 17, 4), (640, 480, 3), (1023, 769, 4)])
@pytest.mark.parametrize("q,sub", [(1, 420), (10, 444), (50, 420), (90, 420), (90, 444), (100, 420)])
def test_ext_matches_oracle(ctx, w, h, c, q, sub):
    px = S.rgb(w * 31 + h + q, w, h, c).tobytes()
    out = ctx.jpeg_encode(q, sub, w, h, c, px)
    assert out == O.jpeg_encode(q, sub, w, h, c, px)


def test_ext_device_4096_roundtrip(ctx):
    """BASELINE's C4 workload shape (4096^2, 4:2:0, q90) through the device-resident entry."""
    import torch
    w = h = 4096
    px = S.rgb(2024, w, h, 3)
    enc = icx.Encoder(ctx)
    d_src = torch.from_numpy(px).cuda()
    d_out = torch.empty(8 << 20, dtype=torch.uint8, device="cuda")
    rc, n = enc.encode_device(90, 420, w, h, 3, d_src.data_ptr(), d_out.data_ptr(), 64)
    assert rc == icx.OUT_OF_MEM and n > 64  # size query without writing
    rc, n2 = enc.encode_device(90, 420, w, h, 3, d_src.data_ptr(), d_out.data_ptr(), d_out.numel())
    assert rc == icx.OK and n2 == n
    jpg = d_out[:n].cpu().numpy().tobytes()
    assert jpg == O.jpeg_encode(90, 420, w, h, 3, px.tobytes())
    code, dw, dh, nc, dec = ctx.decode(jpg)
    assert code == 0 and (dw, dh, nc) == (w, h, 3) and dec == O.decode(jpg)[4]
    enc.close()


def test_ext_rejects(ctx):
    px = bytes(8 * 8 * 4)
    assert ctx.jpeg_encode(0, 444, 8, 8, 3, px) is None
    assert ctx.jpeg_encode(101, 444, 8, 8, 3, px) is None
    assert ctx.jpeg_encode(90, 422, 8, 8, 3, px) is None
    assert ctx.jpeg_encode(90, 420, 8, 8, 2, px) is None
    assert ctx.jpeg_encode(90, 420, 0, 0, 3, b"") == O.jpeg_encode(90, 420, 0, 0, 3, b"")  # header + EOI


def test_ext_device_estimate_regrowth(ctx):
    """The device encoder sizes its stream buffer from the images before; a much larger stream is
    re-run at its exact size (same bytes), and an output that does not fit stays untouched."""
    import torch
    small, big = S.rgb(5, 64, 64, 3), S.rgb(6, 1024, 1024, 3)
    d_out = torch.empty(8 << 20, dtype=torch.uint8, device="cuda")
    enc = icx.Encoder(ctx)
    for px, w, h in ((small, 64, 64), (big, 1024, 1024), (small, 64, 64)):
        d_src = torch.from_numpy(px).cuda()
        rc, n = enc.encode_device(100, 444, w, h, 3, d_src.data_ptr(), d_out.data_ptr(), d_out.numel())
        assert rc == icx.OK
        assert d_out[:n].cpu().numpy().tobytes() == O.jpeg_encode(100, 444, w, h, 3, px.tobytes())
    enc.close()
    enc2 = icx.Encoder(ctx)  # small estimate again, then a big image into a 4 KiB output
    rc, _ = enc2.encode_device(100, 444, 64, 64, 3, torch.from_numpy(small).cuda().data_ptr(), d_out.data_ptr(),
                               d_out.numel())
    assert rc == icx.OK
    d_big = torch.from_numpy(big).cuda()
    d_out.fill_(0xAB)
    rc, n = enc2.encode_device(100, 444, 1024, 1024, 3, d_big.data_ptr(), d_out.data_ptr(), 4096)
    assert rc == icx.OUT_OF_MEM and n > 4096
    assert bool((d_out == 0xAB).all())
    enc2.close()


@pytest.mark.parametrize("q,sub,w,h", [(90, 420, 640, 480), (50, 444, 333, 251), (100, 420, 1024, 768)])
def test_ext_device_batch(ctx, q, sub, w, h):
    """icx_jpeg_encode_device_batch (one fused k_enc_run launch over every run of every image, one
    stuffing pass) gives each image the oracle's bytes; an image whose file exceeds the stride
    reports OUT_OF_MEM and leaves its slot alone."""
    import torch
    imgs = [S.rgb(300 + k, w, h, 3) for k in range(5)]
    d_src = [torch.from_numpy(px).cuda() for px in imgs]
    want = [O.jpeg_encode(q, sub, w, h, 3, px.tobytes()) for px in imgs]
    stride = (max(len(x) for x in want) + 64) | 1  # odd: images 1.. start at every byte alignment
    d_out = torch.full((5 * stride,), 0xAB, dtype=torch.uint8, device="cuda")
    enc = icx.Encoder(ctx)
    st, sizes = enc.encode_device_batch(q, sub, w, h, 3, [t.data_ptr() for t in d_src], d_out.data_ptr(), stride)
    assert list(st) == [icx.OK] * 5 and list(sizes) == [len(x) for x in want]
    out = d_out.cpu().numpy()
    for k in range(5):
        assert out[k * stride: k * stride + sizes[k]].tobytes() == want[k]
    small = min(len(x) for x in want) - 1  # every image too large
    d_out.fill_(0xAB)
    st, sizes = enc.encode_device_batch(q, sub, w, h, 3, [t.data_ptr() for t in d_src], d_out.data_ptr(), small)
    assert list(st) == [icx.OUT_OF_MEM] * 5 and list(sizes) == [len(x) for x in want]
    assert bool((d_out == 0xAB).all())
    enc.close()


def test_ext_device_batch_regrowth_and_launch_split(ctx, monkeypatch):
    """A batch whose words-buffer estimate comes from small flat images meets a large noisy one
    (its stream outgrows the buffer: that image alone is encoded again), and the same batch cut
    into launches of two images (ICX_ENC_BATCH): oracle bytes either way. The images differ in
    content, so every launch interleaves look-back chains of different lengths."""
    import torch
    w, h = 512, 384
    flat = np.zeros((h, w, 3), np.uint8)
    flat[:, :, 0] = np.arange(w, dtype=np.uint8)[None, :]
    imgs = [flat, S.rgb(41, w, h, 3), flat.copy(), S.rgb(42, w, h, 3), flat.copy()]
    want = [O.jpeg_encode(100, 444, w, h, 3, px.tobytes()) for px in imgs]
    d_src = [torch.from_numpy(np.ascontiguousarray(px)).cuda() for px in imgs]
    stride = max(len(x) for x in want) + 64
    enc = icx.Encoder(ctx)
    d_flat = torch.from_numpy(flat).cuda()
    d_out = torch.empty(stride * 5, dtype=torch.uint8, device="cuda")
    rc, _ = enc.encode_device(100, 444, w, h, 3, d_flat.data_ptr(), d_out.data_ptr(), stride)  # small estimate
    assert rc == icx.OK
    for split in (None, "2"):
        if split:
            monkeypatch.setenv("ICX_ENC_BATCH", split)
        d_out.fill_(0xAB)
        st, sizes = enc.encode_device_batch(100, 444, w, h, 3, [t.data_ptr() for t in d_src], d_out.data_ptr(), stride)
        assert list(st) == [icx.OK] * 5 and list(sizes) == [len(x) for x in want]
        out = d_out.cpu().numpy()
        for k in range(5):
            assert out[k * stride: k * stride + sizes[k]].tobytes() == want[k], (split, k)
    enc.close()
