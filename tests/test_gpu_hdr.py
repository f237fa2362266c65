"""GPU Radiance .hdr decode parity (Image::readHdr, codecs.cpp:706-777).

Through the C ABI, every file of the shared corpus (tests/hdrutil.py: the reference's
data/test.hdr, seeded synthetic files in new-style RLE / flat / old-style RLE / mixed layouts,
header errors, truncations, undefined run-length data, fuzz) must give the oracle's result code,
size, decoded row count and float bits. The float step is exact (v * 2^(E-136) is representable
in binary32), so the stated epsilon is 0: bit-identical floats."""
import os

import numpy as np
import pytest

import hdrutil as H
import imagecodecs_amd as icx
from oracle import pyoracle as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def ctx():
    c = icx.Context(0)
    yield c
    c.close()


def _same(got, ref, name=""):
    gcode, gw, gh, grows, garr = got
    rcode, rw, rh, rrows, rarr = ref
    assert gcode == rcode, name
    if rcode in (O.HDR_OK, O.HDR_TRUNCATED, O.HDR_MALFORMED):
        assert (gw, gh, grows) == (rw, rh, rrows), name
        np.testing.assert_array_equal(garr.view(np.uint32), rarr.view(np.uint32), err_msg=name)


def test_hdr_reference_fixture(ctx):
    data = open(os.path.join(GOLDEN, "test.hdr"), "rb").read()
    got = ctx.hdr_decode(data)
    assert got[:4] == (icx.HDR_OK, 499, 289, 289)
    _same(got, O.hdr_decode(data), "test.hdr")
    assert icx.hdr_probe(data) == (icx.HDR_OK, 499, 289)


@pytest.mark.parametrize("case", H.valid_cases(), ids=lambda c: c[0])
def test_hdr_valid_files(ctx, case):
    name, data, px = case
    got = ctx.hdr_decode(data)
    assert got[0] == icx.HDR_OK
    np.testing.assert_array_equal(got[4].view(np.uint32), H.expected_floats(px).view(np.uint32))


def test_hdr_edge_files_single(ctx):
    for name, data in H.edge_cases():
        _same(ctx.hdr_decode(data), O.hdr_decode(data), name)


def _batch(ctx, files, max_w, max_h, pad=0):
    import torch
    dev = torch.device("cuda", 0)
    n = len(files)
    sizes = np.array([len(f) for f in files], np.int64)
    offs = np.zeros(n, np.int64)
    offs[1:] = np.cumsum(sizes)[:-1]
    blob = b"".join(files) or b"\0"
    data = torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).to(dev)
    d_off = torch.from_numpy(offs).to(dev)
    d_sz = torch.from_numpy(sizes).to(dev)
    stride = 4 * max_w * max_h + pad  # pad: floats, so images >= 1 may sit off 16-byte alignment
    out = torch.full((n * stride,), -7.0, dtype=torch.float32, device=dev)
    st = torch.full((n,), -9, dtype=torch.int32, device=dev)
    dims = torch.zeros((n, 3), dtype=torch.int32, device=dev)
    b = icx.HdrBatch(ctx, n, max_w, max_h)
    stream = torch.cuda.current_stream(dev).cuda_stream
    b.decode_device(n, data.data_ptr(), d_off.data_ptr(), d_sz.data_ptr(), out.data_ptr(), stride,
                    st.data_ptr(), dims.data_ptr(), stream)
    torch.cuda.synchronize(dev)
    times = b.stage_times()
    b.close()
    out, st, dims = out.cpu().numpy(), st.cpu().numpy(), dims.cpu().numpy()
    res = []
    for i in range(n):
        w, h, rows = (int(v) for v in dims[i])
        arr = out[i * stride: i * stride + w * h * 4].reshape(h, w, 4) if w * h else None
        res.append((int(st[i]), w, h, rows, arr))
    return res, times


def test_hdr_batch_mixed_corpus(ctx):
    files = [open(os.path.join(GOLDEN, "test.hdr"), "rb").read()]
    files += [f for _, f, _ in H.valid_cases()] + [f for _, f in H.edge_cases()]
    names = ["test.hdr"] + [n for n, _, _ in H.valid_cases()] + [n for n, _ in H.edge_cases()]
    res, times = _batch(ctx, files, 1000, 289)
    assert set(times) == {"parse", "locate", "unpack", "convert"}
    for name, f, got in zip(names, files, res):
        _same(got, O.hdr_decode(f), name)


@pytest.mark.parametrize("mode", [H.RLE, H.FLAT, H.OLD])
def test_hdr_batch_large(ctx, mode):
    """Many rows per image: the parallel locate paths (flat rows / linked new-style scanlines)
    and, for old-style RLE, the serial walk."""
    imgs = [H.S.rgbe(900 + k, w, h) for k, (w, h) in enumerate([(1024, 768), (640, 1100), (2000, 64)])]
    files = [H.S.hdr(px, mode) for px in imgs]
    files.append(H.mixed_file(77, 512, 300)[0])
    res, _ = _batch(ctx, files, 2000, 1100)
    for k, (f, got) in enumerate(zip(files, res)):
        ref = O.hdr_decode(f)
        assert ref[0] == O.HDR_OK
        _same(got, ref, f"large{k}")


def test_hdr_many_rows_beyond_candidate_cap(ctx):
    """More scanlines than k_hdr_link sorts (8192): located by the serial walk instead."""
    px = H.S.rgbe(5, 16, 9000)
    f = H.S.hdr(px, H.RLE)
    res, _ = _batch(ctx, [f], 16, 9000)
    assert res[0][0] == icx.HDR_OK
    np.testing.assert_array_equal(res[0][4].view(np.uint32), H.expected_floats(px).view(np.uint32))


@pytest.mark.parametrize("pad", [1, 2, 3])
def test_hdr_batch_unaligned_stride(ctx, pad):
    """out_stride not a multiple of 4 floats: images 1.. start off 16-byte alignment, and the
    convert kernel must fall back to scalar stores (same float bits)."""
    imgs = [H.S.rgbe(60 + k, 33 + 7 * k, 21 + 3 * k) for k in range(3)]
    files = [H.S.hdr(px, m) for px, m in zip(imgs, [H.RLE, H.FLAT, H.OLD])]
    res, _ = _batch(ctx, files, 64, 40, pad)
    for k, (f, got) in enumerate(zip(files, res)):
        _same(got, O.hdr_decode(f), f"pad{pad}/{k}")


def test_hdr_too_large_for_workspace(ctx):
    f = H.S.hdr(H.S.rgbe(3, 64, 20), H.RLE)
    ok = H.S.hdr(H.S.rgbe(4, 16, 8), H.RLE)
    res, _ = _batch(ctx, [f, ok], 32, 20)
    assert res[0][0] == icx.HDR_TOO_LARGE and res[0][1:4] == (0, 0, 0)
    _same(res[1], O.hdr_decode(ok))


def test_image_read_hdr(tmp_path):
    data = open(os.path.join(GOLDEN, "test.hdr"), "rb").read()
    p = tmp_path / "x.HDR"
    p.write_bytes(data)
    img = icx.Image()
    img.read(str(p))
    assert (img.cols(), img.rows(), img.channels(), img.type()) == (499, 289, 4, icx.Image.FLOAT)
    assert img.totalBytes() == 499 * 289 * 16
    ref = O.hdr_decode(data)[4]
    assert img.data().tobytes() == ref.tobytes()
    bad = tmp_path / "bad.hdr"
    bad.write_bytes(b"#?RGBE\n")
    with pytest.raises(RuntimeError):
        icx.Image().read(str(bad))
