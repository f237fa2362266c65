"""GPU parity tests (tier 2/3 of SURVEY.md §4): the HIP decode path through the C ABI vs the
oracle / the reference's golden vectors. Bit-exact for every byte (integer path)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
import imagecodecs_amd as icx
from oracle import pyoracle as O
from tools import synthpy as S
from driutil import dri_corruptions, elsewhere_case, rst_markers

pytestmark = pytest.mark.gpu

MANIFEST = json.load(open(os.path.join(GOLDEN, "decode_manifest.json")))
SYNTH = json.load(open(os.path.join(GOLDEN, "synth_manifest.json")))


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def ctx():
    c = icx.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_decode_golden(ctx, name):
    exp = MANIFEST[name]
    data = open(os.path.join(GOLDEN, name), "rb").read()
    code, w, h, n, pix = ctx.decode(data)
    assert code == exp["code"], (code, exp["code"])
    if code == icx.OK:
        assert (w, h, n) == (exp["w"], exp["h"], exp["ncomp"])
        assert sha(pix) == exp["sha256"]


def test_nanojpeg_state_api(ctx):
    data = open(os.path.join(GOLDEN, "test.jpg"), "rb").read()
    ctx.nj_init()
    assert ctx.nj_decode(data) == 0
    assert (ctx.nj_get_width(), ctx.nj_get_height(), ctx.nj_is_color()) == (499, 289, 1)
    assert ctx.nj_get_image_size() == 499 * 289 * 3
    assert sha(ctx.nj_get_image()) == MANIFEST["test.jpg"]["sha256"]
    ctx.nj_done()
    assert ctx.nj_get_image_size() == 0 and ctx.nj_get_image() == b""


def test_batch_mixed_goldens(ctx):
    """One batch holding every golden (sizes, samplings, DRI, corrupt files): per-image status,
    one bad image never fails the batch."""
    names = sorted(MANIFEST)
    jpegs = [open(os.path.join(GOLDEN, n), "rb").read() for n in names]
    b = icx.Batch(ctx, len(jpegs), 512, 512)
    res = b.decode_host(jpegs)
    stats = b.path_stats()
    # every stream takes a parallel path (DRI ones one lane per restart interval); only corrupt
    # DRI streams whose markers are not where NanoJPEG reads them go back to the sequential kernel
    n_bad_dri = sum(1 for nm in names if os.path.basename(nm).startswith("bad_dri"))
    assert stats["parallel"] >= 40 and stats["fallback"] <= n_bad_dri, stats
    for name, (code, w, h, n, pix) in zip(names, res):
        exp = MANIFEST[name]
        assert code == exp["code"], name
        if code == icx.OK:
            assert (w, h, n) == (exp["w"], exp["h"], exp["ncomp"]), name
            assert sha(pix.tobytes()) == exp["sha256"], name
    b.close()


@pytest.mark.parametrize("key", sorted(SYNTH))
def test_synth_large(ctx, key):
    e = SYNTH[key]
    data = S.synth_jpeg(e["seed"], e["w"], e["h"], e["sampling"], e["quality"], e["restart"])
    assert sha(data) == e["jpeg_sha256"]
    code, w, h, n, pix = ctx.decode(data)
    assert code == e["code"] == 0 and (w, h) == (e["w"], e["h"])
    assert sha(pix) == e["sha256"]


def _expected_groups(n, slots, pipes=2):
    """icx_api.cpp batch_split: the groups a call launches (ceil(n / per))."""
    want = min(n, -(-n // slots))
    per = -(-n // want)
    ng = -(-n // per)
    if pipes > 1 and ng > 1 and ng % pipes:
        up = -(-ng // pipes) * pipes
        if up <= n:
            per2 = -(-n // up)
            if -(-n // per2) % pipes == 0:
                per, ng = per2, -(-n // per2)
    return ng, per


@pytest.mark.parametrize("group,n", [(3, 10), (5, 9), (4, 4), (2, 7), (2, 5), (6, 7)])
def test_batch_group_count_balanced_and_exact(ctx, group, n):
    """A call is cut into equal groups; icx_batch_groups reports exactly the groups launched
    ((group 2, n 5) used to report 4 for 3 launched), a multiple of the two pipelines
    when rounding the count up still yields one ((6, 7): 3 -> 4 groups of 2; 3 groups on 2 pipes
    would run the third alone), and every cut decodes every image exactly as the oracle -- with
    the generic upsample's planes in the coefficient pool (a 4:4:4 / 4:2:2 / 4:1:1 / gray mix
    beside 4:2:0 in each group)."""
    samplings = ["420", "444", "422", "411", "gray", "440"]
    imgs = [S.synth_jpeg(4000 + k, 40 + 17 * k, 33 + 11 * k, samplings[k % len(samplings)], 60 + 4 * k) for k in range(n)]
    b = icx.Batch(ctx, n, 256, 256, group)
    g = b.groups_per_call(n)
    slots = b.group
    eg, per = _expected_groups(n, slots)
    assert g == eg and per <= slots and -(-n // per) == g, (g, eg, per, slots, n)
    if (group, n) == (6, 7):
        assert g == 4
    for data, (code, w, h, c, pix) in zip(imgs, b.decode_host(imgs)):
        ocode, ow, oh, on, opix = O.decode(data)
        assert (code, w, h) == (ocode, ow, oh) and pix.tobytes() == opix
    b.close()


def test_batch_out_of_capacity_is_oom(ctx):
    small = S.synth_jpeg(1, 64, 64)
    big = S.synth_jpeg(2, 200, 100)
    b = icx.Batch(ctx, 2, 128, 128)
    res = b.decode_host([small, big])
    assert res[0][0] == icx.OK and res[1][0] == icx.OUT_OF_MEM
    assert res[0][4].tobytes() == O.decode(small)[4]


@pytest.mark.parametrize("stride_extra", [1, 2, 3])
def test_decode_host_unaligned_out_stride(ctx, stride_extra):
    """An out_stride that is not a multiple of 4: images 1.. start at odd device addresses, so
    the dword-storing convert paths must check the image base (tiny 4:2:0 chroma and 4:1:1 take
    k_convert_fused / the generic passes)."""
    # chroma planes of 3 samples (W or H = 5..6 at 4:2:0) are below k_convert_stream's minimum of 4
    cases = [(6, 6, "420"), (5, 10, "420"), (10, 6, "420"), (12, 12, "420"), (36, 20, "411"), (64, 64, "422"),
             (100, 52, "420"), (24, 16, "440"), (6, 40, "422")]
    jpegs = [S.synth_jpeg(7000 + k, w, h, smp, 75) for k, (w, h, smp) in enumerate(cases)]
    b = icx.Batch(ctx, len(jpegs), 100, 64)
    res = b.decode_host(jpegs, out_stride=100 * 64 * 3 + stride_extra)
    for j, (code, w, h, n, pix) in zip(jpegs, res):
        ocode, ow, oh, on, opix = O.decode(j)
        assert code == ocode == 0 and (w, h, n) == (ow, oh, on)
        assert pix.tobytes() == opix
    b.close()


@pytest.mark.parametrize("group", [1200, 2400, 100000])
def test_batch_create_failure_frees_device_memory(ctx, group):
    """An explicit group too large for HBM fails part-way through the workspace allocation
    (inside pipe 0, or in pipe 1 after pipe 0 succeeded): nothing may stay allocated."""
    import torch
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(0)[0]
    with pytest.raises(icx.ICXError):
        icx.Batch(ctx, group, 4096, 4096, group)
    free1 = torch.cuda.mem_get_info(0)[0]
    assert free0 - free1 < 64 << 20, (free0, free1)
    # the failed hipMalloc is reported by icx, not left as HIP's sticky last error for torch
    x = torch.ones(1 << 20, device="cuda")
    torch.cuda.synchronize()
    assert float(x.sum()) == float(1 << 20)


def test_path_stats_after_device_decode_without_sync(ctx):
    """path_stats right after an asynchronous device decode: it must order itself after the
    decode's streams instead of reading stale counters."""
    import torch
    dev = torch.device("cuda", 0)
    jpegs = [S.synth_jpeg(7100 + i, 640, 480, "420", 90) for i in range(6)]
    sizes = [len(j) for j in jpegs]
    offs = np.cumsum([0] + sizes[:-1]).astype(np.uint64)
    data = torch.from_numpy(np.frombuffer(b"".join(jpegs), np.uint8).copy()).to(dev)
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_sz = torch.from_numpy(np.array(sizes, np.int64)).to(dev)
    stride = 640 * 480 * 3
    out = torch.zeros(len(jpegs) * stride, dtype=torch.uint8, device=dev)
    st = torch.zeros((len(jpegs),), dtype=torch.int32, device=dev)
    dims = torch.zeros((len(jpegs), 3), dtype=torch.int32, device=dev)
    b = icx.Batch(ctx, len(jpegs), 640, 480, 2)
    b.decode_device(len(jpegs), data.data_ptr(), d_off.data_ptr(), d_sz.data_ptr(), out.data_ptr(), stride,
                    st.data_ptr(), dims.data_ptr(), 0)
    assert b.path_stats() == {"parallel": len(jpegs), "fallback": 0, "sequential": 0}
    b.close()


def test_device_resident_batch_torch(ctx):
    """The throughput API: device pointers in, device pointers out, per-image statuses."""
    import torch
    dev = torch.device("cuda", 0)
    jpegs = [S.synth_jpeg(100 + i, 96 + 8 * i, 80 - 4 * i, ["420", "444", "422", "gray"][i % 4], 80, i % 2)
             for i in range(8)]
    sizes = [len(j) for j in jpegs]
    offs = np.cumsum([0] + sizes[:-1]).astype(np.uint64)
    data = torch.from_numpy(np.frombuffer(b"".join(jpegs), np.uint8).copy()).to(dev)
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_sz = torch.from_numpy(np.array(sizes, np.int64)).to(dev)
    stride = 160 * 96 * 3
    out = torch.zeros(len(jpegs) * stride, dtype=torch.uint8, device=dev)
    st = torch.full((len(jpegs),), -1, dtype=torch.int32, device=dev)
    dims = torch.zeros((len(jpegs), 3), dtype=torch.int32, device=dev)
    b = icx.Batch(ctx, len(jpegs), 160, 96)
    stream = torch.cuda.current_stream(dev).cuda_stream
    b.decode_device(len(jpegs), data.data_ptr(), d_off.data_ptr(), d_sz.data_ptr(), out.data_ptr(), stride,
                    st.data_ptr(), dims.data_ptr(), stream)
    torch.cuda.synchronize(dev)
    st, dims, out = st.cpu().numpy(), dims.cpu().numpy(), out.cpu().numpy()
    for i, j in enumerate(jpegs):
        code, w, h, n, pix = O.decode(j)
        assert st[i] == code == 0 and tuple(dims[i]) == (w, h, n)
        assert out[i * stride: i * stride + w * h * n].tobytes() == pix


@pytest.mark.parametrize("sampling", ["420", "444", "422", "gray", "440", "411"])
def test_parallel_path_large_bit_exact(ctx, sampling):
    """Several large images in one batch: all must take the parallel entropy path (no
    fallback) and match the oracle byte for byte."""
    jpegs = [S.synth_jpeg(300 + k, 777 + 64 * k, 555 + 32 * k, sampling, 60 + 15 * k) for k in range(3)]
    b = icx.Batch(ctx, len(jpegs), 1024, 1024)
    res = b.decode_host(jpegs)
    stats = b.path_stats()
    assert stats == {"parallel": 3, "fallback": 0, "sequential": 0}, stats
    for j, (code, w, h, n, pix) in zip(jpegs, res):
        ocode, ow, oh, on, opix = O.decode(j)
        assert code == ocode == 0 and (w, h, n) == (ow, oh, on)
        assert pix.tobytes() == opix


def test_parallel_path_coefficients_match_trace(ctx):
    """Stage-level parity: error-free random streams across sizes/qualities."""
    rng = np.random.default_rng(5)
    jpegs = []
    for k in range(24):
        w, h = int(rng.integers(16, 700)), int(rng.integers(16, 700))
        jpegs.append(S.synth_jpeg(900 + k, w, h, ["420", "444", "422", "gray"][k % 4], int(rng.integers(5, 100))))
    b = icx.Batch(ctx, len(jpegs), 700, 700)
    res = b.decode_host(jpegs)
    assert b.path_stats()["fallback"] == 0
    for j, (code, w, h, n, pix) in zip(jpegs, res):
        assert code == 0 and pix.tobytes() == O.decode(j)[4]


@pytest.mark.parametrize("restart,sampling", [(1, "420"), (7, "420"), (64, "444"), ("row", "422"), (1000, "420"),
                                              (3, "gray")])
def test_dri_parallel_bit_exact(ctx, restart, sampling):
    """Restart-interval (DRI) streams: one write lane per interval (jpeg_dec.h:707-715); every
    image stays on the parallel path and matches the oracle byte for byte."""
    dims = [(1024, 768), (1000, 1000), (640, 487)]
    jpegs = []
    for k, (w, h) in enumerate(dims):
        mcu_w = 8 if sampling in ("444", "gray") else 16
        r = (w + mcu_w - 1) // mcu_w if restart == "row" else restart
        jpegs.append(S.synth_jpeg(4000 + k, w, h, sampling, 85, r))
    b = icx.Batch(ctx, len(jpegs), 1024, 1024)
    res = b.decode_host(jpegs)
    stats = b.path_stats()
    assert stats == {"parallel": len(jpegs), "fallback": 0, "sequential": 0}, stats
    for j, (code, w, h, n, pix) in zip(jpegs, res):
        ocode, ow, oh, on, opix = O.decode(j)
        assert code == ocode == 0 and (w, h, n) == (ow, oh, on)
        assert pix.tobytes() == opix
    b.close()


def test_dri_corrupt_markers_decided_in_parallel(ctx):
    """Corrupt restart markers (wrong number, shifted, missing, doubled, swapped), flipped data
    and truncation: the first interval not ending at its marker decides the image on the parallel
    path (k_spec_write mode 3, dri_end_kind) -- NanoJPEG's status, no sequential decode -- and
    the images that stay OK match the oracle byte for byte."""
    rng = np.random.default_rng(41)
    cases = []
    for restart, smp in [(1, "420"), (5, "420"), (3, "gray"), (16, "444")]:
        cases += dri_corruptions(S.synth_jpeg(4100 + restart, 320, 240, smp, 80, restart), rng, 16)
    b = icx.Batch(ctx, len(cases), 320, 240)
    res = b.decode_host(cases)
    stats = b.path_stats()
    assert stats["fallback"] == 0 and stats["sequential"] == 0, stats
    for j, (code, w, h, n, pix) in zip(cases, res):
        ocode, _, _, _, opix = O.decode(j)
        assert code == ocode
        if code == 0:
            assert pix.tobytes() == opix
    b.close()


@pytest.mark.parametrize("gw_env", ["1", "0"])
def test_dri_guess_write_lanes_bit_exact(ctx, monkeypatch, gw_env):
    """Restart intervals on the guess-write path (ICX_GW=1 with ICX_DRI_GW=1: intervals from 512
    unstuffed bytes, cut into interval-aligned lanes, k_spec_plan/lane_span): long and short
    intervals, one batch, every sampling -- bit-exact against the oracle, all on the parallel path.
    ICX_DRI_GW=0 runs the same batch on the interval lanes alone."""
    monkeypatch.setenv("ICX_GW", "1")
    monkeypatch.setenv("ICX_DRI_GW", gw_env)
    specs = [(1024, 768, "420", 64), (1000, 1000, "420", 1000), (640, 487, "444", 64), (800, 600, "422", 50),
             (777, 555, "gray", 97), (1024, 1024, "420", 7), (512, 512, "420", 1), (1023, 999, "444", 300)]
    jpegs = [S.synth_jpeg(4400 + k, w, h, smp, 60 + 5 * k, r) for k, (w, h, smp, r) in enumerate(specs)]
    b = icx.Batch(ctx, len(jpegs), 1024, 1024)
    res = b.decode_host(jpegs)
    stats = b.path_stats()
    assert stats == {"parallel": len(jpegs), "fallback": 0, "sequential": 0}, stats
    for j, (code, w, h, n, pix) in zip(jpegs, res):
        ocode, ow, oh, on, opix = O.decode(j)
        assert code == ocode == 0 and (w, h, n) == (ow, oh, on)
        assert pix.tobytes() == opix
    b.close()


def test_dri_guess_write_corrupt_markers(ctx, monkeypatch):
    """Corrupt restart markers, flipped data and truncation on the guess-write DRI lanes: an image
    its lanes cannot decide exactly falls back to the interval lanes (dri_gw_fallback), which give
    NanoJPEG's status; the ones that stay OK match the oracle byte for byte. Nothing goes to the
    sequential kernel."""
    monkeypatch.setenv("ICX_GW", "1")
    monkeypatch.setenv("ICX_DRI_GW", "1")
    rng = np.random.default_rng(43)
    cases = []
    for seed, (w, h, smp, r) in enumerate([(640, 480, "420", 40), (640, 480, "444", 80), (640, 480, "gray", 40),
                                           (512, 512, "422", 64)]):
        cases += dri_corruptions(S.synth_jpeg(4500 + seed, w, h, smp, 85, r), rng, 24)
    b = icx.Batch(ctx, len(cases), 640, 512)
    res = b.decode_host(cases)
    stats = b.path_stats()
    assert stats["sequential"] == 0, stats
    for j, (code, w, h, n, pix) in zip(cases, res):
        ocode, _, _, _, opix = O.decode(j)
        assert code == ocode
        if code == 0:
            assert pix.tobytes() == opix
    b.close()


def test_dri_marker_read_elsewhere_falls_back_exactly(ctx):
    """FF D0+(j&7) at interval j's end that is stuffed data, not marker j: NanoJPEG resumes there,
    where no lane started, so that image alone goes to the sequential kernel -- with NanoJPEG's
    status and pixels."""
    v, _ = elsewhere_case()
    good = S.synth_jpeg(4200, 512, 512, "420", 90, 1)
    b = icx.Batch(ctx, 2, 512, 512)
    res = b.decode_host([v, good])
    assert b.path_stats() == {"parallel": 1, "fallback": 1, "sequential": 0}
    for j, (code, w, h, n, pix) in zip([v, good], res):
        ocode, _, _, _, opix = O.decode(j)
        assert code == ocode
        if code == 0:
            assert pix.tobytes() == opix
    b.close()


def test_corrupt_dri_images_cost_no_sequential_time(ctx):
    """A 64-image batch of 2048^2 DRI images (one interval per MCU row) with 8 corrupt ones
    (wrong marker numbers, a byte lost): all are decided on the parallel path, and the batch takes
    less than twice the clean batch's time (a sequential decode of one 2048^2 image alone takes
    longer than the whole clean batch)."""
    import time
    pool = [S.synth_jpeg(4300 + k, 2048, 2048, "420", 90, 128) for k in range(8)]
    clean = [pool[k % 8] for k in range(64)]
    bad = list(clean)
    for k in range(0, 64, 8):
        d = bytearray(pool[k // 8 % 8])
        mk = rst_markers(d)
        q = mk[len(mk) // 2 + k]
        if k % 16 == 0:
            d[q + 1] = 0xD0 + ((d[q + 1] + 3) & 7)
        else:
            del d[q - 1]
        bad[k] = bytes(d)
    b = icx.Batch(ctx, 64, 2048, 2048)

    def run(batch):
        b.decode_host(batch)  # (warm)
        t0 = time.perf_counter()
        res = b.decode_host(batch)
        return time.perf_counter() - t0, res

    t_clean, _ = run(clean)
    t_bad, res = run(bad)
    stats = b.path_stats()
    assert stats == {"parallel": 64, "fallback": 0, "sequential": 0}, stats
    for k in range(0, 64, 8):
        assert res[k][0] == O.decode(bad[k])[0] != 0
    assert res[1][0] == 0 and res[1][4].tobytes() == O.decode(clean[1])[4]
    assert t_bad < 2 * t_clean, (t_bad, t_clean)
    b.close()


@pytest.mark.parametrize("mode,seg", [("0", None), ("1", None), ("2", None), ("3", None), ("3", "1"), ("3", "3"), ("4", None), ("5", None)])
def test_420_plane_modes_bit_exact(ctx, monkeypatch, mode, seg):
    """Every 4:2:0 plane mode -- 0: k_idct, 1: k_idct420c + k_fused420 (luma IDCT inside the
    conversion), 2: k_idct420y + k_idct420c, 3: k_back420 (the whole back half, no planes; with
    1- and 3-MCU-row segments too, so most rows sit next to a segment edge), 4: k_idct420s (one lane
    per block, all three planes), 5 (default): k_idct420s for the chroma planes + k_fused420s (the
    one-lane luma IDCT inside the conversion, border lanes through the luma plane and
    k_convert_edge) -- decodes every golden and odd-sized synthetic 4:2:0 images exactly as the
    oracle."""
    monkeypatch.setenv("ICX_FUSE420", mode)
    if seg is not None:
        monkeypatch.setenv("ICX_BSEG", seg)
    names = sorted(MANIFEST)
    jpegs = [open(os.path.join(GOLDEN, n), "rb").read() for n in names]
    b = icx.Batch(ctx, len(jpegs), 512, 512)
    res = b.decode_host(jpegs)
    for n, (code, w, h, c, pix) in zip(names, res):
        exp = MANIFEST[n]
        assert code == exp["code"], n
        if code == icx.OK:
            assert sha(pix) == exp["sha256"], n
    rng = np.random.default_rng(420)
    imgs = []
    for k in range(6):
        w, h = int(rng.integers(17, 1500)), int(rng.integers(17, 700))
        imgs.append(S.synth_jpeg(900 + k, w, h, "420", int(rng.integers(30, 100))))
    b2 = icx.Batch(ctx, len(imgs), 1500, 700)
    for data, (code, w, h, c, pix) in zip(imgs, b2.decode_host(imgs)):
        ocode, ow, oh, on, opix = O.decode(data)
        assert (code, w, h) == (ocode, ow, oh) and pix.tobytes() == opix


def test_batch_create_failure_frees_partial_workspaces(ctx):
    """A batch whose second pipeline's workspace cannot be allocated (two pipes of 600 4096^2 slots,
    ~175 GB each, against 288 GB of HBM) fails cleanly and frees what it had already allocated:
    device free memory is unchanged after repeated failures (icx_batch_create leaked
    the first pipe's buffers on a partial failure)."""
    import torch

    torch.cuda.mem_get_info(0)  # (torch's own context first, so it is not counted below)
    free0, _ = torch.cuda.mem_get_info(0)
    for _ in range(2):
        with pytest.raises(icx.ICXError):
            icx.Batch(ctx, 1200, 4096, 4096, group=1200)
    free1, _ = torch.cuda.mem_get_info(0)
    assert abs(free1 - free0) < (256 << 20), (free0, free1)
