"""Where images leave the parallel entropy path, and what that costs (VERDICT r2 weak #7 / next #6,
VERDICT r3 next #6).

* Capacity: a group's unstuffed-byte pool and lane records are sized for 2 B/px on average
  (ICX_UPOOL_BPP). A batch whose scans pass it (4:4:4 q100 images are 2.5 B/px here) defers the
  images that do not fit to further entropy rounds over the freed pools (k_spec_plan, up to eight
  rounds, ICX_ROUNDS), never to the one-lane sequential kernel: every round after the first plans
  at least a pool's worth, and conforming scans stay far below 8 B/px.
* What still goes sequential: streams NanoJPEG decodes that the parallel path cannot take --
  more than 16 blocks per MCU (beyond the JPEG limit of 10 blocks per MCU, so non-conforming),
  a restart marker that NanoJPEG reads where no lane starts, or (with ICX_ROUNDS lowered) a batch
  deeper than the rounds. They decode bit-exactly; their cost is measured here and stated in
  DESIGN.md.
"""
import time

import pytest

import imagecodecs_amd as icx
from driutil import elsewhere_case
from oracle import pyoracle as O
from tools import synthpy as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = icx.Context(0)
    yield c
    c.close()


def _check(res, jpegs):
    for j, (code, w, h, n, pix) in zip(jpegs, res):
        ocode, ow, oh, on, opix = O.decode(j)
        assert (code, w, h) == (ocode, ow, oh)
        if code == 0:
            assert pix.tobytes() == opix


@pytest.mark.parametrize("rounds,parallel", [(None, 16), ("1", None), ("3", 16)])
def test_pool_overflow_deferred_to_next_round(ctx, monkeypatch, rounds, parallel):
    """16 slots of 512^2 over two pipelines (8 each), 16 images at 2.5 B/px, the U pool cut to
    1 B/px (10 slots x 256 KiB per pipeline: about 3 images a round). The default rounds or three:
    all 16 on the parallel path. One round: the rest go to the sequential kernel (the old
    behaviour) -- bit-exact either way."""
    monkeypatch.setenv("ICX_UPOOL_BPP", "1")  # (so a pool holds ~3 of these images)
    if rounds is None:
        monkeypatch.delenv("ICX_ROUNDS", raising=False)
    else:
        monkeypatch.setenv("ICX_ROUNDS", rounds)
    jpegs = [S.synth_jpeg(6100 + k, 512, 512, "444", 100) for k in range(16)]
    assert sum(len(j) for j in jpegs) > 18 * 512 * 512  # more than one pool's worth
    b = icx.Batch(ctx, 16, 512, 512, group=16)
    res = b.decode_host(jpegs)
    st = b.path_stats()
    if parallel is not None:
        assert st == {"parallel": parallel, "fallback": 0, "sequential": 0}, st
    else:
        assert st["parallel"] < 16 and st["parallel"] + st["sequential"] == 16, st
    _check(res, jpegs)
    b.close()


def test_pool_overflow_beyond_rounds_is_exact(ctx, monkeypatch):
    """One group of 20 at 2.5 B/px against a pool of 22 x 512 KiB, one round (ICX_ROUNDS=1): what
    fits takes the parallel path, the rest the sequential kernel; every image bit-exact."""
    monkeypatch.delenv("ICX_UPOOL_BPP", raising=False)
    monkeypatch.setenv("ICX_ROUNDS", "1")
    jpegs = [S.synth_jpeg(6200 + k, 512, 512, "444", 100) for k in range(20)]
    b = icx.Batch(ctx, 20, 512, 512, group=20)
    res = b.decode_host(jpegs)
    st = b.path_stats()
    assert st["parallel"] + st["sequential"] == 20 and st["sequential"] > 0, st
    _check(res, jpegs)
    b.close()


def test_deep_batch_never_sequential(ctx, monkeypatch, capsys):
    """ten 4096^2 4:4:4 q100 images (2.5 B/px) in one group whose U pool is cut
    to 1 B/px (ICX_UPOOL_BPP=1: 12 x 16 MiB), so the batch is more than two pools deep. With the
    default rounds every image takes the parallel path (sequential == 0), bit-exact, and the
    batch costs less than twice the time per compressed byte of a clean 4:2:0 q90 batch of the
    same size decoded in one round."""
    monkeypatch.delenv("ICX_ROUNDS", raising=False)
    monkeypatch.setenv("ICX_UPOOL_BPP", "1")
    monkeypatch.setenv("ICX_PIPES", "1")  # (one workspace of 10 slots: a 12-slot U pool)
    W, N = 4096, 10
    from multiprocessing.pool import ThreadPool
    with ThreadPool(8) as p:  # (the generator is C through ctypes)
        deep = p.map(lambda k: S.synth_jpeg(6500 + k, W, W, "444", 100), range(N))
        clean = p.map(lambda k: S.synth_jpeg(6600 + k, W, W, "420", 90), range(N))
    assert sum(len(j) for j in deep) > 2 * 12 * W * W  # more than two pools
    b = icx.Batch(ctx, N, W, W, group=N)

    def run(batch):
        b.decode_host(batch)  # (warm)
        t0 = time.perf_counter()
        res = b.decode_host(batch)
        return time.perf_counter() - t0, res

    t_clean, _ = run(clean)
    t_deep, res = run(deep)
    st = b.path_stats()
    assert st == {"parallel": N, "fallback": 0, "sequential": 0}, st
    _check(res, deep)
    per_clean = t_clean / sum(len(j) for j in clean)
    per_deep = t_deep / sum(len(j) for j in deep)
    with capsys.disabled():
        print(f"\n  {N} x 4096^2: 4:2:0 q90 {t_clean * 1e3:.1f} ms ({sum(map(len, clean)) / 1e6:.0f} MB), "
              f"4:4:4 q100 over >2 pools {t_deep * 1e3:.1f} ms ({sum(map(len, deep)) / 1e6:.0f} MB)")
    assert per_deep < 2 * per_clean, (t_deep, t_clean)
    b.close()


def test_sequential_fallback_cost(ctx, capsys):
    """A 64-image 512^2 batch with one non-conforming 18-blocks-per-MCU image and one DRI image
    whose restart marker NanoJPEG reads where no lane starts: both decode exactly (the only two),
    on the sequential kernel, and what they add is one image's serial walk each (~40-60 ms for a
    512^2 image on one MI355X lane), not a per-batch cost.

    The two walks run side by side (the batch's two pipelines, one image each): the time they
    add to the clean batch stays under 1.5x the slower one decoded alone. Two walks that
    serialise (70 -> 149 ms between rounds; a kernel trace of this test in round 5
    showed them overlapped, 60 and 41 ms) add their sum and fail. Each time is the best of three
    calls, so a host hiccup in one call does not decide it."""
    clean = [S.synth_jpeg(6300 + k % 8, 512, 512, "420", 90) for k in range(64)]
    bad = list(clean)
    bad[5] = S.synth_jpeg(6399, 512, 512, "y44", 90)
    bad[40], _ = elsewhere_case()
    b = icx.Batch(ctx, 64, 512, 512)

    def run(batch):
        res = b.decode_host(batch)  # (warm)
        best = float("inf")
        for _ in range(3):
            t0 = time.perf_counter()
            b.decode_host(batch)
            best = min(best, time.perf_counter() - t0)
        return best, res

    t_clean, _ = run(clean)
    t_bad, res = run(bad)
    st = b.path_stats()  # (of the last call)
    assert st["parallel"] == 62 and st["fallback"] + st["sequential"] == 2, st
    _check(res, bad)
    t_one = [run([bad[k]])[0] for k in (5, 40)]  # each walk alone
    added = t_bad - t_clean
    with capsys.disabled():
        print(f"\n  64 x 512^2: clean {t_clean * 1e3:.1f} ms, with 2 sequential images {t_bad * 1e3:.1f} ms "
              f"(+{added * 1e3:.1f}); alone {t_one[0] * 1e3:.1f} / {t_one[1] * 1e3:.1f} ms")
    assert added < 1.5 * max(t_one), (t_bad, t_clean, t_one)
    b.close()


def test_full_group_half_flat_photos_stay_parallel(ctx):
    """a full group of 4096^2 photos whose top half is flat (a gradient with no
    noise: a few bits per block, so the lanes over it hold thousands of blocks each and overflow
    their static slots into the coefficient pool's tail) and whose bottom half is textured: every
    image stays on the parallel path (fallback == 0, sequential == 0), bit-exact (four of them
    checked against the oracle)."""
    import numpy as np
    from multiprocessing.pool import ThreadPool
    from tools import foreign
    W, N = 4096, 24

    def make(k):
        px = foreign.photo(6700 + k, W, W)
        g = np.linspace(40, 220, W // 2, dtype=np.float32)[:, None]
        px[: W // 2, :, 0] = g.astype(np.uint8)
        px[: W // 2, :, 1] = (g * 0.8 + 20).astype(np.uint8)
        px[: W // 2, :, 2] = (255 - g).astype(np.uint8)
        return S.jpeg(px, "420", 90)

    with ThreadPool(8) as p:
        jpegs = p.map(make, range(N))
    b = icx.Batch(ctx, N, W, W, group=N)
    res = b.decode_host(jpegs)
    st = b.path_stats()
    assert st == {"parallel": N, "fallback": 0, "sequential": 0}, st
    assert all(r[0] == 0 for r in res)
    _check(res[:4], jpegs[:4])
    b.close()


@pytest.mark.parametrize("how", ["capture", "env"])
def test_batch_decode_without_host_waits(ctx, monkeypatch, how):
    """icx_jpeg_batch_decode waits on the host for each group's plan (to launch only
    the entropy rounds a group needs). Under stream capture it must not: the decode is captured
    into a graph (every round and every layout's back half enqueued), replayed, and gives the
    oracle's pixels on a batch deep enough to need several rounds; ICX_HOST_WAIT=0 takes the same
    form eagerly."""
    import numpy as np
    import torch
    dev = torch.device("cuda", 0)
    monkeypatch.setenv("ICX_UPOOL_BPP", "1")  # (a pool holds ~3 of these images: several rounds)
    if how == "env":
        monkeypatch.setenv("ICX_HOST_WAIT", "0")
    jpegs = [S.synth_jpeg(6300 + k, 512, 512, "444", 100) for k in range(12)] + \
            [S.synth_jpeg(6320 + k, 512, 384, "420", 90) for k in range(4)]
    n = len(jpegs)
    sizes = [len(j) for j in jpegs]
    offs = np.cumsum([0] + sizes[:-1]).astype(np.int64)
    data = torch.from_numpy(np.frombuffer(b"".join(jpegs), np.uint8).copy()).to(dev)
    d_off = torch.from_numpy(offs).to(dev)
    d_sz = torch.from_numpy(np.array(sizes, np.int64)).to(dev)
    stride = 512 * 512 * 3
    out = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    st = torch.full((n,), -1, dtype=torch.int32, device=dev)
    dims = torch.zeros((n, 3), dtype=torch.int32, device=dev)
    b = icx.Batch(ctx, n, 512, 512, group=16)
    args = (n, data.data_ptr(), d_off.data_ptr(), d_sz.data_ptr(), out.data_ptr(), stride, st.data_ptr(), dims.data_ptr())
    if how == "capture":
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            b.decode_device(*args, torch.cuda.current_stream(dev).cuda_stream)
        assert int(st[0].item()) == -1  # captured, not run
        g.replay()
    else:
        b.decode_device(*args, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    assert b.path_stats() == {"parallel": n, "fallback": 0, "sequential": 0}
    st, dims, out = st.cpu().numpy(), dims.cpu().numpy(), out.cpu().numpy()
    for i, j in enumerate(jpegs):
        code, w, h, nc, pix = O.decode(j)
        assert st[i] == code == 0 and tuple(dims[i]) == (w, h, nc)
        assert out[i * stride: i * stride + w * h * nc].tobytes() == pix
    b.close()
