"""Per-image records and the C-ABI multi-GPU decode.

icx_jpeg_records computes {status, w, h, ncomp, checksum64} on the device; icx_multi_decode_host
shards a batch by compressed size over several devices (one thread, context, workspace and
stream each) and gathers records and pixels. On a one-GPU box the multi-device path runs with
the device listed twice: two contexts, two workspaces, two threads, the same sharding and
gather code as on an 8-GPU node. Records must equal the oracle's pixels' checksums."""
import numpy as np
import pytest

import imagecodecs_amd as icx
from imagecodecs_amd import shard
from oracle import pyoracle as O
from tools import synthpy as S

pytestmark = pytest.mark.gpu


def _jobs():
    jpegs = [S.synth_jpeg(800 + k, 64 + 97 * k, 48 + 61 * k, ["420", "444", "422", "gray", "420"][k % 5], 40 + 7 * k)
             for k in range(10)]
    jpegs[3] = jpegs[3][: len(jpegs[3]) // 3]         # truncated scan -> NJ_SYNTAX_ERROR (or OK per NanoJPEG)
    jpegs.append(b"\xff\xd8\xff\xc2" + jpegs[0][4:])   # SOF2 -> NJ_UNSUPPORTED
    jpegs.append(b"not a jpeg")                        # NJ_NO_JPEG
    return jpegs


def _expect(j):
    code, w, h, n, pix = O.decode(j)
    return (code, w, h, n, shard.checksum64(pix)) if code == 0 else (code, 0, 0, 0, 0)


def _all_devices():
    import torch
    n = torch.cuda.device_count()
    return list(range(n)) if n > 1 else None


@pytest.mark.parametrize("devices", [[0], [0, 0], "all"])
def test_multi_decode_records_and_pixels(devices):
    """The records gather: RCCL over distinct devices (all of a multi-GPU box), host memory for one
    device or a device listed twice (RCCL needs distinct GPUs), with the same records either way."""
    if devices == "all":
        devices = _all_devices()
        if devices is None:
            pytest.skip("one GPU: the RCCL gather needs distinct devices")
    jpegs = _jobs()
    m = icx.Multi(devices, 1024, 1024)
    if len(set(devices)) > 1:
        assert m.gather == "rccl", m.gather
    else:
        assert m.gather.startswith("host ("), m.gather
    rec, owner, pix = m.decode_host(jpegs)
    assert list(owner) == list(icx.multi_shard([len(j) for j in jpegs], len(devices)))
    assert list(owner) == [next(r for r, p in enumerate(shard.shard_by_size([len(j) for j in jpegs], len(devices)))
                                if i in p) for i in range(len(jpegs))]
    if len(devices) > 1:
        assert len(set(owner)) == len(devices)
    for i, j in enumerate(jpegs):
        e = _expect(j)
        got = (int(rec[i]["status"]), int(rec[i]["width"]), int(rec[i]["height"]), int(rec[i]["ncomp"]),
               int(rec[i]["checksum"]))
        assert got == e, (i, got, e)
        if e[0] == 0:
            assert pix[i].tobytes() == O.decode(j)[4]
    m.close()


def test_records_device_after_batch_decode():
    """icx_jpeg_records on a device-resident batch (unaligned out_stride: the byte-assembled path)."""
    import torch
    jpegs = _jobs()
    ctx = icx.Context(0)
    for extra in (0, 3):
        stride = 1024 * 1024 * 3 + extra
        n = len(jpegs)
        sizes = np.array([len(j) for j in jpegs], np.int64)
        offs = np.zeros(n, np.int64)
        offs[1:] = np.cumsum((sizes[:-1] + 15) // 16 * 16)
        blob = np.zeros(int(offs[-1] + sizes[-1]), np.uint8)
        for i, j in enumerate(jpegs):
            blob[offs[i]: offs[i] + sizes[i]] = np.frombuffer(j, np.uint8)
        dev = torch.device("cuda", 0)
        d_data, d_off, d_sz = (torch.from_numpy(x).to(dev) for x in (blob, offs, sizes))
        d_out = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
        d_st = torch.empty(n, dtype=torch.int32, device=dev)
        d_dims = torch.empty((n, 3), dtype=torch.int32, device=dev)
        d_rec = torch.empty(n * 24, dtype=torch.uint8, device=dev)
        b = icx.Batch(ctx, n, 1024, 1024)
        s = torch.cuda.current_stream(dev).cuda_stream
        b.decode_device(n, d_data.data_ptr(), d_off.data_ptr(), d_sz.data_ptr(), d_out.data_ptr(), stride,
                        d_st.data_ptr(), d_dims.data_ptr(), s)
        icx.records_device(ctx, n, d_out.data_ptr(), stride, d_st.data_ptr(), d_dims.data_ptr(), 1024, 1024,
                           d_rec.data_ptr(), s)
        torch.cuda.synchronize(dev)
        rec = d_rec.cpu().numpy().view(icx.RECORD_DTYPE)
        t = shard.records_from_numpy(rec).numpy()
        for i, j in enumerate(jpegs):
            e = _expect(j)
            assert (int(rec[i]["status"]), int(rec[i]["width"]), int(rec[i]["height"]), int(rec[i]["ncomp"]),
                    int(rec[i]["checksum"])) == e
            assert int(t[i:i + 1, 4].view(np.uint64)[0]) == e[4]
        b.close()
    ctx.close()
