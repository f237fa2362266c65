"""Multi-process sharding and the final status gather (imagecodecs_amd/shard.py) on gloo with
world_size 2 -- the same code bench.py runs over RCCL on the GPU node."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from imagecodecs_amd import shard


def test_shard_range_partitions():
    for n in (0, 1, 7, 512, 4096, 4097):
        for world in (1, 2, 3, 8):
            got = [shard.shard_range(n, world, r) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1
    assert shard.shard_range(4096, 8, 3) == (1536, 2048)  # C3: 512 images per GPU
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def test_shard_by_size_balances():
    sizes = [100, 1, 1, 1, 50, 50, 2, 3]
    parts = shard.shard_by_size(sizes, 2)
    assert sorted(i for p in parts for i in p) == list(range(len(sizes)))
    loads = [sum(sizes[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(sizes)
    assert sorted(loads) == [104, 104]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = shard.shard_range(n_total, world, rank)
    # each rank "decodes" its shard: status = image index % 6 (a stand-in for nj_result_t)
    local = torch.tensor([i % 6 for i in range(a, b)], dtype=torch.int32)
    full = shard.gather_results(local, dist)
    # max-over-ranks timing reduction, as bench.py does
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    q.put((rank, full.tolist(), float(t.item())))
    dist.destroy_process_group()


def test_gather_world2_gloo():
    world, n_total = 2, 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, full, tmax in res:
        assert full == [i % 6 for i in range(n_total)]
        assert tmax == 2.0


def _oracle_records(jpegs):
    """CPU stand-in for a rank's device records: the oracle decode of each image, with the
    checksum the records kernel computes (shard.checksum64, = icx_checksum64)."""
    import numpy as np
    from oracle import pyoracle as O
    rec = np.zeros((len(jpegs), 5), np.int64)
    for k, j in enumerate(jpegs):
        code, w, h, n, pix = O.decode(j)
        rec[k] = (code, w, h, n, np.int64(np.uint64(shard.checksum64(pix))) if code == 0 else 0) if code == 0 \
            else (code, 0, 0, 0, 0)
    return torch.from_numpy(rec)


def _jobs():
    from tools import synthpy as S
    jpegs = [S.synth_jpeg(600 + k, 40 + 23 * k, 30 + 11 * k, ["420", "444", "422", "gray"][k % 4], 50 + 5 * k)
             for k in range(9)]
    jpegs[4] = jpegs[4][: len(jpegs[4]) // 2]  # truncated -> a failed record in rank 1's shard
    jpegs.append(b"\xff\xd8\xff\xc2" + jpegs[0][4:])  # progressive marker -> NJ_UNSUPPORTED
    return jpegs


def _rec_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    jpegs = _jobs()
    parts = shard.shard_by_size([len(j) for j in jpegs], world)  # unequal shards
    mine = parts[rank]
    local = _oracle_records([jpegs[i] for i in mine])
    full, counts = shard.gather_records(local, dist)
    idx = torch.tensor(mine, dtype=torch.int64)
    all_idx, _ = shard.gather_records(torch.stack([idx] * 5, dim=1), dist)  # (indices ride the same gather)
    q.put((rank, full.tolist(), counts, all_idx[:, 0].tolist()))
    dist.destroy_process_group()


def test_gather_records_unequal_shards_world2_gloo():
    """Real records (oracle decodes of real JPEGs, incl. a truncated and a progressive one) from
    unequal shard_by_size shards, gathered over gloo with padding: rank order, counts and
    every record equal the serial computation."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rec_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    jpegs = _jobs()
    parts = shard.shard_by_size([len(j) for j in jpegs], world)
    assert len(parts[0]) != len(parts[1])
    want = _oracle_records(jpegs).tolist()
    for rank, full, counts, order in res:
        assert counts == [len(p) for p in parts]
        assert order == parts[0] + parts[1]
        assert [full[k] for k in range(len(order))] == [want[i] for i in order]
        assert sum(1 for r in full if r[0] != 0) == 2
