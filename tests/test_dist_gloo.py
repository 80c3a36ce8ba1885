"""Multi-process (world_size 2, gloo on CPU) coverage of the N>1 path: key and
table broadcast from rank 0, byte-balanced contiguous sharding, per-rank
processing (oracle stands in for the kernel here — no GPU on CPU runners),
hit-histogram sum and max-over-ranks timing.  The union of the shards must
equal the single-process result exactly."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from smart_nic_amd import dist as sdist
from smart_nic_amd import pktgen

MS_KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    from oracle import pyoracle as po

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank 0 owns the configuration; everyone else starts from garbage
        if rank == 0:
            key = torch.tensor(list(MS_KEY), dtype=torch.uint8)
            table = torch.from_numpy((np.arange(128) % 16).astype(np.int32))
        else:
            key = torch.zeros(40, dtype=torch.uint8)
            table = torch.full((128,), -1, dtype=torch.int32)
        key, table = sdist.broadcast_rss_config(key, table, dist)
        rng = np.random.default_rng(3)
        lens = pktgen.imix_lengths(3000, rng)
        frames, desc, _ = pktgen.make_batch(lens, seed=3, proto=17)
        bounds = sdist.shard_by_bytes(lens, world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        cs, h, qq, _, hits = po.rx_batch(frames, desc[lo:hi], bytes(key.numpy()), table.numpy().view(np.uint16))
        hits_t = torch.from_numpy(hits.astype(np.int64))
        sdist.sum_hits(hits_t, dist)
        t = sdist.max_over_ranks(float(rank + 1), dist)
        q.put((rank, lo, hi, cs, h, qq, hits_t.numpy(), t, bytes(key.numpy()), table.numpy().copy(),
               int(lens[lo:hi].sum())))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_matches_single_process():
    from oracle import pyoracle as po

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(3)
    lens = pktgen.imix_lengths(3000, rng)
    frames, desc, _ = pktgen.make_batch(lens, seed=3, proto=17)
    table = (np.arange(128) % 16).astype(np.uint16)
    cs, h, qq, _, hits = po.rx_batch(frames, desc, MS_KEY, table)
    assert res[0][1] == 0 and res[0][2] == res[1][1] and res[1][2] == 3000
    np.testing.assert_array_equal(np.concatenate([r[3] for r in res]), cs)
    np.testing.assert_array_equal(np.concatenate([r[4] for r in res]), h)
    np.testing.assert_array_equal(np.concatenate([r[5] for r in res]), qq)
    for r in res:
        np.testing.assert_array_equal(r[6].astype(np.uint64), hits)  # summed histogram on every rank
        assert r[7] == 2.0  # max over ranks
        assert r[8] == MS_KEY  # broadcast key
        np.testing.assert_array_equal(r[9].view(np.uint16), table)
    # byte balance: shards within one max-size packet of each other
    assert abs(res[0][10] - res[1][10]) <= 1518 * 2


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_by_bytes_properties(world):
    rng = np.random.default_rng(world)
    for n in [0, 1, 5, 100, 4097]:
        lens = pktgen.imix_lengths(n, rng) if n else np.zeros(0, np.int64)
        b = sdist.shard_by_bytes(lens, world)
        assert b[0] == 0 and b[-1] == n and np.all(np.diff(b) >= 0)
        if world > 1:
            assert b.size == world + 1
            if n >= world:
                assert np.all(np.diff(b) >= 1)
            if n >= 100 * world:
                per = np.array([lens[b[r]:b[r + 1]].sum() for r in range(world)])
                assert per.max() - per.min() <= 2 * 1518
