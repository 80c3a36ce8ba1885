"""Multi-process (world_size 2, gloo on CPU) coverage of the N>1 path: key and
table broadcast from rank 0, byte-balanced contiguous sharding, per-rank
processing (oracle stands in for the kernel here — no GPU on CPU runners),
hit-histogram sum and max-over-ranks timing.  Every rank processes its slice
of one job batch; the concatenated results must equal one single-process run
over the whole batch exactly."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from smart_nic_amd import dist as sdist
from smart_nic_amd import pktgen

JOB_SEED = 2024
MS_KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    """One rank of bench.py's multi-GPU path (smart_nic_amd.dist: init_ranks,
    plan_shard, setup_rss, job_queue_hits, max_over_ranks, finish) on gloo;
    the oracle stands in for the kernel (no GPU here)."""
    from oracle import pyoracle as po

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    ranks = sdist.init_ranks(backend="gloo")
    try:
        assert (ranks.rank, ranks.world) == (rank, world) and ranks.dist is not None
        # rank 0 owns the configuration; setup_rss zeroes it on the others
        # before the broadcast, so only a working broadcast gives them the key
        table = (np.arange(128) % 16) if rank == 0 else np.full(128, 7)
        key_t, tab_t = sdist.setup_rss(ranks, MS_KEY if rank == 0 else bytes(40), table)
        shard = sdist.plan_shard("c3", ranks, packets_per_gpu=1500)
        c2 = sdist.plan_shard("c2", ranks, packets_per_gpu=64)
        # the job batch, made once from one seed (as a NIC's ring would hold
        # it), and this rank's contiguous slice of it by the shard bounds
        job = pktgen.imix_lengths(3000, np.random.default_rng(sdist.WORKLOADS["c3"]["seed"]))
        assert np.array_equal(shard.lengths, job[shard.lo:shard.hi])
        frames, desc_all, _ = pktgen.make_batch(job, seed=JOB_SEED, proto=shard.proto)
        desc = np.ascontiguousarray(desc_all[shard.lo:shard.hi])
        cs, h, qq, _, hits = po.rx_batch(frames, desc, bytes(key_t.numpy()), tab_t.numpy().view(np.uint16))
        hits_t = torch.from_numpy(hits.astype(np.int64))
        job, per, ok = sdist.job_queue_hits(ranks, hits_t)
        t = sdist.max_over_ranks(float(rank + 1), ranks.dist)
        tot = sdist.sum_over_ranks(shard.hi - shard.lo, ranks.dist)
        q.put((rank, shard.lo, shard.hi, cs, h, qq, job, t, bytes(key_t.numpy()), tab_t.numpy().copy(),
               int(shard.lengths.sum()), ok, tot, (c2.lo, c2.hi, c2.job_packets), shard.seed,
               [p.copy() for p in per]))
    finally:
        sdist.finish(ranks)


def test_two_rank_sharding_matches_single_process():
    """The union of the ranks' C3 shards equals the single-process result;
    the job-wide queue_hits (all-reduce) equals the single-process histogram
    and the per-rank ones (all-gather); key/table broadcast, max over ranks."""
    from oracle import pyoracle as po

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # ONE single-process run over the whole job batch; each rank's results
    # must be exactly its slice of it, and the slices must tile the batch
    job = pktgen.imix_lengths(3000, np.random.default_rng(sdist.WORKLOADS["c3"]["seed"]))
    table = (np.arange(128) % 16).astype(np.uint16)
    frames, desc, _ = pktgen.make_batch(job, seed=JOB_SEED, proto=17)
    cs, h, qq, _, want_hits = po.rx_batch(frames, desc, MS_KEY, table)
    assert res[0][1] == 0 and res[0][2] == res[1][1] and res[1][2] == 3000
    for r in res:
        lo, hi = r[1], r[2]
        np.testing.assert_array_equal(r[3], cs[lo:hi])
        np.testing.assert_array_equal(r[4], h[lo:hi])
        np.testing.assert_array_equal(r[5], qq[lo:hi])
    assert np.array_equal(np.concatenate([r[4] for r in res]), h)
    for r in res:
        np.testing.assert_array_equal(r[6], want_hits)  # summed histogram on every rank
        assert r[11]  # all-reduce == sum of the all-gathered per-rank histograms
        assert int(r[6].sum()) == 3000 and r[12] == 3000
        assert r[7] == 2.0  # max over ranks
        assert r[8] == MS_KEY  # broadcast key
        np.testing.assert_array_equal(r[9].view(np.uint16), table)
    assert res[0][13] == (0, 64, 128) and res[1][13] == (64, 128, 128)  # C2: equal per-rank batches
    # byte balance: shards within two max-size packets of each other
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
