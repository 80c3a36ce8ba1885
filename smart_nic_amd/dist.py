"""Multi-GPU plumbing for the RX offload path (one process per GPU).

The path shards trivially: every packet's checksum and hash
depend only on its own bytes and the read-only key/table.  So:
  * packets are split into contiguous per-rank ranges — for IMIX balanced by
    BYTES (its packets differ 24x in size) — with no data-path collective;
  * once at setup, rank 0's RSS key and indirection table are broadcast
    (RCCL over xGMI with backend "nccl"; gloo on CPU for tests);
  * once per batch, the per-table-index hit histograms are summed so every
    rank holds the job-wide RssStats.queue_hits (rss.cpp:54-58 counts per
    table index), and checked against the per-rank histograms;
  * timing takes the max over ranks.

bench.py's rank setup lives here (init_ranks, plan_shard, setup_rss,
job_queue_hits, max_over_ranks, finish), so tests/test_dist_gloo.py runs the
same code at world size 2 on CPU, with the oracle in place of the kernel.
"""

from __future__ import annotations

import dataclasses
import os

import numpy as np

# BASELINE.json configs: C2 = 1 M x 1518 B TCP per GPU (4 queues), C3 = IMIX
# 64/576/1518 at 7:4:1 (16 queues); SURVEY §8(d)
WORKLOADS = {
    "c2": {"packets_per_gpu": 1 << 20, "queues": 4, "proto": 6, "seed": 42},
    "c3": {"packets_per_gpu": 1 << 22, "queues": 16, "proto": 17, "seed": 33},
}


def shard_by_bytes(lengths: np.ndarray, world: int) -> np.ndarray:
    """Contiguous packet ranges [bounds[r], bounds[r+1]) with ~equal bytes.

    Every rank gets at least one packet when len(lengths) >= world."""
    lengths = np.asarray(lengths, dtype=np.int64)
    n = lengths.size
    if world <= 1:
        return np.array([0, n], dtype=np.int64)
    if n == 0:
        return np.zeros(world + 1, dtype=np.int64)
    csum = np.cumsum(np.maximum(lengths, 1))
    total = int(csum[-1])
    targets = (np.arange(1, world) * total) // world
    cuts = np.searchsorted(csum, targets, side="left") + 1
    bounds = np.concatenate([[0], cuts, [n]]).astype(np.int64)
    bounds = np.maximum.accumulate(np.minimum(bounds, n))
    if n >= world:  # no empty shard
        for r in range(1, world):
            bounds[r] = min(max(bounds[r], bounds[r - 1] + 1), n - (world - r))
    return bounds


@dataclasses.dataclass
class Ranks:
    """This process's place in the job.  `dist` is torch.distributed when a
    process group is up (world > 1, or forced), else None."""
    rank: int = 0
    world: int = 1
    local: int = 0
    dist: object = None
    device: object = None  # torch.device the rank's tensors live on


def init_ranks(force: bool = False, backend: str = "nccl") -> Ranks:
    """One process per GPU, as torch.distributed.run launches it (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* in the environment).  With backend
    "nccl" (RCCL) the rank's GPU is LOCAL_RANK; with "gloo" (CPU tests) the
    device is the CPU.  At world size 1 no group is created unless `force`
    (bench.py --dist: the RCCL path on a one-GPU box)."""
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = backend == "nccl"
    if gpu:
        torch.cuda.set_device(local if (world > 1 or force) else 0)
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    d = None
    if world > 1 or force:
        import torch.distributed as d

        if gpu:
            d.init_process_group("nccl", device_id=device)
        else:
            d.init_process_group("gloo", rank=rank, world_size=world)
    return Ranks(rank=rank, world=world, local=local, dist=d, device=device)


@dataclasses.dataclass
class Shard:
    """The packets this rank owns: lengths[lo:hi] of the job's batch."""
    workload: str
    lengths: np.ndarray  # this rank's packet lengths
    lo: int
    hi: int
    job_packets: int
    job_bytes: int
    seed: int  # frame-content seed of this rank's batch
    queues: int
    proto: int


def plan_shard(workload: str, ranks: Ranks, packets_per_gpu: int | None = None) -> Shard:
    """C2: every rank owns its own packets_per_gpu x 1518 B batch (weak
    scaling, equal sizes).  C3: the job's IMIX batch is world x
    packets_per_gpu packets whose lengths come from one seed on every rank;
    each rank takes its byte-balanced contiguous range (shard_by_bytes), so
    per-GPU work stays fixed as the world grows."""
    w = WORKLOADS[workload]
    n = int(packets_per_gpu or w["packets_per_gpu"])
    if workload == "c2":
        lens = np.full(n, 1518, dtype=np.int64)
        return Shard(workload, lens, ranks.rank * n, (ranks.rank + 1) * n, n * ranks.world, n * ranks.world * 1518,
                     w["seed"] + ranks.rank, w["queues"], w["proto"])
    from smart_nic_amd import pktgen

    job = pktgen.imix_lengths(n * ranks.world, np.random.default_rng(w["seed"]))
    bounds = shard_by_bytes(job, ranks.world)
    lo, hi = int(bounds[ranks.rank]), int(bounds[ranks.rank + 1])
    return Shard(workload, job[lo:hi].copy(), lo, hi, int(job.size), int(job.sum()), w["seed"] + ranks.rank,
                 w["queues"], w["proto"])


def broadcast_rss_config(key, table, dist, src: int = 0):
    """Broadcast the RSS key (uint8 tensor) and indirection table (int32
    tensor holding the uint16 queue ids — RCCL/NCCL and gloo have no 16-bit
    integer type) in place from `src`; sizes must agree on every rank.
    Returns (key, table as int16 ready for nicgpu_rss_set_table_device)."""
    dist.broadcast(key, src=src)
    dist.broadcast(table, src=src)
    import torch

    return key, table.to(torch.int16)


def setup_rss(ranks: Ranks, key: bytes, table: np.ndarray):
    """Rank 0's key and table on every rank (RCCL broadcast at world > 1;
    the other ranks start from zeros so a failed broadcast shows).  Returns
    (key uint8 tensor, table int16 tensor) on the rank's device."""
    import torch

    key_t = torch.tensor(list(key), dtype=torch.uint8, device=ranks.device)
    tab_t = torch.from_numpy(np.asarray(table, dtype=np.int32)).to(ranks.device)
    if ranks.dist is None:
        return key_t, tab_t.to(torch.int16)
    if ranks.rank != 0:
        key_t.zero_()
        tab_t.zero_()
    return broadcast_rss_config(key_t, tab_t, ranks.dist)


def sum_hits(hits, dist):
    """Sum per-rank queue-hit histograms (int64 tensors) in place."""
    dist.all_reduce(hits, op=dist.ReduceOp.SUM)
    return hits


def job_queue_hits(ranks: Ranks, hits):
    """The job-wide RssStats.queue_hits from this rank's histogram (int64
    tensor): an all-reduce sum, checked against an all-gather of the per-rank
    histograms summed on the host.  Returns (job hits as np.uint64, per-rank
    hits as a list of np.uint64 arrays, check ok)."""
    local = hits.detach().cpu().numpy().astype(np.uint64)
    if ranks.dist is None:
        return local, [local], True
    import torch

    d = ranks.dist
    job = hits.clone()
    sum_hits(job, d)
    parts = [torch.empty_like(hits) for _ in range(ranks.world)]
    d.all_gather(parts, hits)
    per = [p.cpu().numpy().astype(np.uint64) for p in parts]
    job_np = job.cpu().numpy().astype(np.uint64)
    ok = bool(np.array_equal(job_np, np.sum(per, axis=0, dtype=np.uint64))
              and np.array_equal(per[ranks.rank], local))
    return job_np, per, ok


def max_over_ranks(value: float, dist, device=None) -> float:
    import torch

    if dist is None:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_over_ranks(values, dist, device=None) -> list:
    """Every rank's list of floats (same length on every rank), in rank order."""
    import torch

    if dist is None:
        return [[float(v) for v in values]]
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [p.cpu().tolist() for p in parts]


def sum_over_ranks(value: int, dist, device=None) -> int:
    import torch

    if dist is None:
        return int(value)
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def barrier(ranks: Ranks):
    if ranks.dist is not None:
        ranks.dist.barrier()


def finish(ranks: Ranks):
    if ranks.dist is not None:
        ranks.dist.barrier()
        ranks.dist.destroy_process_group()
