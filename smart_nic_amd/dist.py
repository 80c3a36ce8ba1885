"""Multi-GPU plumbing for the RX offload path (one process per GPU).

The path shards trivially: every packet's checksum and hash
depend only on its own bytes and the read-only key/table.  So:
  * packets are split into contiguous per-rank ranges balanced by BYTES
    (IMIX packets differ 24x in size), no data-path collective;
  * once at setup, rank 0's RSS key and indirection table are broadcast
    (RCCL over xGMI with backend "nccl"; gloo on CPU for tests);
  * optionally, once per batch, the per-table-index hit histograms are summed
    so rank 0 can rebuild RssStats.queue_hits for the whole job;
  * timing takes the max over ranks.
"""

from __future__ import annotations

import numpy as np


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


def broadcast_rss_config(key, table, dist, src: int = 0):
    """Broadcast the RSS key (uint8 tensor) and indirection table (int32
    tensor holding the uint16 queue ids — RCCL/NCCL and gloo have no 16-bit
    integer type) in place from `src`; sizes must agree on every rank.
    Returns (key, table as int16 ready for nicgpu_rss_set_table_device)."""
    dist.broadcast(key, src=src)
    dist.broadcast(table, src=src)
    import torch

    return key, table.to(torch.int16)


def sum_hits(hits, dist):
    """Sum per-rank queue-hit histograms (int64 tensors) in place."""
    dist.all_reduce(hits, op=dist.ReduceOp.SUM)
    return hits


def max_over_ranks(value: float, dist, device=None) -> float:
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
