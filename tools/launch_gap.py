"""Launch-gap experiment for bench.py's timed loop (C2, production RX kernel).

Times K back-to-back nicgpu_rx_offload launches three ways on one stream:
  events   per-launch HIP event pairs (bench.py's current loop)
  plain    no events between launches, one event pair around the K launches
  graph    the K launches captured once in a HIP graph, replayed
and prints one JSON line with the wall time per launch and the event time
per launch of each. Output only; nothing here is used by bench.py.
"""

from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import smart_nic_amd as sna  # noqa: E402
from smart_nic_amd import pktgen  # noqa: E402

MS_KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")


def main():
    k = int(os.environ.get("K", "50"))
    rounds = int(os.environ.get("ROUNDS", "5"))
    n = 1 << 20
    torch.cuda.set_device(0)
    frames, desc, _ = pktgen.make_batch(np.full(n, 1518), seed=42, proto=6, corrupt_frac=0.01)
    f = torch.from_numpy(frames).cuda()
    d = torch.from_numpy(desc.view(np.int64)).cuda()
    cs = torch.empty(n, dtype=torch.int16, device="cuda")
    hs = torch.empty(n, dtype=torch.int32, device="cuda")
    qs = torch.empty(n, dtype=torch.int16, device="cuda")
    hits = torch.zeros(128, dtype=torch.int64, device="cuda")
    ctx = sna.RssContext(0)
    ctx.set_key(MS_KEY)
    ctx.set_table(np.arange(128) % 4)

    s = torch.cuda.Stream()

    def step():
        sna.rx_offload(ctx, f, d, sna.TUPLE_AUTO, 0, 0, cs, hs, qs, hits)

    with torch.cuda.stream(s):
        for _ in range(5):
            step()
    torch.cuda.synchronize()

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(k):
            step()
    torch.cuda.synchronize()

    res = {"events": [], "plain": [], "graph": []}
    for _ in range(rounds):
        with torch.cuda.stream(s):
            # events
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(k):
                ev[i][0].record(s)
                step()
                ev[i][1].record(s)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / k
            res["events"].append((wall * 1e6, float(np.mean([a.elapsed_time(b) for a, b in ev])) * 1e3))
            # plain
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a.record(s)
            for i in range(k):
                step()
            b.record(s)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / k
            res["plain"].append((wall * 1e6, a.elapsed_time(b) * 1e3 / k))
            # graph
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a.record(s)
            g.replay()
            b.record(s)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / k
            res["graph"].append((wall * 1e6, a.elapsed_time(b) * 1e3 / k))
    out = {m: {"wall_us_per_launch_median": round(float(np.median([x[0] for x in v])), 2),
               "event_us_per_launch_median": round(float(np.median([x[1] for x in v])), 2),
               "rounds": [[round(x[0], 2), round(x[1], 2)] for x in v]} for m, v in res.items()}
    out["k"] = k
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
