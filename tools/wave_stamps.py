#!/usr/bin/env python3
"""Per-wave start/end timestamps of one RX launch (libnicgpu_tune.so,
nicgpu_tune_set_stamps): how long the grid's tail is, and whether it is one
XCD or a spread of waves.  Tuning infrastructure only.

  python tools/wave_stamps.py --workloads c2,imix --variant 0

Prints one JSON object per workload: the launch span (first wave start to last
wave end, us), start / end quantiles relative to the first start, per-XCD
median and max end, and how much of the span the last 10 % of waves take.
s_memrealtime runs at 100 MHz (10 ns ticks).
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MS_KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")
TICK_US = 0.01


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c2,imix")
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--stream", action="store_true", help="stamp the read-ceiling kernel instead of the RX kernel")
    ap.add_argument("--bpc", type=int, default=0, help="RX blocks-per-CU cap (nicgpu_tune_set_bpc; 0 = occupancy maximum)")
    args = ap.parse_args()

    import torch

    import smart_nic_amd as sna
    from smart_nic_amd import pktgen

    tl = ctypes.CDLL(os.path.join(ROOT, "smart_nic_amd", "libnicgpu_tune.so"))
    vp, sz, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int
    tl.nicgpu_tune_rx_offload.restype = i32
    tl.nicgpu_tune_rx_offload.argtypes = [i32, vp, vp, vp, sz, i32, u32, u32, vp, vp, vp, vp, vp]
    tl.nicgpu_tune_set_stamps.argtypes = [vp]
    tl.nicgpu_tune_stream_read.restype = i32
    tl.nicgpu_tune_stream_read.argtypes = [vp, sz, i32, i32, vp, vp]
    tl.nicgpu_tune_set_bpc.argtypes = [u32]
    tl.nicgpu_tune_set_bpc(args.bpc)
    tl.nicgpu_tune_variant_name.restype = ctypes.c_char_p
    tl.nicgpu_tune_variant_name.argtypes = [i32]
    tl.nicgpu_rss_create.argtypes = [ctypes.POINTER(vp), i32]
    tl.nicgpu_rss_set_key.argtypes = [vp, vp, sz, vp]
    tl.nicgpu_rss_set_table.argtypes = [vp, vp, sz, vp]
    torch.cuda.set_device(0)
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    h = ctypes.c_void_p()
    assert tl.nicgpu_rss_create(ctypes.byref(h), 0) == 0
    key = (ctypes.c_uint8 * 40).from_buffer_copy(MS_KEY)
    max_waves = 256 * 64
    stamps = torch.zeros(max_waves * 4, dtype=torch.int64, device="cuda")
    rng = np.random.default_rng(0)
    for w in args.workloads.split(","):
        if w == "c2":
            lens, nq, proto = np.full(1 << 20, 1518), 4, 6
        elif w == "imix":
            lens, nq, proto = pktgen.imix_lengths(4 << 20, rng), 16, 17
        elif w == "u64":
            lens, nq, proto = np.full(4 << 20, 64), 4, 17
        else:
            lens, nq, proto = np.full(160_000, 9000), 4, 6
        frames, desc, _ = pktgen.make_batch(lens, seed=7, proto=proto, corrupt_frac=0.01)
        n = desc.size
        table = (np.arange(128) % nq).astype(np.uint16)
        assert tl.nicgpu_rss_set_key(h, key, 40, sp) == 0
        assert tl.nicgpu_rss_set_table(h, table.ctypes.data, 128, sp) == 0
        f = torch.from_numpy(frames).cuda()
        d = torch.from_numpy(desc.view(np.int64)).cuda()
        cs = torch.empty(n, dtype=torch.int16, device="cuda")
        hs = torch.empty(n, dtype=torch.int32, device="cuda")
        qs = torch.empty(n, dtype=torch.int16, device="cuda")
        hits = torch.zeros(128, dtype=torch.int64, device="cuda")

        sink = torch.zeros(1, dtype=torch.int32, device="cuda")

        def run():
            if args.stream:  # the same-box read ceiling's kernel (unroll 4, 2 blocks per CU) over the frames
                assert tl.nicgpu_tune_stream_read(f.data_ptr(), f.numel() // 16 * 16, 2, 4, sink.data_ptr(), sp) == 0
                return
            assert tl.nicgpu_tune_rx_offload(args.variant, h, f.data_ptr(), d.data_ptr(), n, sna.TUPLE_AUTO, 0, 0,
                                             cs.data_ptr(), hs.data_ptr(), qs.data_ptr(), hits.data_ptr(), sp) == 0

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        spans, rows = [], []
        for _ in range(args.launches):
            stamps.zero_()
            tl.nicgpu_tune_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
            tl.nicgpu_tune_set_stamps(None)
            s = stamps.view(-1, 4).cpu().numpy()
            s = s[s[:, 0] != 0]
            t0 = s[:, 0].min()
            start = (s[:, 0] - t0) * TICK_US
            end = (s[:, 1] - t0) * TICK_US
            xcc = s[:, 2] & 15
            span = float(end.max())
            spans.append(span)
            per_xcd = {int(x): {"end_med": round(float(np.median(end[xcc == x])), 1),
                                "end_max": round(float(end[xcc == x].max()), 1), "waves": int((xcc == x).sum())}
                       for x in sorted(set(xcc.tolist()))}
            q = lambda a, p: round(float(np.quantile(a, p)), 1)
            rows.append({
                "event_us": round(e0.elapsed_time(e1) * 1e3, 1), "span_us": round(span, 1), "waves": int(len(s)),
                "start_q": [q(start, p) for p in (0, 0.5, 0.9, 1)],
                "end_q": [q(end, p) for p in (0, 0.1, 0.5, 0.9, 1)],
                "tail_last10pct_us": round(span - q(end, 0.9), 1), "per_xcd": per_xcd,
            })
        best = int(np.argmin(spans))
        out = {"workload": w, "kernel": "stream_read<4>" if args.stream else "rx", "bpc": args.bpc, "variant": tl.nicgpu_tune_variant_name(args.variant).decode(), "packets": int(n),
               "bytes": int(lens.sum()), "spans_us": [round(x, 1) for x in spans], "best": rows[best]}
        print(json.dumps(out), flush=True)
        del f, d


if __name__ == "__main__":
    main()
