#!/usr/bin/env python3
"""Attribution of the f1 delivery (deliver_kernel) on a C3-shaped write list,
inputs resident in HBM: 1 M IMIX frames (64/576/1518 at 7:4:1) packed at
16-B aligned offsets (the TX buffers) delivered into 2-KiB RX slots, every
completion Success, RSS with the MS key and a 16-queue table — the writes
nic::BatchedQueuePair hands the kernel for bench_rx_stage c3.

Timed with HIP events per launch (median of --iters after warm-up), all in
one process, rounds interleaved:
  production       nicgpu_tune_deliver mode 0 (what nicgpu_qp_deliver launches)
  no_rss           the same writes without RSS (deliver_kernel<false>)
  mode N           tuning modes of deliver_kernel (f1.hip kDlv*; outputs wrong):
                   1 no stores, 2 no loads, 4 no hash, 8 packed destinations
                   (the frames written contiguously, as the source); 32 round 3's
                   kernel (deliver_v1_kernel), 32|1|4 and 32|2|4 its loads / stores alone
  gather           nicgpu_segment_gather (one wave per write) over the same list
  copy_packed      torch copy of the TX bytes to a packed destination (a plain
                   device copy of the same bytes: the copy ceiling)

  python tools/f1_deliver_bench.py [--n 1048576] [--iters 10] [--rounds 3]
Prints one JSON line.
"""

import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MS_KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")
WRITE_DT = np.dtype([("dst", "<u8"), ("src_a", "<u8"), ("src_b", "<u8"), ("len_a", "<u4"), ("len_b", "<u4"),
                     ("prefix", "<u4"), ("prefix_len", "<u4")])
COMPL_DT = np.dtype([("queue_id", "<u2"), ("descriptor_index", "<u2"), ("status", "<u4"), ("flags", "u1", 8),
                     ("segments", "<u2"), ("vlan", "<u2")])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--slot", type=int, default=2048)
    ap.add_argument("--modes", default="0,1,2,4,8,6,5,7,32")
    ap.add_argument("--frames", choices=["udp", "random"], default="udp",
                    help="udp: IPv4/UDP headers (pktgen); random: random bytes behind EtherType 0x0800, as "
                         "tools/bench_rx_stage.cpp builds them (IHL random: most tuples end past the 48-B stage)")
    ap.add_argument("--rx-base", choices=["page", "packed"], default="page",
                    help="page: RX slots from the next 4-KiB boundary after the TX bytes; packed: right after them "
                         "(16-B aligned only, as tools/bench_rx_stage.cpp lays them out)")
    ap.add_argument("--rx-shift", type=int, default=0, help="bytes added to the RX slot base (a multiple of 16)")
    ap.add_argument("--lib", default=os.path.join(ROOT, "smart_nic_amd", "libnicgpu_tune.so"),
                    help="tuning library to time (an A/B build of libnicgpu_tune.so)")
    ap.add_argument("--patterns", action="store_true",
                    help="also time bare 16-B store kernels writing 64/576/1518-B frames at 2-KiB strides and packed "
                         "(nicgpu_tune_store_pattern): the store shape's ceiling")
    args = ap.parse_args()

    import torch

    from smart_nic_amd import pktgen

    assert WRITE_DT.itemsize == 40 and COMPL_DT.itemsize == 20
    tl = ctypes.CDLL(args.lib)
    vp, sz, i32, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
    tl.nicgpu_tune_deliver.restype = i32
    tl.nicgpu_tune_deliver.argtypes = [i32, vp, u64, vp, vp, sz, vp, vp, vp, vp, vp, u64, vp]
    tl.nicgpu_segment_gather.restype = i32
    tl.nicgpu_segment_gather.argtypes = [vp, u64, vp, sz, vp]
    tl.nicgpu_rss_create.argtypes = [ctypes.POINTER(vp), i32]
    tl.nicgpu_rss_set_key.argtypes = [vp, vp, sz, vp]
    tl.nicgpu_rss_set_table.argtypes = [vp, vp, sz, vp]

    n = args.n
    rng = np.random.default_rng(33)
    lens = pktgen.imix_lengths(n, rng)
    frames, desc, _ = pktgen.make_batch(lens, seed=33, proto=17, corrupt_frac=0.0)
    off = (desc & np.uint64((1 << 40) - 1)).astype(np.uint64)
    if args.frames == "random":
        frames = rng.integers(0, 256, frames.size, dtype=np.uint8)
        frames[off.astype(np.int64) + 12] = 0x08
        frames[off.astype(np.int64) + 13] = 0x00
    tx_bytes = (int(frames.size) + 4095) // 4096 * 4096 if args.rx_base == "page" else (int(frames.size) + 15) // 16 * 16
    tx_bytes += args.rx_shift
    mem_size = tx_bytes + n * args.slot
    mem = torch.zeros(mem_size + 64, dtype=torch.uint8, device="cuda")
    mem[: frames.size].copy_(torch.from_numpy(frames))
    w = np.zeros(n, WRITE_DT)
    w["dst"] = tx_bytes + np.arange(n, dtype=np.uint64) * np.uint64(args.slot)
    w["src_a"] = off
    w["len_a"] = lens.astype(np.uint32)
    w_dev = torch.from_numpy(w.view(np.uint8)).cuda()
    rxc = np.zeros(n, COMPL_DT)  # status 0 = Success
    rxc_dev = torch.from_numpy(rxc.view(np.uint8)).cuda()
    ctx = vp()
    assert tl.nicgpu_rss_create(ctypes.byref(ctx), 0) == 0
    kb = (ctypes.c_uint8 * len(MS_KEY)).from_buffer_copy(MS_KEY)
    assert tl.nicgpu_rss_set_key(ctx, kb, len(MS_KEY), None) == 0
    tab = (np.arange(128) % 16).astype(np.uint16)
    assert tl.nicgpu_rss_set_table(ctx, tab.ctypes.data, tab.size, None) == 0
    h = torch.zeros(n, dtype=torch.int32, device="cuda")
    q = torch.zeros(n, dtype=torch.int16, device="cuda")
    hits = torch.zeros(128, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()
    sp = vp(stream.cuda_stream)
    packed_dst = torch.empty(frames.size, dtype=torch.uint8, device="cuda")
    src_view = mem[: frames.size]

    def deliver(mode, rss=True):
        def f():
            rc = tl.nicgpu_tune_deliver(mode, mem.data_ptr(), mem_size, w_dev.data_ptr(), rxc_dev.data_ptr(), n,
                                        ctx if rss else None, h.data_ptr(), q.data_ptr(), hits.data_ptr(),
                                        cnt.data_ptr(), tx_bytes, sp)
            assert rc == 0, rc
        return f

    def gather():
        assert tl.nicgpu_segment_gather(mem.data_ptr(), mem_size, w_dev.data_ptr(), n, sp) == 0

    cases = {"production": deliver(0), "no_rss": deliver(0, rss=False), "gather": gather,
             "copy_packed": lambda: packed_dst.copy_(src_view)}
    for m in [int(x) for x in args.modes.split(",") if x]:
        if m:
            cases[f"mode{m}"] = deliver(m)
    if args.patterns:
        tl.nicgpu_tune_store_pattern.restype = i32
        tl.nicgpu_tune_store_pattern.argtypes = [vp, u64, ctypes.c_uint32, ctypes.c_uint32, i32, i32, vp]
        rx_base = mem.data_ptr() + tx_bytes
        for flen in (64, 576, 1518):
            nf = int((lens == flen).sum())
            for slot, nt in ((args.slot, 0), (args.slot, 1), ((flen + 15) // 16 * 16, 0)):
                def pat(nf=nf, flen=flen, slot=slot, nt=nt):
                    assert tl.nicgpu_tune_store_pattern(rx_base, nf, flen, slot, 8, nt, sp) == 0
                cases[f"store_{flen}B_slot{slot}" + ("_nt" if nt else "")] = pat
    times = {k: [] for k in cases}
    for _ in range(args.rounds):
        for name, fn in cases.items():
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.iters + 1)]
            ev[0].record()
            for i in range(args.iters):
                fn()
                ev[i + 1].record()
            torch.cuda.synchronize()
            times[name] += [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(args.iters)]
    # check the production delivery wrote the frames
    deliver(0)()
    torch.cuda.synchronize()
    k = min(n, 4096)
    got = mem[tx_bytes: tx_bytes + k * args.slot].view(k, args.slot).cpu().numpy()
    ok = all(np.array_equal(got[i, : lens[i]], frames[int(off[i]): int(off[i]) + lens[i]]) for i in range(k))
    moved = 2 * int(lens.sum())
    out = {"lib": os.path.basename(args.lib), "frames": args.frames, "rx_base": args.rx_base, "rx_base_mod128": tx_bytes % 128,
           "n": n, "slot": args.slot, "frame_bytes": int(lens.sum()), "moved_bytes": moved, "delivered_ok": bool(ok),
           "success_count": int(cnt.item()), "us_median": {}, "tbps_rw": {}}
    for name, ts in times.items():
        med = float(np.median(ts))
        out["us_median"][name] = round(med, 1)
        if name.startswith("store_"):
            flen = int(name.split("_")[1][:-1])
            out["tbps_rw"][name] = round(int((lens == flen).sum()) * ((flen + 15) // 16 * 16) / med / 1e6, 3)
        else:
            out["tbps_rw"][name] = round(moved / med / 1e6, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
