#!/usr/bin/env python3
"""A/B every RX kernel variant of libnicgpu_tune.so in ONE process, interleaved
rounds (cdna_hip_programming.md §5.4 rule 24), on the bench workloads, plus the
read-only streaming ceiling of this box.  Tuning infrastructure only.

Prints a JSON summary (median per-launch µs, GB/s of algorithmic bytes, % of
the 8 TB/s spec peak and of the measured read ceiling) and checks every variant
bit-exactly against variant 0.
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MS_KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--workloads", default="c2,imix,u64")
    ap.add_argument("--variants", default="all")
    ap.add_argument("--modes", default="auto,none", help="timed tuple modes: auto (checksum+RSS), none (checksum only)")
    ap.add_argument("--no-ceiling", action="store_true", help="skip the read-ceiling sweeps (PMC runs)")
    ap.add_argument("--xpf", type=int, default=-1, help="XPF variants: prefetch tiles of at most this many chunks")
    ap.add_argument("--bpcs", default="0", help="comma list of RX blocks-per-CU caps to A/B per variant "
                    "(nicgpu_tune_set_bpc; 0 = occupancy maximum)")
    args = ap.parse_args()

    import torch

    import smart_nic_amd as sna
    from smart_nic_amd import pktgen

    tl = ctypes.CDLL(os.path.join(ROOT, "smart_nic_amd", "libnicgpu_tune.so"))
    vp, sz, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int
    tl.nicgpu_tune_num_variants.restype = i32
    tl.nicgpu_tune_variant_name.restype = ctypes.c_char_p
    tl.nicgpu_tune_variant_name.argtypes = [i32]
    tl.nicgpu_tune_rx_offload.restype = i32
    tl.nicgpu_tune_rx_offload.argtypes = [i32, vp, vp, vp, sz, i32, u32, u32, vp, vp, vp, vp, vp]
    tl.nicgpu_tune_stream_read.restype = i32
    tl.nicgpu_tune_stream_read.argtypes = [vp, sz, i32, i32, vp, vp]
    if args.xpf >= 0:
        tl.nicgpu_tune_set_xpf.argtypes = [u32]
        tl.nicgpu_tune_set_xpf(args.xpf)
    nv = tl.nicgpu_tune_num_variants()
    base_names = [tl.nicgpu_tune_variant_name(i).decode() for i in range(nv)]
    base_variants = list(range(nv)) if args.variants == "all" else [int(x) for x in args.variants.split(",")]
    bpcs = [int(x) for x in args.bpcs.split(",")]
    tl.nicgpu_tune_set_bpc.argtypes = [u32]
    # (variant, blocks-per-CU cap) combinations, named variant[_bpcN]
    combos = [(v, b) for v in base_variants for b in bpcs]
    variants = list(range(len(combos)))
    names = [base_names[v] + (f"_bpc{b}" if b else "") for v, b in combos]

    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    # contexts must come from the tuning library (its own nicgpu_rss_ctx)
    h = ctypes.c_void_p()
    tl.nicgpu_rss_create.argtypes = [ctypes.POINTER(vp), i32]
    tl.nicgpu_rss_set_key.argtypes = [vp, vp, sz, vp]
    tl.nicgpu_rss_set_table.argtypes = [vp, vp, sz, vp]
    assert tl.nicgpu_rss_create(ctypes.byref(h), 0) == 0
    key = (ctypes.c_uint8 * 40).from_buffer_copy(MS_KEY)

    out = {"variants": names, "workloads": {}}
    rng = np.random.default_rng(0)
    wls = []
    for w in args.workloads.split(","):
        if w == "c2":
            wls.append(("c2_1518", np.full(1 << 20, 1518), 4, 6))
        elif w == "imix":
            wls.append(("c3_imix_16q", pktgen.imix_lengths(4 << 20, rng), 16, 17))
        elif w == "u64":
            wls.append(("u64", np.full(4 << 20, 64), 4, 17))
        elif w == "jumbo":
            wls.append(("jumbo_9000", np.full(160_000, 9000), 4, 6))

    ceiling_buf = None
    for name, lens, nq, proto in wls:
        t0 = time.time()
        frames, desc, _ = pktgen.make_batch(lens, seed=7, proto=proto, corrupt_frac=0.01)
        print(f"# {name}: generated {desc.size} pkts in {time.time()-t0:.1f}s", file=sys.stderr, flush=True)
        n = desc.size
        table = (np.arange(128) % nq).astype(np.uint16)
        assert tl.nicgpu_rss_set_key(h, key, 40, sp) == 0
        assert tl.nicgpu_rss_set_table(h, table.ctypes.data, 128, sp) == 0
        f = torch.from_numpy(frames).cuda()
        d = torch.from_numpy(desc.view(np.int64)).cuda()
        if ceiling_buf is None or f.numel() > ceiling_buf.numel():
            ceiling_buf = f
        cs = torch.empty(n, dtype=torch.int16, device="cuda")
        hs = torch.empty(n, dtype=torch.int32, device="cuda")
        qs = torch.empty(n, dtype=torch.int16, device="cuda")
        hits = torch.zeros(128, dtype=torch.int64, device="cuda")
        alg = int(lens.sum()) + 16 * n

        def run(c, mode=sna.TUPLE_AUTO):
            v, b = combos[c]
            tl.nicgpu_tune_set_bpc(b)
            st = tl.nicgpu_tune_rx_offload(v, h, f.data_ptr(), d.data_ptr(), n, mode, 0, 0, cs.data_ptr(),
                                           hs.data_ptr() if mode else None, qs.data_ptr() if mode else None,
                                           hits.data_ptr() if mode else None, sp)
            assert st == 0, st

        # correctness vs variant 0 at full occupancy
        tl.nicgpu_tune_set_bpc(0)
        assert tl.nicgpu_tune_rx_offload(0, h, f.data_ptr(), d.data_ptr(), n, sna.TUPLE_AUTO, 0, 0, cs.data_ptr(),
                                         hs.data_ptr(), qs.data_ptr(), hits.data_ptr(), sp) == 0
        torch.cuda.synchronize()
        ref = (cs.clone(), hs.clone(), qs.clone())
        for v in variants:
            run(v)
            torch.cuda.synchronize()
            assert torch.equal(cs, ref[0]) and torch.equal(hs, ref[1]) and torch.equal(qs, ref[2]), names[v]
        times = {v: [] for v in variants}
        times_csum = {v: [] for v in variants}
        for r in range(args.rounds):
            for v in variants:
                for mode, bucket in ((sna.TUPLE_AUTO, times), (sna.TUPLE_NONE, times_csum)):
                    if (mode == sna.TUPLE_AUTO and "auto" not in args.modes) or (
                            mode == sna.TUPLE_NONE and "none" not in args.modes):
                        continue
                    run(v, mode)
                    e = [torch.cuda.Event(enable_timing=True) for _ in range(args.iters + 1)]
                    e[0].record()
                    for i in range(args.iters):
                        run(v, mode)
                        e[i + 1].record()
                    torch.cuda.synchronize()
                    bucket[v] += [e[i].elapsed_time(e[i + 1]) * 1e3 for i in range(args.iters)]
        res = {}
        for v in variants:
            med = float(np.median(times[v])) if times[v] else float("nan")
            medc = float(np.median(times_csum[v])) if times_csum[v] else float("nan")
            res[names[v]] = {
                "us_median": round(med, 2), "us_min": round(float(np.min(times[v])), 2) if times[v] else None,
                "alg_gbs": round(alg / med / 1e3, 1), "frac_spec": round(alg / med / 1e3 / 8000, 4),
                "csum_only_us": round(medc, 2), "csum_only_gbs": round((int(lens.sum()) + 10 * n) / medc / 1e3, 1),
                "mpkts": round(n / med, 1),
            }
        out["workloads"][name] = {"packets": n, "alg_bytes": alg, "results": res}
        print(json.dumps({name: res}), file=sys.stderr, flush=True)
        del f, d

    # C5: 9000 B frames through TSO segmentation (H = 54, mss = 1448 -> 7 segments)
    if "tso" in args.workloads.split(","):
        import smart_nic_amd as sna_p

        nf = 131072
        frames, desc, _ = pktgen.make_batch(np.full(nf, 9000), seed=9, proto=6, corrupt_frac=0.0)
        nseg = (9000 - 54 + 1447) // 1448
        f = torch.from_numpy(frames).cuda()
        d = torch.from_numpy(desc.view(np.int64)).cuda()
        hdr = torch.full((nf,), 54, dtype=torch.int16, device="cuda")
        mss = torch.full((nf,), 1448, dtype=torch.int16, device="cuda")
        base = torch.arange(nf, dtype=torch.int32, device="cuda") * nseg
        out_t = torch.empty(nf * nseg, dtype=torch.int16, device="cuda")
        plib = sna_p.load_library()
        ts = []
        for r in range(args.rounds * args.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert plib.nicgpu_tso_checksum(f.data_ptr(), d.data_ptr(), hdr.data_ptr(), mss.data_ptr(),
                                            base.data_ptr(), nf, out_t.data_ptr(), sp) == 0
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        med = float(np.median(ts))
        alg = nf * (9000 + 16) + nf * nseg * 2
        out["workloads"]["c5_tso_9000"] = {"packets": nf, "segments": nf * nseg, "alg_bytes": alg, "results": {
            "tso_checksum_kernel": {"us_median": round(med, 2), "alg_gbs": round(alg / med / 1e3, 1),
                                    "frac_spec": round(alg / med / 1e3 / 8000, 4),
                                    "msegs_per_s": round(nf * nseg / med, 1)}}}
        print(json.dumps({"c5_tso_9000": out["workloads"]["c5_tso_9000"]}), file=sys.stderr, flush=True)
        del f, d

    # read-only streaming ceiling on the largest buffer
    if ceiling_buf is not None and not args.no_ceiling:
        nbytes = ceiling_buf.numel() // 16 * 16
        sink = torch.zeros(1, dtype=torch.int32, device="cuda")
        ceil = {}
        for unroll in (1, 2, 4, 8):
            for bpc in (2, 4, 8):
                ts = []
                for _ in range(args.rounds * 2):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    assert tl.nicgpu_tune_stream_read(ceiling_buf.data_ptr(), nbytes, bpc, unroll, sink.data_ptr(), sp) == 0
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3)
                med = float(np.median(ts))
                ceil[f"u{unroll}_bpc{bpc}"] = round(nbytes / med / 1e3, 1)
        tl.nicgpu_tune_stream_tiles.restype = i32
        tl.nicgpu_tune_stream_tiles.argtypes = [vp, sz, sz, i32, i32, vp, vp]
        tiles = {}
        for tile_kb in (24, 96):
            for unroll in (1, 2, 4):
                for bpc in (4, 5, 8):
                    ts = []
                    for _ in range(args.rounds):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        assert tl.nicgpu_tune_stream_tiles(ceiling_buf.data_ptr(), nbytes, tile_kb * 1024, bpc, unroll,
                                                           sink.data_ptr(), sp) == 0
                        e1.record()
                        torch.cuda.synchronize()
                        ts.append(e0.elapsed_time(e1) * 1e3)
                    med = float(np.median(ts))
                    used = nbytes // (tile_kb * 1024) * (tile_kb * 1024)
                    tiles[f"t{tile_kb}k_u{unroll}_bpc{bpc}"] = round(used / med / 1e3, 1)
        out["tile_stream_gbs"] = tiles
        tl.nicgpu_tune_stream_btiles.restype = i32
        tl.nicgpu_tune_stream_btiles.argtypes = [vp, sz, sz, i32, i32, vp, vp]
        btiles = {}
        for tile_kb in (96, 384, 1536):
            for unroll in (1, 2, 4):
                for bpc in (2, 4, 5, 8):
                    ts = []
                    for _ in range(args.rounds):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        assert tl.nicgpu_tune_stream_btiles(ceiling_buf.data_ptr(), nbytes, tile_kb * 1024, bpc, unroll,
                                                            sink.data_ptr(), sp) == 0
                        e1.record()
                        torch.cuda.synchronize()
                        ts.append(e0.elapsed_time(e1) * 1e3)
                    med = float(np.median(ts))
                    used = nbytes // (tile_kb * 1024) * (tile_kb * 1024)
                    btiles[f"bt{tile_kb}k_u{unroll}_bpc{bpc}"] = round(used / med / 1e3, 1)
        out["block_tile_stream_gbs"] = btiles
        out["read_ceiling_gbs"] = ceil
        best = max(ceil.values())
        out["read_ceiling_best_gbs"] = best
        for wl in out["workloads"].values():
            for r in wl["results"].values():
                r["frac_ceiling"] = round(r["alg_gbs"] / best, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
